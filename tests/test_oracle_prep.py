"""exp.py's data preparation (exp.py:60-99) and the Dirichlet partitioner (utils.py:314-349)
pinned to the reference's OWN output (tests/golden/prep_*.npz, written by make_golden.py
through /root/reference/functions/utils.py's load_full_data / get_Dirichlet_distribution).

CPU only: the oracle's restatement (oracle.exp_prepare, oracle.dirichlet_partition) and the
product's host-side partitioner (functions/utils.get_Dirichlet_distribution) against those
fixtures.  Tolerances: indices, labels, splits and RNG states exact; features 1e-5 absolute
(numpy's float32 cos vs torch's; |phi| <= 1/sqrt(D)); heterogeneity 1e-4 relative (a
difference of near-equal fp32 Gram matrices; the reference reduces in torch's order)."""
import os

import numpy as np
import pytest
import torch

from oracle import fedsim_oracle as O
from tests.fixtures import load


def _split(flat, lens):
    off = np.concatenate([[0], np.cumsum(lens)])
    return [flat[off[i]:off[i + 1]] for i in range(len(lens))]


@pytest.mark.parametrize('name', ['a9a', 'covtype'])
def test_dirichlet_partition_matches_reference(name):
    import fedamw_amd  # noqa: F401
    from fedamw_amd.functions import utils
    d = load('prep_dirichlet_' + name)
    labels = d['labels'].astype(np.float64)
    nc = int(d['n_clients'])
    ref = [list(p) for p in _split(d['parts'], d['part_len'])]
    np.random.seed(100)
    parts, _ = utils.get_Dirichlet_distribution(labels, [1.0 / nc] * nc, float(d['alpha']), verbose=False)
    assert [list(p) for p in parts] == ref
    np.testing.assert_array_equal(np.random.randint(0, 1 << 30, 4), d['after_np'])    # same numpy stream used
    np.random.seed(100)
    assert [list(p) for p in O.dirichlet_partition(labels, nc, float(d['alpha']))] == ref


def test_exp_prepare_matches_reference():
    d = load('prep_a9a')
    import fedamw_amd  # noqa: F401
    from fedamw_amd.functions import utils
    y = utils.svmlight_labels(d['y'], 'a9a')            # utils.py:39-45 as the reference applies it
    yt = utils.svmlight_labels(d['y_test'], 'a9a')
    N, D = int(d['n_clients']), int(d['D'])
    torch.manual_seed(100)
    np.random.seed(100)
    r = O.exp_prepare(d['X'], y, d['X_test'], yt, N, float(d['alpha']), float(d['k_par']), D)
    np.testing.assert_array_equal(torch.empty(4, dtype=torch.int64).random_().numpy(), d['after_torch'])
    np.testing.assert_array_equal(np.random.randint(0, 1 << 30, 4), d['after_np'])
    parts = _split(d['parts'], d['part_len'])
    assert [list(p) for p in r['parts']] == [list(p) for p in parts]
    # per-client rows: the partition addresses the shuffled full batch
    order = d['order']
    vi, ti = _split(d['val_idx'], d['split_len']), _split(d['train_idx'], d['part_len'] - d['split_len'])
    yv = np.concatenate([d['y_all'][p][v] for p, v in zip(parts, vi)]).astype(np.int64)
    np.testing.assert_array_equal(r['y_val'], yv)
    for j, p in enumerate(parts):
        np.testing.assert_array_equal(r['y_train'][j], d['y_all'][p][ti[j]])
        np.testing.assert_array_equal(d['y_all'][p], y[order][p])
    # features: the head of every client's (pre-split) block and of the test map, block sums
    for j in range(N):
        assert np.abs(r['X_clients'][j][:4] - d['phi_head'][j]).max() <= 1e-5, j
        assert abs(float(r['X_clients'][j].astype(np.float64).sum()) - d['phi_sum'][j]) <= 1e-5 * r['X_clients'][j].size
    assert abs(r['hete'] - float(d['hete'])) <= 1e-4 * abs(float(d['hete']))
    assert np.abs(r['X_test'][:16] - d['phi_test_head']).max() <= 1e-5


def test_oracle_exp_sequence_matches_reference():
    """exp.py's whole sequence on one un-reseeded stream (exp_satimage.npz): the oracle's
    restatement of exp.py:60-99 and its six algorithms called in exp.py's order, against
    every value the reference returned, the heterogeneity and both generators' end state."""
    import json
    from tests.fixtures import GOLDEN, LOSS_RTOL
    d = load('exp_satimage')
    P = json.load(open(os.path.join(GOLDEN, 'params.json')))[str(d['dataset'])]
    y, yt = d['y'] - d['y'].min(), d['y_test'] - d['y'].min()         # utils.py:43-44 (> 2 classes)
    D, N, R, le, B = int(d['D']), int(d['N']), int(d['Round']), int(d['local_epoch']), int(d['batch_size'])
    C = int(d['C'])
    torch.manual_seed(100)
    np.random.seed(100)
    r = O.exp_prepare(d['X'], y, d['X_test'], yt, N, float(d['alpha']), P['kernel_par'], D)
    a = (r['X_train'], r['y_train'], r['X_test'], yt.astype(np.int64))
    lr = P['lr']
    out = [O.Centralized(*a, 'classification', C, D, lr, le * R, B, False, 0, False, 0),
           O.Distributed(*a, 'classification', C, D, lr, le * R, B, False, 0, False, 0),
           O.FedAMW_OneShot(*a, r['X_val'], r['y_val'], 'classification', C, D, lr, le * R, B, False, 0, True,
                            P['lambda_reg_os'], R, P['lr_p_os']),
           O.FedAvg(*a, 'classification', C, D, lr, le, B, False, 0, False, 0, R),
           O.FedProx(*a, 'classification', C, D, lr, le, B, True, P['lambda_prox'], False, 0, R),
           O.FedAMW(*a, r['X_val'], r['y_val'], 'classification', C, D, lr, le, B, False, 0, True, P['lambda_reg'], R,
                    P['lr_p'])]
    np.testing.assert_array_equal(torch.empty(4, dtype=torch.int64).random_().numpy(), d['after_torch'])
    np.testing.assert_array_equal(np.random.randint(0, 1 << 30, 4), d['after_np'])
    assert abs(r['hete'] - float(d['heterogeneity'])) <= 1e-4 * abs(float(d['heterogeneity']))
    for k, o in enumerate(out):
        for j, key in enumerate(('train_loss', 'test_loss')):
            got = np.broadcast_to(np.asarray(o[j], dtype=np.float64), (R,))
            np.testing.assert_allclose(got, d[key][k], rtol=0, atol=LOSS_RTOL * max(1.0, np.abs(d[key][k]).max()),
                                       err_msg='%s %d' % (key, k))
        acc = np.broadcast_to(np.asarray(o[2], dtype=np.float64), (R,))
        assert np.abs(acc - d['test_acc'][k]).max() <= 100.0 / len(yt) + 1e-4, k
