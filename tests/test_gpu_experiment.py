"""exp.py-counterpart on the MI355X: the heterogeneity kernels (fs_gram, fs_hetero) vs the
oracle, the driver's data preparation vs the oracle's restatement of exp.py:60-99 (same seeds,
same synthetic LIBSVM-shaped input), and an end-to-end run of all six algorithms.

Tolerances: Gram within 1e-5 * max|G| (fp32 MFMA vs BLAS summation order); per-client
squared distances within 1e-3 relative and the heterogeneity within 1e-4 relative (a
difference of near-equal fp32 matrices amplifies the Gram's rounding); features as in
tests/test_gpu_single.py; indices, labels and the split exact.
"""
import os
import pickle

import numpy as np
import pytest
import torch

from oracle import fedsim_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def amd():
    import fedamw_amd
    from fedamw_amd import _lib, engine, experiment
    from fedamw_amd.functions import utils
    _lib.lib()
    return type('amd', (), dict(lib=_lib, engine=engine, experiment=experiment, utils=utils))


@pytest.mark.parametrize('sizes,D', [([200, 3, 150, 347], 100), ([64, 64], 64), ([500, 120, 33], 257)])
def test_gram_and_heterogeneity_vs_oracle(amd, sizes, D):
    rs = np.random.RandomState(sum(sizes) + D)
    Xs = [(np.cos(rs.normal(size=(n, D)) + k) / np.sqrt(D)).astype(np.float32) for k, n in enumerate(sizes)]
    ys = [np.zeros(n, np.int64) for n in sizes]
    feats = amd.engine.Features([torch.from_numpy(x) for x in Xs], [torch.from_numpy(y) for y in ys], D,
                                torch.device('cuda'))
    hete, S = amd.engine.heterogeneity(feats)
    phi = np.concatenate(Xs)
    off = np.concatenate([[0], np.cumsum(sizes)])
    parts = [np.arange(off[i], off[i + 1]) for i in range(len(sizes))]
    G = phi.astype(np.float64).T @ phi.astype(np.float64)
    Sref = [np.sum((G / len(phi) - phi[p].astype(np.float64).T @ phi[p] / len(p)) ** 2) for p in parts]
    np.testing.assert_allclose(S, Sref, rtol=1e-3)
    ref = O.heterogeneity(phi, parts)
    assert abs(hete - ref) <= 1e-4 * abs(ref)
    Gd = torch.empty(D, D, device='cuda')
    amd.lib.check(amd.lib.lib().fs_gram(amd.lib.ptr(feats.phi), feats.ld, int(feats.rows), D, amd.lib.ptr(Gd), D,
                                        amd.lib.stream_ptr()), 'fs_gram')
    Gg = Gd.cpu().numpy()
    assert np.array_equal(Gg, Gg.T)
    assert np.abs(Gg - G).max() <= 1e-5 * np.abs(G).max()


def test_prepare_matches_oracle(amd):
    synth = dict(n_train=900, n_test=150)
    D, N, alpha = 64, 4, 0.5
    params = {'kernel_par': 0.1, 'kernel_type': 'gaussian'}
    torch.manual_seed(100)
    np.random.seed(100)
    d = amd.experiment.prepare('a9a', D, N, alpha, params, '/nonexistent/', synth=synth, verbose=False)
    after_t = torch.empty(3, dtype=torch.int64).random_().numpy()
    after_np = np.random.randint(0, 1 << 30, 3)
    X, y, Xt, yt = amd.utils.synthetic_libsvm('a9a', **synth)
    torch.manual_seed(100)
    np.random.seed(100)
    r = O.exp_prepare(X, y, Xt, yt, N, alpha, 0.1, D)
    np.testing.assert_array_equal(torch.empty(3, dtype=torch.int64).random_().numpy(), after_t)
    np.testing.assert_array_equal(np.random.randint(0, 1 << 30, 3), after_np)
    assert [list(p) for p in d['index_partitions']] == [list(p) for p in r['parts']]
    tol = 4 * np.finfo(np.float32).eps / np.sqrt(D) * 8
    for a, b, ya, yb in zip(d['X_train'], r['X_train'], d['y_train'], r['y_train']):
        np.testing.assert_array_equal(ya.numpy(), yb)
        assert np.abs(a.cpu().numpy() - b).max() <= tol
    np.testing.assert_array_equal(d['y_val'].numpy(), r['y_val'])
    assert np.abs(d['X_val'].numpy() - r['X_val']).max() <= tol
    assert np.abs(d['X_test'].cpu().numpy() - r['X_test']).max() <= tol
    assert abs(d['heterogeneity'] - r['hete']) <= 1e-4 * abs(r['hete'])


def test_prepare_matches_reference_fixture(amd, tmp_path):
    """experiment.prepare (LIBSVM parse, Dirichlet partition, full-batch replay, fs_feature_map,
    fs_gram / fs_hetero, 20/80 split) on the LIBSVM files the reference's own load_full_data
    read in make_golden.py (prep_a9a.npz), against the reference's outputs."""
    from sklearn.datasets import dump_svmlight_file
    from tests.fixtures import load
    d = load('prep_a9a')
    root = tmp_path / 'datasets'
    root.mkdir()
    dump_svmlight_file(d['X'], d['y'], str(root / 'a9a'), zero_based=False)
    dump_svmlight_file(d['X_test'], d['y_test'], str(root / 'a9a.t'), zero_based=False)
    N, D = int(d['n_clients']), int(d['D'])
    torch.manual_seed(100)
    np.random.seed(100)
    r = amd.experiment.prepare('a9a', D, N, float(d['alpha']), {'kernel_par': float(d['k_par']),
                                                                 'kernel_type': 'gaussian'},
                               str(root) + '/', verbose=False)
    np.testing.assert_array_equal(torch.empty(4, dtype=torch.int64).random_().numpy(), d['after_torch'])
    np.testing.assert_array_equal(np.random.randint(0, 1 << 30, 4), d['after_np'])
    off = np.concatenate([[0], np.cumsum(d['part_len'])])
    parts = [d['parts'][off[i]:off[i + 1]] for i in range(N)]
    assert [list(p) for p in r['index_partitions']] == [list(p) for p in parts]
    soff = np.concatenate([[0], np.cumsum(d['split_len'])])
    toff = np.concatenate([[0], np.cumsum(d['part_len'] - d['split_len'])])
    yv = np.concatenate([d['y_all'][p][d['val_idx'][soff[j]:soff[j + 1]]] for j, p in enumerate(parts)])
    np.testing.assert_array_equal(r['y_val'].numpy(), yv)
    for j, p in enumerate(parts):
        np.testing.assert_array_equal(r['y_train'][j].numpy(), d['y_all'][p][d['train_idx'][toff[j]:toff[j + 1]]])
    # features (fs_feature_map vs torch's CPU map): the validation rows of every client's block
    Xv = r['X_val'].numpy()
    for j in range(N):
        vi = d['val_idx'][soff[j]:soff[j + 1]]
        for k, row in enumerate(vi):
            if row < 4:
                assert np.abs(Xv[soff[j] + k] - d['phi_head'][j][row]).max() <= 1e-5, (j, row)
    assert np.abs(r['X_test'][:16].cpu().numpy() - d['phi_test_head']).max() <= 1e-5
    assert abs(r['heterogeneity'] - float(d['hete'])) <= 1e-4 * abs(float(d['hete']))


def test_experiment_end_to_end(amd, tmp_path):
    out = amd.experiment.run('a9a', D=64, num_partitions=4, local_epoch=1, Round=3, n_repeats=1, alpha_Dirk=0.5,
                             data_dir='/nonexistent/', result_dir=str(tmp_path), synth=dict(n_train=700, n_test=120),
                             verbose=False)
    for k in ('train_loss', 'test_loss', 'test_acc'):
        assert out[k].shape == (6, 3, 1) and np.isfinite(out[k]).all(), k
    assert out['name'] == ['CL', 'DL', 'FedAMW_OneShot', 'FedAvg', 'FedProx', 'FedAMW']
    with open(os.path.join(str(tmp_path), 'exp1_a9a.pkl'), 'rb') as f:      # written by this test
        saved = pickle.load(f)
    assert saved['epochs'] == 3 and saved['heterogeneity'].shape == (1,)
    assert ((out['test_acc'] >= 0) & (out['test_acc'] <= 100)).all()


def test_experiment_matches_reference_sequence(amd, tmp_path):
    """exp.py's whole sequence on ONE un-reseeded stream (exp_satimage.npz: the reference's
    load_full_data on the same LIBSVM files, exp.py:61-99 restated, then its six algorithm calls
    in order with get_parameter('satimage')): every returned loss / accuracy of the six
    algorithms, the heterogeneity and where both global generators end up -- so the stream
    continuity across the calls is pinned, not just each call after a reseed."""
    from sklearn.datasets import dump_svmlight_file
    from tests.fixtures import LOSS_RTOL, load
    d = load('exp_satimage')
    root = tmp_path / 'datasets'
    root.mkdir()
    name = str(d['dataset'])
    dump_svmlight_file(d['X'], d['y'], str(root / name), zero_based=False)
    dump_svmlight_file(d['X_test'], d['y_test'], str(root / (name + '.t')), zero_based=False)
    out = amd.experiment.run(name, D=int(d['D']), num_partitions=int(d['N']), local_epoch=int(d['local_epoch']),
                             Round=int(d['Round']), batch_size=int(d['batch_size']), n_repeats=1,
                             alpha_Dirk=float(d['alpha']), data_dir=str(root) + '/', save=False, verbose=False)
    np.testing.assert_array_equal(torch.empty(4, dtype=torch.int64).random_().numpy(), d['after_torch'])
    np.testing.assert_array_equal(np.random.randint(0, 1 << 30, 4), d['after_np'])
    assert abs(out['heterogeneity'][0] - float(d['heterogeneity'])) <= 1e-4 * abs(float(d['heterogeneity']))
    for key in ('train_loss', 'test_loss'):
        got, ref = out[key][:, :, 0], d[key]
        np.testing.assert_allclose(got, ref, rtol=0, atol=LOSS_RTOL * max(1.0, np.abs(ref).max()), err_msg=key)
    assert np.abs(out['test_acc'][:, :, 0] - d['test_acc']).max() <= 100.0 / len(d['y_test']) + 1e-4
