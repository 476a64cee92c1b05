"""The CPU oracle's single-shot algorithms and RFF map against the reference's golden vectors
(tests/golden/make_golden.py: single_*.npz, rff_*.npz)."""
import glob
import os

import numpy as np
import pytest
import torch

from oracle import fedsim_oracle as O
from tests.fixtures import GOLDEN, LOSS_RTOL, P_RTOL, W_RTOL, acc_tol, load, split_clients

SINGLE = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, 'single_*.npz')))
RFF = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, 'rff_*.npz')))


def single_positional(d):
    """tools.py:240 / 258 / 279 positional order (no ``round``)."""
    return ('classification', int(d['C']), int(d['D']), float(d['lr']), int(d['epoch']), int(d['batch_size']),
            bool(d['prox']), float(d['mu']), bool(d['reg']), float(d['lam']))


def run_single_oracle(d):
    Xs, ys = split_clients(d)
    torch.manual_seed(int(d['torch_seed']))
    algo = str(d['algo'])
    if algo == 'centralized':
        return O.Centralized(Xs, ys, d['X_test'], d['y_test'], *single_positional(d))
    if algo == 'distributed':
        return O.Distributed(Xs, ys, d['X_test'], d['y_test'], *single_positional(d))
    return O.FedAMW_OneShot(Xs, ys, d['X_test'], d['y_test'], d['X_val'], d['y_val'], *single_positional(d),
                            int(d['R']), float(d['lr_p']))


def test_fixture_sets_present():
    assert len(SINGLE) >= 6 and len(RFF) >= 2


@pytest.mark.parametrize('name', SINGLE)
def test_single_shot_match_reference(name):
    d = load(name)
    tr, tl, ta, trace = run_single_oracle(d)
    W, Wref = trace['W'], d['W']
    assert W.shape == Wref.shape
    for t in range(len(W)):
        assert np.abs(W[t] - Wref[t]).max() <= W_RTOL * np.abs(Wref[t]).max(), (name, t)
    assert abs(float(tr) - float(d['train_loss'])) <= LOSS_RTOL * max(1.0, abs(float(d['train_loss'])))
    np.testing.assert_allclose(np.atleast_1d(tl), np.atleast_1d(d['test_loss']), rtol=0,
                               atol=LOSS_RTOL * max(1, np.abs(d['test_loss']).max()))
    assert np.abs(np.atleast_1d(ta) - np.atleast_1d(d['test_acc'])).max() <= acc_tol(d)
    if 'p' in d:
        assert np.abs(trace['p'] - d['p']).max() <= P_RTOL * np.abs(d['p']).max()
    # the generator is left exactly where the reference leaves it
    np.testing.assert_array_equal(torch.empty(4, dtype=torch.int64).random_().numpy(), d['rng_after'])


@pytest.mark.parametrize('name', RFF)
def test_rff_draw_bit_exact(name):
    d = load(name)
    torch.manual_seed(int(d['seed']))
    W, b = O.rff(d['X'].shape[1], float(d['sigma']), int(d['D']))
    np.testing.assert_array_equal(W, d['W_rff'])
    np.testing.assert_array_equal(b, d['b_rff'])


@pytest.mark.parametrize('name', RFF)
def test_feature_mapping_matches_reference(name):
    """phi within 4 float32 ulps of the reference's scale (1/sqrt(D)): the K = d matmul's
    summation order (numpy vs MKL) moves cos's argument by ulps."""
    d = load(name)
    D = int(d['D'])
    torch.manual_seed(int(d['seed']))
    tr, te = O.feature_mapping(d['X'][None], d['X_test'], float(d['sigma']), D)
    tol = 4 * np.finfo(np.float32).eps / np.sqrt(D) * max(1.0, float(np.abs(d['X'] @ d['W_rff']).max()))
    assert tr.shape == d['phi'].shape and te.shape == d['phi_test'].shape
    assert np.abs(tr - d['phi']).max() <= tol
    assert np.abs(te - d['phi_test']).max() <= tol
    np.testing.assert_array_equal(torch.empty(4, dtype=torch.int64).random_().numpy(), d['rng_after'])
