"""HIP path of the single-shot algorithms (Centralized, Distributed, FedAMW_OneShot;
tools.py:240-326) and of the RFF feature map (tools.py:15-31) vs the reference's golden
vectors and the CPU oracle (MI355X box).

Tolerances: global W within 1e-5 * max|W_ref| (tests/fixtures.py), losses 1e-5, accuracy one
test sample, p 1e-5 * max|p|; feature map within 4 fp32 ulps of scale * max(1, |X W|) (the
K = d dot product's summation order moves cos's argument by ulps).
"""
import glob
import os

import numpy as np
import pytest
import torch

from oracle import fedsim_oracle as O
from tests.fixtures import GOLDEN, LOSS_RTOL, P_RTOL, W_RTOL, acc_tol, load, split_clients
from tests.test_oracle_single import RFF, SINGLE, single_positional

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def amd():
    import fedamw_amd
    from fedamw_amd import _lib, engine
    from fedamw_amd.functions import tools
    _lib.lib()
    return type('amd', (), dict(lib=_lib, engine=engine, tools=tools))


def _dl(X, y, bs=16):
    return torch.utils.data.DataLoader(torch.utils.data.TensorDataset(torch.from_numpy(X), torch.from_numpy(y)),
                                       batch_size=bs, shuffle=True)


@pytest.mark.parametrize('name', SINGLE)
def test_single_shot_dropin_matches_reference(amd, name):
    d = load(name)
    Xs, ys = split_clients(d)
    Xs = [torch.from_numpy(x) for x in Xs]
    ys = [torch.from_numpy(y) for y in ys]
    Xt, yt = torch.from_numpy(d['X_test']), torch.from_numpy(d['y_test'])
    algo = str(d['algo'])
    stats = {'trace': True}
    torch.manual_seed(int(d['torch_seed']))
    if algo == 'centralized':
        tr, tl, ta = amd.tools.Centralized(Xs, ys, Xt, yt, *single_positional(d), stats=stats, verbose=False)
        assert all(isinstance(v, float) for v in (tr, tl, ta))      # Meter averages (tools.py:255)
        W = stats['W_global'].cpu().numpy()[None]
    elif algo == 'distributed':
        tr, tl, ta = amd.tools.Distributed(Xs, ys, Xt, yt, *single_positional(d), stats=stats, verbose=False)
        assert isinstance(tr, torch.Tensor) and tr.dim() == 0 and tr.dtype == torch.float32
        W = stats['W_global'].cpu().numpy()[None]
    else:
        tr, tl, ta = amd.tools.FedAMW_OneShot(Xs, ys, Xt, yt, _dl(d['X_val'], d['y_val']), *single_positional(d),
                                              int(d['R']), float(d['lr_p']), stats=stats, verbose=False)
        assert tl.shape == (int(d['R']),) and ta.shape == (int(d['R']),)
        W = stats['W_rounds']
        p = stats['p_rounds']
        assert np.abs(p - d['p']).max() <= P_RTOL * np.abs(d['p']).max()
    Wref = d['W']
    assert W.shape == Wref.shape
    for t in range(len(Wref)):
        err = np.abs(W[t] - Wref[t]).max()
        assert err <= W_RTOL * np.abs(Wref[t]).max(), (name, t, err)
    assert abs(float(tr) - float(d['train_loss'])) <= LOSS_RTOL * max(1.0, abs(float(d['train_loss'])))
    tl, ta = np.atleast_1d(np.asarray(tl, dtype=np.float64)), np.atleast_1d(np.asarray(ta, dtype=np.float64))
    np.testing.assert_allclose(tl, np.atleast_1d(d['test_loss']), rtol=0,
                               atol=LOSS_RTOL * max(1, np.abs(d['test_loss']).max()))
    assert np.abs(ta - np.atleast_1d(d['test_acc'])).max() <= acc_tol(d)
    # the global generator is left exactly where the reference leaves it
    np.testing.assert_array_equal(torch.empty(4, dtype=torch.int64).random_().numpy(), d['rng_after'])


def _fm_tol(X, W, D):
    return 4 * np.finfo(np.float32).eps / np.sqrt(D) * max(1.0, float(np.abs(X @ W).max()))


@pytest.mark.parametrize('name', RFF)
def test_feature_mapping_dropin_matches_reference(amd, name):
    d = load(name)
    D = int(d['D'])
    torch.manual_seed(int(d['seed']))
    tr, te = amd.tools.feature_mapping(torch.from_numpy(d['X'][None]), torch.from_numpy(d['X_test']),
                                       float(d['sigma']), D, 'gaussian')
    np.testing.assert_array_equal(torch.empty(4, dtype=torch.int64).random_().numpy(), d['rng_after'])
    assert tr.is_cuda and tuple(tr.shape) == d['phi'].shape and tuple(te.shape) == d['phi_test'].shape
    tol = _fm_tol(d['X'], d['W_rff'], D)
    assert np.abs(tr.cpu().numpy() - d['phi']).max() <= tol
    assert np.abs(te.cpu().numpy() - d['phi_test']).max() <= tol


@pytest.mark.parametrize('n,d,D,ldo', [
    (1, 1, 1, 1),            # smallest
    (63, 5, 64, 64),         # one row short of a tile
    (130, 123, 2000, 2048),  # a9a width (d % 4 != 0, > one 32-wide K chunk), D padded to the engine's ld
    (97, 54, 200, 256),      # covtype width, D not a multiple of 64
    (64, 33, 130, 130),      # K chunk boundary + 1
])
def test_feature_map_kernel_vs_oracle(amd, n, d, D, ldo):
    rs = np.random.RandomState(n + d + D)
    X = (rs.rand(n, d) < 0.2).astype(np.float32)
    X[:, : min(3, d)] = rs.rand(n, min(3, d))
    W = rs.normal(0, 0.7, size=(d, D)).astype(np.float32)
    b = rs.uniform(0, 2 * np.pi, size=(1, D)).astype(np.float32)
    out = amd.engine.feature_map(torch.from_numpy(X), torch.from_numpy(W), torch.from_numpy(b), D, ldo=ldo)
    got = out.cpu().numpy()
    ref = O.feature_map(X, W, b, D)
    assert np.abs(got[:, :D] - ref).max() <= _fm_tol(X, W, D)
    assert (got[:, D:] == 0).all()


def test_feature_map_full_size_properties(amd):
    """Config-3-sized map (covtype-shaped, 200k rows x 4096 features): sampled rows vs the oracle,
    |phi| <= 1/sqrt(D) everywhere, padding zero."""
    n, d, D, ldo = 200_000, 54, 4096, 4096 + 64
    g = torch.Generator().manual_seed(5)
    X = (torch.rand(n, d, generator=g) < 0.25).float()
    X[:, :10] = torch.rand(n, 10, generator=g)
    W = torch.randn(d, D, generator=g) * 0.1
    b = torch.rand(1, D, generator=g) * 2 * np.pi
    out = amd.engine.feature_map(X, W, b, D, ldo=ldo)
    scale = np.float32(1 / np.sqrt(D))
    assert float(out[:, :D].abs().max()) <= scale * (1 + 1e-6)
    assert float(out[:, D:].abs().max()) == 0.0
    rows = np.random.RandomState(0).choice(n, 512, replace=False)
    ref = O.feature_map(X[rows].numpy(), W.numpy(), b.numpy(), D)
    assert np.abs(out[rows, :D].cpu().numpy() - ref).max() <= _fm_tol(X[rows].numpy(), W.numpy(), D)
