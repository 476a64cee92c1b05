"""The split form's multi-block MFMA instances ("mb", round 6, ABI 16: fs_tuning.split_mb).

The classes of the forward z = X_b W^T and the backward grad = g^T X_b run on the 16-block
v_mfma_f32_4x4x1_16b_f32 in ceil(C / 4) blocks of 4 instead of v_mfma_f32_16x16x4_f32 padded to
16 classes (local_train_split.hip, MBK; layouts checked on one wave by scripts/probe/mb_layout.hip).
Same steps, hand-off, softmax and row schedule as the 16x16x4 instances; the products are summed
in another order, so these tests hold them to the oracle (the fp32 tolerance of the reference,
2e-5 relative, as every local-training parity test) and to the 16x16x4 instances at the same
tolerance -- not bitwise.  Reference: train_loop, /root/reference/functions/tools.py:177-215.
"""
import numpy as np
import pytest
import torch

from oracle import fedsim_oracle as O
from tests.test_gpu_parity import _rand_clients, _train_via_abi, amd  # noqa: F401 (fixture)

pytestmark = pytest.mark.gpu

TOL = 2e-5


def _run(amd, Xs, ys, W0, *args, seed=3, split=None, mb=1):
    with amd.lib.tuning(split_mb=mb):
        W, loss = _train_via_abi(amd, Xs, ys, W0, *args, seed=seed, split=split)
        k = amd.lib.LT_KERNELS[amd.lib.lib().fs_local_train_last_kernel()]
    return W, loss, k


def _vs_oracle(Xs, ys, W0, W, loss, lr, E, B, prox, mu, reg, lam, chained, seed):
    torch.manual_seed(seed)     # the oracle draws the same passes (client-major, epoch-minor)
    start = W0
    for j, (X, y) in enumerate(zip(Xs, ys)):
        Wr, lref = O.train_client(X, y, start, lr, E, B, prox, mu, reg, lam)
        assert np.abs(W[j] - Wr).max() <= TOL * max(1.0, np.abs(Wr).max()), (j, np.abs(W[j] - Wr).max())
        assert abs(loss[j] - lref) <= TOL * max(1.0, abs(lref)), (j, loss[j], lref)
        if chained:
            start = Wr


@pytest.mark.parametrize('G', [2, 4, 8, 16])
@pytest.mark.parametrize('C', [2, 7, 10, 16])
@pytest.mark.parametrize('terms', ['', 'reg', 'prox', 'prox+reg'])
@pytest.mark.parametrize('chained', [False, True])
def test_mb_full_slices_vs_oracle(amd, G, C, terms, chained):
    """Full 16-tile slices (D = 1024 G - 24: the padded columns stay 0; the early-issue
    instances), every class-block count (C = 2, 7, 10, 16 -> 1, 2, 3, 4 blocks), ridge and
    FedProx terms, chained and parallel clients, ragged clients with tail batches of 1 and 7 rows
    and an empty client."""
    if G >= 8 and 32 * C + 2 > 512:
        pytest.skip('the split form exchanges at most 512 values at G >= 8 (C = %d does not fit)' % C)
    reg, prox = 'reg' in terms, 'prox' in terms
    rs = np.random.RandomState(G + 3 * C + 5 * reg + 7 * prox + 11 * chained)
    D, E, B = 1024 * G - 24, 2, 32
    sizes = [65, 33, 0, 7, 96, 1, 40]
    Xs, ys = _rand_clients(rs, sizes, D, C)
    W0 = (rs.normal(size=(C, D)) * 0.1).astype(np.float32)
    args = (0.4, E, B, prox, 0.03, reg, 0.002, chained)
    W, loss, k = _run(amd, Xs, ys, W0, *args, seed=11, split=G)
    assert k == 'mb'
    _vs_oracle(Xs, ys, W0, W, loss, *args, seed=11)


@pytest.mark.parametrize('D,G', [(200, 2), (300, 4), (1000, 2), (2500, 4), (5000, 8)])
@pytest.mark.parametrize('C', [3, 10])
@pytest.mark.parametrize('prox', [False, True])
@pytest.mark.parametrize('chained', [False, True])
def test_mb_partial_slices_vs_oracle(amd, D, G, C, prox, chained):
    """Slices that are not full (fewer tiles than 8 waves x 2, D not a multiple of 64): the late
    instances, whose tile guards split the step; B = 20 (a partial second row tile)."""
    rs = np.random.RandomState(D + G + C + 13 * prox + 17 * chained)
    Xs, ys = _rand_clients(rs, [50, 21, 0, 9, 77], D, C)
    W0 = (rs.normal(size=(C, D)) * 0.1).astype(np.float32)
    args = (0.3, 2, 20, prox, 0.05, True, 0.001, chained)
    W, loss, k = _run(amd, Xs, ys, W0, *args, seed=5, split=G)
    assert k == 'mb'
    _vs_oracle(Xs, ys, W0, W, loss, *args, seed=5)


@pytest.mark.parametrize('G,tiles', [(4, 4), (8, 4), (16, 4), (4, 8), (8, 8)])
@pytest.mark.parametrize('C', [2, 10])
@pytest.mark.parametrize('prox', [False, True])
def test_mb_narrow_chained_vs_oracle(amd, G, tiles, C, prox):
    """The narrow chained instances (exp.py's config 1 shape class: one tile per wave, 4 waves at
    4 tiles per slice, 8 at 8) on the mb MFMAs."""
    rs = np.random.RandomState(G + tiles + C + 3 * prox)
    D = 64 * tiles * G - 48
    Xs, ys = _rand_clients(rs, [300, 33, 0, 7, 96, 1, 64], D, C)
    W0 = (rs.normal(size=(C, D)) * 0.1).astype(np.float32)
    args = (0.4, 2, 32, prox, 0.05, True, 0.002, True)
    W, loss, k = _run(amd, Xs, ys, W0, *args, seed=7, split=G)
    assert k == 'mb'
    _vs_oracle(Xs, ys, W0, W, loss, *args, seed=7)


@pytest.mark.parametrize('N,G', [(301, 2), (700, 4), (300, 16)])
def test_mb_many_clients(amd, N, G):
    """More clients than groups: every group walks several clients (LPT order, snake over the
    groups), restarting from W_start at each; against the 16x16x4 instances (tolerance) and a
    sample against the oracle."""
    rs = np.random.RandomState(N)
    D, C, B, E = 1024 * G, 10, 32, 2
    sizes = list(rs.randint(0, 90, size=N))
    Xs, ys = _rand_clients(rs, sizes, D, C)
    W0 = (rs.normal(size=(C, D)) * 0.1).astype(np.float32)
    args = (0.3, E, B, False, 0.0, True, 0.001, False)
    Wm, lm, k = _run(amd, Xs, ys, W0, *args, seed=9, split=G)
    assert k == 'mb'
    Ws, ls, k2 = _run(amd, Xs, ys, W0, *args, seed=9, split=G, mb=-1)
    assert k2 == 'split'
    assert np.abs(Wm - Ws).max() <= TOL * max(1.0, np.abs(Ws).max())
    assert np.abs(lm - ls).max() <= TOL * max(1.0, np.abs(ls).max())
    torch.manual_seed(9)
    for j, (X, y) in enumerate(zip(Xs, ys)):
        if j % 97 == 0 or sizes[j] == 0:
            Wr, lref = O.train_client(X, y, W0, *args[:-1])
            assert np.abs(Wm[j] - Wr).max() <= TOL * max(1.0, np.abs(Wr).max()), j
            assert abs(lm[j] - lref) <= TOL * max(1.0, abs(lref)), j
        else:
            torch.empty(2 * E, dtype=torch.int64).random_()     # the oracle's draws for client j


def test_mb_timeout_raises(amd):
    """The injected hand-off timeout (fs_tuning.inject_timeout) surfaces as FedsimError."""
    rs = np.random.RandomState(5)
    D, C = 2048, 10
    Xs, ys = _rand_clients(rs, [64, 40], D, C)
    W0 = (rs.normal(size=(C, D)) * 0.1).astype(np.float32)
    with amd.lib.tuning(inject_timeout=1, split_mb=1):
        with pytest.raises(amd.lib.FedsimError, match='timed out'):
            _train_via_abi(amd, Xs, ys, W0, 0.3, 2, 32, False, 0.0, False, 0.0, False, split=2)


def test_mb_selection(amd):
    """Which launches take the mb instances: by shape (split_mb = 0) where C <= 8 (at most 2
    class blocks: configs 1 and 3) or C <= 12 at G = 16 (config 5), split_mb = 1 wherever the split form runs with 16 < B <= 32;
    B <= 16 (one row tile) stays on the 16x16x4 instances; -1 never."""
    rs = np.random.RandomState(8)

    def kernel(D, B, G, chained=False, C=10, **tune):
        Xs, ys = _rand_clients(rs, [40, 33], D, C)
        W0 = (rs.normal(size=(C, D)) * 0.1).astype(np.float32)
        with amd.lib.tuning(**tune):
            _train_via_abi(amd, Xs, ys, W0, 0.3, 2, B, False, 0.0, False, 0.0, chained, split=G)
            return amd.lib.LT_KERNELS[amd.lib.lib().fs_local_train_last_kernel()]

    assert kernel(2048, 32, 2) == 'split'                  # C = 10 at G = 2 by shape: the 16x16x4 instances
    assert kernel(16384, 32, 16) == 'mb'                   # C = 10 at G = 16 (config 5's shape class)
    assert kernel(2048, 32, 2, C=8) == 'mb'                # C <= 8 by shape
    assert kernel(4096, 32, 4, C=7) == 'mb'                # config 3's shape class
    assert kernel(2000, 32, 8, chained=True, C=2) == 'mb'  # config 1's (narrow chained)
    assert kernel(2048, 32, 2, C=7, split_mb=-1) == 'split'
    assert kernel(2048, 32, 2, split_mb=1) == 'mb'
    assert kernel(2048, 32, 2, split_mb=-1) == 'split'
    assert kernel(2048, 16, 2, split_mb=1) == 'split'     # one row tile
    assert kernel(2048, 32, 8, chained=True, split_mb=1) == 'mb'


@pytest.mark.parametrize('algo', ['fedavg', 'fedprox', 'fedamw'])
def test_mb_dropin_vs_16x16(amd, algo):
    """Through the drop-ins (the round plan, the deferred evaluation fused into the training
    launch, FedAMW's p-solve): the mb instances' rounds against the 16x16x4 instances' at config
    2's shape class (D = 2048, C = 10, B = 32, parallel clients), within the fp32 tolerance."""
    rs = np.random.RandomState(77)
    D, C = 2048, 10
    sizes = [96, 64, 33, 40, 7]
    Xs, ys = _rand_clients(rs, sizes, D, C)
    Xt = (np.cos(rs.normal(size=(200, D))) / np.sqrt(D)).astype(np.float32)
    yt = rs.randint(0, C, size=200).astype(np.int64)
    Xv = (np.cos(rs.normal(size=(64, D))) / np.sqrt(D)).astype(np.float32)
    yv = rs.randint(0, C, size=64).astype(np.int64)
    out = []
    for mb in (1, -1):
        with amd.lib.tuning(split_mb=mb, split_pipe=-1, train_form=1):
            torch.manual_seed(5)
            Xs_t = [torch.from_numpy(x) for x in Xs]
            ys_t = [torch.from_numpy(y) for y in ys]
            stats = {'trace': True}
            Xt_t, yt_t = torch.from_numpy(Xt), torch.from_numpy(yt)
            if algo == 'fedamw':
                vl = torch.utils.data.DataLoader(torch.utils.data.TensorDataset(torch.from_numpy(Xv), torch.from_numpy(yv)),
                                                 batch_size=16, shuffle=True)
                r = amd.tools.FedAMW(Xs_t, ys_t, Xt_t, yt_t, vl, 'classification', C, D,
                                     0.4, 2, 32, False, 0.0, True, 0.001, 4, 1e-3, clients='parallel', stats=stats,
                                     verbose=False)
            elif algo == 'fedprox':
                r = amd.tools.FedProx(Xs_t, ys_t, Xt_t, yt_t, 'classification', C, D,
                                      0.4, 2, 32, True, 0.05, False, 0.0, 4, clients='parallel', stats=stats,
                                      verbose=False)
            else:
                r = amd.tools.FedAvg(Xs_t, ys_t, Xt_t, yt_t, 'classification', C, D,
                                     0.4, 2, 32, False, 0.0, False, 0.0, 4, clients='parallel', stats=stats,
                                     verbose=False)
            out.append((r, stats['W_rounds']))
    (a, Wa), (b, Wb) = out
    # 4 rounds of 2-epoch local training and the aggregate: the per-round drift stays within
    # the horizon tolerance the round-level goldens use (2e-5 per round, relative)
    assert np.abs(Wa - Wb).max() <= 4 * TOL * max(1.0, np.abs(Wb).max())
    for x, y in zip(a, b):
        assert np.allclose(x.numpy(), y.numpy(), rtol=0, atol=4 * TOL * max(1.0, float(np.abs(y.numpy()).max())))
