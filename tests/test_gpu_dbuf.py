"""The double-buffered instance of the split form (csrc/local_train_dbuf.hip, round 6).

The split form's step with the batch rows streamed ahead of the hand-off (each wave's last tile
two steps ahead into a second register buffer, its other tiles one step ahead) and every
in-loop load counted by hand.  It runs the split form's arithmetic at the same width in the same
order, so the two must agree BITWISE (weights and losses) on every covered shape -- and the
split form is itself pinned to the oracle and the reference fixtures (test_gpu_parity.py).
fs_tuning.split_dbuf = 1 / -1 selects it / the split form's own instances; 0 (default) never
chooses it (a measured tie at configs 2 and 5, slower at config 1: DESIGN.md 4.1).  Reference: train_loop, /root/reference/functions/tools.py:177-215.
"""
import numpy as np
import pytest
import torch

from oracle import fedsim_oracle as O
from tests.test_gpu_parity import _rand_clients, _train_via_abi, amd  # noqa: F401 (fixture)

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("mb_off")]


def _both(amd, Xs, ys, W0, *args, seed=3, split=None):
    """(dbuf W, dbuf loss), (split W, split loss) for the same launch; asserts which ran."""
    with amd.lib.tuning(split_dbuf=1):
        Wd, ld_ = _train_via_abi(amd, Xs, ys, W0, *args, seed=seed, split=split)
        kd = amd.lib.LT_KERNELS[amd.lib.lib().fs_local_train_last_kernel()]
    with amd.lib.tuning(split_dbuf=-1):
        Ws, ls = _train_via_abi(amd, Xs, ys, W0, *args, seed=seed, split=split)
        ks = amd.lib.LT_KERNELS[amd.lib.lib().fs_local_train_last_kernel()]
    assert (kd, ks) == ('dbuf', 'split'), (kd, ks)
    return (Wd, ld_), (Ws, ls)


@pytest.mark.parametrize('G', [2, 4, 8, 16])
@pytest.mark.parametrize('B', [32, 20])
@pytest.mark.parametrize('C', [10, 16, 2])
@pytest.mark.parametrize('reg', [False, True])
@pytest.mark.parametrize('chained', [False, True])
def test_dbuf_bitwise_equals_split(amd, G, B, C, reg, chained):
    """dbuf == split at width G on full 16-tile slices (D = 1024 G - 24: the padded columns stay
    0), ragged clients with tail batches of 1 and 7 rows and an empty client, chained and parallel
    clients, ridge on and off (FedAMW's local training carries it)."""
    if G >= 8 and 32 * C + 2 > 512:
        pytest.skip('the split form exchanges at most 512 values at G >= 8 (C = %d does not fit)' % C)
    rs = np.random.RandomState(G + B + 3 * C + 7 * reg + 11 * chained)
    D, E = 1024 * G - 24, 2
    sizes = [65, 33, 0, 7, 96, 40, 1, 17, 64]
    Xs, ys = _rand_clients(rs, sizes, D, C)
    W0 = (rs.normal(size=(C, D)) * 0.1).astype(np.float32)
    (Wd, ld_), (Ws, ls) = _both(amd, Xs, ys, W0, 0.4, E, B, False, 0.0, reg, 0.002, chained, split=G)
    assert np.array_equal(Wd, Ws), np.abs(Wd - Ws).max()
    assert np.array_equal(ld_, ls), np.abs(ld_ - ls).max()


@pytest.mark.parametrize('G', [4, 8, 16])
@pytest.mark.parametrize('B', [32, 20])
@pytest.mark.parametrize('C', [2, 10])
@pytest.mark.parametrize('terms', ['', 'reg', 'prox', 'prox+reg'])
def test_dbuf_narrow_chained_bitwise(amd, G, B, C, terms):
    """The narrow chained instance (exp.py's config 1: 4 tiles per slice, 4 waves of one tile each,
    every tile double-buffered) == the split form's narrow instance, with FedProx's anchor (the
    previous chained client's result) and the ridge term on and off."""
    reg, prox = 'reg' in terms, 'prox' in terms
    rs = np.random.RandomState(G + B + C + 5 * reg + 9 * prox)
    D, E = 256 * G, 2
    sizes = [300, 33, 0, 7, 96, 1, 64]
    Xs, ys = _rand_clients(rs, sizes, D, C)
    W0 = (rs.normal(size=(C, D)) * 0.1).astype(np.float32)
    (Wd, ld_), (Ws, ls) = _both(amd, Xs, ys, W0, 0.4, E, B, prox, 0.05, reg, 0.002, True, split=G)
    assert np.array_equal(Wd, Ws), np.abs(Wd - Ws).max()
    assert np.array_equal(ld_, ls), np.abs(ld_ - ls).max()


@pytest.mark.parametrize('N,G', [(301, 2), (700, 4), (300, 16)])
def test_dbuf_many_clients(amd, N, G):
    """More clients than groups: every group walks several clients (LPT order, snake over the
    groups), restarting from W_start at each, with the rows of the next client streaming during
    the previous client's last steps.  Bitwise the split form; a sample against the oracle."""
    rs = np.random.RandomState(N)
    D, C, B, E = 1024 * G, 6, 32, 2
    sizes = list(rs.randint(0, 90, size=N))
    Xs, ys = _rand_clients(rs, sizes, D, C)
    W0 = (rs.normal(size=(C, D)) * 0.1).astype(np.float32)
    args = (0.3, E, B, False, 0.0, True, 0.001, False)
    (Wd, ld_), (Ws, ls) = _both(amd, Xs, ys, W0, *args, seed=9, split=G)
    assert np.array_equal(Wd, Ws) and np.array_equal(ld_, ls)
    torch.manual_seed(9)
    for j, (X, y) in enumerate(zip(Xs, ys)):
        if j % 97 == 0 or sizes[j] == 0:
            Wr, lref = O.train_client(X, y, W0, 0.3, E, B, False, 0.0, True, 0.001)
            assert np.abs(Wd[j] - Wr).max() <= 2e-5 * max(1.0, np.abs(Wr).max()), j
            assert abs(ld_[j] - lref) <= 2e-5 * max(1.0, abs(lref)), j
        else:
            torch.empty(2 * E, dtype=torch.int64).random_()     # the oracle's draws for client j


def test_dbuf_vs_oracle_config2_width(amd):
    """The double-buffered instance at config 2's shape (D = 2048, C = 10, B = 32, G = 2), FedAvg,
    every client against the oracle (2e-5 relative: fp32 MFMA vs BLAS summation order)."""
    rs = np.random.RandomState(21)
    D, C, B, E = 2048, 10, 32, 2
    sizes = [512, 100, 33, 1, 64]
    Xs, ys = _rand_clients(rs, sizes, D, C)
    W0 = (rs.normal(size=(C, D)) * 0.1).astype(np.float32)
    lr = 0.4
    with amd.lib.tuning(split_dbuf=1):
        W, loss = _train_via_abi(amd, Xs, ys, W0, lr, E, B, False, 0.0, False, 0.0, False, seed=11, split=2)
        assert amd.lib.LT_KERNELS[amd.lib.lib().fs_local_train_last_kernel()] == 'dbuf'
    torch.manual_seed(11)
    for j, (X, y) in enumerate(zip(Xs, ys)):
        Wr, lref = O.train_client(X, y, W0, lr, E, B, False, 0.0, False, 0.0)
        assert np.abs(W[j] - Wr).max() <= 2e-5 * max(1.0, np.abs(Wr).max()), j
        assert abs(loss[j] - lref) <= 2e-5 * max(1.0, abs(lref)), j


def test_dbuf_timeout_raises(amd):
    """The injected hand-off timeout (fs_tuning.inject_timeout) surfaces as FedsimError."""
    rs = np.random.RandomState(5)
    D, C = 2048, 10
    Xs, ys = _rand_clients(rs, [64, 40], D, C)
    W0 = (rs.normal(size=(C, D)) * 0.1).astype(np.float32)
    with amd.lib.tuning(inject_timeout=1, split_dbuf=1):
        with pytest.raises(amd.lib.FedsimError, match='timed out'):
            _train_via_abi(amd, Xs, ys, W0, 0.3, 2, 32, False, 0.0, False, 0.0, False, split=2)


def test_dbuf_by_shape(amd):
    """Which launches take the double-buffered instance: never by shape (fs_tuning.split_dbuf = 0:
    it measured a tie at configs 2 and 5 and slower at config 1); with split_dbuf = 1 the full
    16-tile slices without a prox term (its 8-wave instance would spill) and the narrow chained
    shape; B <= 16 and the prox term stay on the split form's instances; -1 never."""
    rs = np.random.RandomState(8)
    C = 10

    def kernel(D, B, prox, chained, G, **tune):
        Xs, ys = _rand_clients(rs, [40, 33], D, C)
        W0 = (rs.normal(size=(C, D)) * 0.1).astype(np.float32)
        with amd.lib.tuning(**tune):
            _train_via_abi(amd, Xs, ys, W0, 0.3, 2, B, prox, 0.05, False, 0.0, chained, split=G)
            return amd.lib.LT_KERNELS[amd.lib.lib().fs_local_train_last_kernel()]

    assert kernel(2048, 32, False, False, 2) == 'split'         # by shape: not chosen
    assert kernel(2048, 32, False, True, 8) == 'split'
    assert kernel(2048, 32, False, False, 2, split_dbuf=1) == 'dbuf'
    assert kernel(2048, 32, False, False, 2, split_dbuf=-1) == 'split'
    assert kernel(2048, 32, True, False, 2, split_dbuf=1) == 'split'    # prox: the 8-wave instance stays split
    assert kernel(2048, 16, False, False, 2, split_dbuf=1) == 'split'   # one row tile
    assert kernel(2048, 32, False, True, 8, split_dbuf=1) == 'dbuf'     # narrow chained (4 tiles per slice)
    assert kernel(2048, 32, True, True, 8, split_dbuf=1) == 'dbuf'


@pytest.mark.parametrize('algo', ['fedavg', 'fedamw'])
def test_dbuf_dropin_bitwise(amd, algo):
    """Through the drop-ins (the round plan, the deferred evaluation fused into the training
    launch, FedAMW's p-solve): the double-buffered instance gives bitwise the split form's results
    at config 2's shape class (D = 2048, C = 10, B = 32, parallel clients)."""
    from tests.fixtures import positional  # noqa: F401
    rs = np.random.RandomState(77)
    D, C = 2048, 10
    sizes = [96, 64, 33, 40, 7]
    Xs, ys = _rand_clients(rs, sizes, D, C)
    Xt = (np.cos(rs.normal(size=(200, D))) / np.sqrt(D)).astype(np.float32)
    yt = rs.randint(0, C, size=200).astype(np.int64)
    Xv = (np.cos(rs.normal(size=(64, D))) / np.sqrt(D)).astype(np.float32)
    yv = rs.randint(0, C, size=64).astype(np.int64)
    out = []
    for dbuf in (1, -1):
        with amd.lib.tuning(split_dbuf=dbuf, split_pipe=-1, train_form=1):
            torch.manual_seed(5)
            Xs_t = [torch.from_numpy(x) for x in Xs]
            ys_t = [torch.from_numpy(y) for y in ys]
            stats = {'trace': True}
            if algo == 'fedamw':
                vl = torch.utils.data.DataLoader(torch.utils.data.TensorDataset(torch.from_numpy(Xv), torch.from_numpy(yv)),
                                                 batch_size=16, shuffle=True)
                r = amd.tools.FedAMW(Xs_t, ys_t, torch.from_numpy(Xt), torch.from_numpy(yt), vl, 'classification', C, D,
                                     0.4, 2, 32, False, 0.0, True, 0.001, 4, 1e-3, clients='parallel', stats=stats,
                                     verbose=False)
            else:
                r = amd.tools.FedAvg(Xs_t, ys_t, torch.from_numpy(Xt), torch.from_numpy(yt), 'classification', C, D,
                                     0.4, 2, 32, False, 0.0, False, 0.0, 4, clients='parallel', stats=stats,
                                     verbose=False)
            out.append((r, stats['W_rounds']))
    (a, Wa), (b, Wb) = out
    assert np.array_equal(Wa, Wb)
    for x, y in zip(a, b):
        assert torch.equal(x, y)
