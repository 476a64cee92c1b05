"""The pipelined split form of fs_local_train (csrc/local_train_pipe.hip, ABI 14, G | G_PIPE).

A group of G workgroups trains one client at a time as the split form does, with each step's
hand-off pipelined by 16-row tile and the softmax computed per wave in registers; per step it
runs the split form's arithmetic at the same width in the same order, so the two forms must
agree BITWISE (weights and losses) on every covered shape -- and the split form is itself pinned
to the oracle and the reference fixtures (test_gpu_parity.py).  Reference: train_loop,
/root/reference/functions/tools.py:177-215 (FedAvg / FedAMW local training; FedProx's prox term).
"""
import numpy as np
import pytest
import torch

from oracle import fedsim_oracle as O
from tests.test_gpu_parity import _rand_clients, _train_via_abi, amd  # noqa: F401 (fixture)

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("mb_off")]


def _pipe(amd, G):
    return G | amd.lib.G_PIPE


@pytest.mark.parametrize('G', [2, 4, 8, 16])
@pytest.mark.parametrize('B', [32, 20])
@pytest.mark.parametrize('C', [10, 16, 2])
@pytest.mark.parametrize('terms', ['', 'reg', 'prox', 'prox+reg'])
@pytest.mark.parametrize('chained', [False, True])
def test_pipe_bitwise_equals_split(amd, G, B, C, terms, chained):
    """Pipe form == split form at width G, bitwise: D = 1024 G - 24 (the padded columns stay 0),
    ragged clients incl. tail batches of 1 and 7 rows and an empty client, chained and parallel
    clients, ridge on and off (FedAMW's local training carries the ridge term), FedProx's prox
    term on and off (its anchor: W_start, or in a chain the previous client's result)."""
    if G >= 8 and 32 * C + 2 > 512:
        pytest.skip('the split form exchanges at most 512 values at G >= 8 (C = %d does not fit)' % C)
    reg, prox = 'reg' in terms, 'prox' in terms
    rs = np.random.RandomState(G + B + 3 * C + 7 * reg + 11 * chained + 13 * prox)
    D, E = 1024 * G - 24, 2
    sizes = [65, 33, 0, 7, 96, 40, 1, 17, 64]
    Xs, ys = _rand_clients(rs, sizes, D, C)
    W0 = (rs.normal(size=(C, D)) * 0.1).astype(np.float32)
    lr, lam, mu = 0.4, 0.002, 0.05
    Wp, lp = _train_via_abi(amd, Xs, ys, W0, lr, E, B, prox, mu, reg, lam, chained, seed=3, split=_pipe(amd, G))
    assert _train_via_abi.last_G == _pipe(amd, G)
    Ws, ls = _train_via_abi(amd, Xs, ys, W0, lr, E, B, prox, mu, reg, lam, chained, seed=3, split=G)
    assert _train_via_abi.last_G == G
    assert np.array_equal(Wp, Ws), np.abs(Wp - Ws).max()
    assert np.array_equal(lp, ls), np.abs(lp - ls).max()


@pytest.mark.parametrize('N,G', [(301, 2), (700, 4), (300, 16)])
def test_pipe_many_clients(amd, N, G):
    """More clients than groups: every group walks several clients (LPT order, snake over the
    groups), restarting from W_start at each; the next client's rows stream during the previous
    client's last step.  Bitwise the split form; a sample of clients against the oracle."""
    rs = np.random.RandomState(N)
    D, C, B, E = 1024 * G, 6, 32, 2
    sizes = list(rs.randint(0, 90, size=N))
    Xs, ys = _rand_clients(rs, sizes, D, C)
    W0 = (rs.normal(size=(C, D)) * 0.1).astype(np.float32)
    args = (0.3, E, B, False, 0.0, True, 0.001, False)
    Wp, lp = _train_via_abi(amd, Xs, ys, W0, *args, seed=9, split=_pipe(amd, G))
    Ws, ls = _train_via_abi(amd, Xs, ys, W0, *args, seed=9, split=G)
    assert np.array_equal(Wp, Ws) and np.array_equal(lp, ls)
    torch.manual_seed(9)
    for j, (X, y) in enumerate(zip(Xs, ys)):
        if j % 97 == 0 or sizes[j] == 0:
            Wr, lref = O.train_client(X, y, W0, 0.3, E, B, False, 0.0, True, 0.001)
            assert np.abs(Wp[j] - Wr).max() <= 2e-5 * max(1.0, np.abs(Wr).max()), j
            assert abs(lp[j] - lref) <= 2e-5 * max(1.0, abs(lref)), j
        else:
            torch.empty(2 * E, dtype=torch.int64).random_()     # the oracle's draws for client j


def test_pipe_vs_oracle_config2_width(amd):
    """The pipe form at config 2's shape (D = 2048, C = 10, B = 32, G = 2), FedAvg, every client
    against the oracle (2e-5 relative: fp32 MFMA vs BLAS summation order)."""
    rs = np.random.RandomState(21)
    D, C, B, E = 2048, 10, 32, 2
    sizes = [512, 100, 33, 1, 64]
    Xs, ys = _rand_clients(rs, sizes, D, C)
    W0 = (rs.normal(size=(C, D)) * 0.1).astype(np.float32)
    lr = 0.4
    W, loss = _train_via_abi(amd, Xs, ys, W0, lr, E, B, False, 0.0, False, 0.0, False, seed=11,
                             split=_pipe(amd, 2))
    assert _train_via_abi.last_G == _pipe(amd, 2)
    torch.manual_seed(11)
    for j, (X, y) in enumerate(zip(Xs, ys)):
        Wr, lref = O.train_client(X, y, W0, lr, E, B, False, 0.0, False, 0.0)
        assert np.abs(W[j] - Wr).max() <= 2e-5 * max(1.0, np.abs(Wr).max()), j
        assert abs(loss[j] - lref) <= 2e-5 * max(1.0, abs(lref)), j


def test_pipe_timeout_raises(amd):
    """The injected hand-off timeout (fs_tuning.inject_timeout) surfaces as FedsimError."""
    rs = np.random.RandomState(5)
    D, C = 2048, 10
    Xs, ys = _rand_clients(rs, [64, 40], D, C)
    W0 = (rs.normal(size=(C, D)) * 0.1).astype(np.float32)
    with amd.lib.tuning(inject_timeout=1):
        with pytest.raises(amd.lib.FedsimError, match='timed out'):
            _train_via_abi(amd, Xs, ys, W0, 0.3, 2, 32, False, 0.0, False, 0.0, False, split=_pipe(amd, 2))


def test_pipe_planner(amd):
    """fs_local_train_plan: an explicit pipe request is honoured where the form covers the shape
    (ld = 1024 G, 16 < B <= 32, C <= 16) and falls back to the planner's own choice
    elsewhere; fs_tuning.split_pipe = 1 picks it wherever it fits, -1 never."""
    import ctypes
    L = amd.lib.lib()

    def plan(N, C, B, ld, chained=0, prox=0, want=0):
        g, ws = ctypes.c_int(want), ctypes.c_int64(0)
        amd.lib.check(L.fs_local_train_plan(N, C, B, 2, ld, 2 * 512, chained, prox, ctypes.byref(g),
                                            ctypes.byref(ws)), 'plan')
        return g.value, ws.value

    P = amd.lib.G_PIPE
    assert plan(100, 10, 32, 2048, want=2 | P)[0] == 2 | P
    assert plan(100, 10, 32, 4096, want=4 | P)[0] == 4 | P
    assert plan(1000, 10, 32, 16384, want=16 | P)[0] == 16 | P
    assert plan(10, 2, 32, 2048, chained=1, want=2 | P)[0] == 2 | P
    assert plan(100, 7, 32, 4096, prox=1, want=4 | P)[0] == 4 | P
    for args in [dict(B=16), dict(B=32, ld=1024 * 2 + 64), dict(B=32, C=17)]:
        a = dict(N=100, C=10, B=32, ld=2048)
        a.update(args)
        assert not plan(want=2 | P, **a)[0] & P, args
    with amd.lib.tuning(split_pipe=1):
        g, ws = plan(100, 10, 32, 2048)
        assert g == 2 | P and ws > 256
        # explicit split / pair / team requests keep their own form under split_pipe = 1
        # (they used to come back as the pipe form)
        assert plan(100, 10, 32, 2048, want=4)[0] == 4
        assert plan(100, 10, 32, 2048, want=4 | amd.lib.G_PAIR)[0] == 4 | amd.lib.G_PAIR
        assert plan(100, 10, 32, 2048, want=4 | amd.lib.G_TEAMS)[0] == 4 | amd.lib.G_TEAMS
    with amd.lib.tuning(split_pipe=-1):
        assert not plan(100, 10, 32, 2048)[0] & P


@pytest.mark.parametrize('algo', ['fedavg', 'fedamw'])
def test_pipe_dropin_bitwise(amd, algo):
    """Through the drop-ins (the round plan, the deferred evaluation fused into the training
    launch, FedAMW's p-solve): fs_tuning.split_pipe = 1 gives bitwise the split form's results
    at a pipe-covered shape (D = 2048, C = 10, B = 32, parallel clients)."""
    tools = amd.tools
    rs = np.random.RandomState(13)
    N, D, C, R = 12, 2048, 10, 3
    sizes = list(rs.randint(20, 80, size=N))
    Xs, ys = _rand_clients(rs, sizes, D, C)
    Xt, yt = _rand_clients(rs, [300], D, C)
    Xv, yv = _rand_clients(rs, [160], D, C)
    X_train = [torch.from_numpy(x) for x in Xs]
    y_train = [torch.from_numpy(y) for y in ys]
    X_test, y_test = torch.from_numpy(Xt[0]), torch.from_numpy(yt[0])

    def run(pipe):
        with amd.lib.tuning(split_pipe=1 if pipe else -1, train_form=1):
            torch.manual_seed(4)
            if algo == 'fedavg':
                return tools.FedAvg(X_train, y_train, X_test, y_test, 'classification', C, D, 0.3, 2, 32,
                                    False, 0.1, False, 0.01, R, clients='parallel', verbose=False)
            vl = torch.utils.data.DataLoader(torch.utils.data.TensorDataset(torch.from_numpy(Xv[0]),
                                                                            torch.from_numpy(yv[0])),
                                             batch_size=16, shuffle=True)
            return tools.FedAMW(X_train, y_train, X_test, y_test, vl, 'classification', C, D, 0.3, 2, 32,
                                False, 0.1, True, 0.01, R, 1e-3, clients='parallel', verbose=False)

    a, b = run(True), run(False)
    for x, y in zip(a, b):
        assert torch.equal(x, y), (x, y)
