"""The pair-client form of fs_local_train (csrc/local_train_pair.hip, since ABI 10).

A group of G workgroups trains two clients at a time, interleaved; per step it runs the
split form's arithmetic at the same width in the same order, so the two forms must agree
BITWISE (weights and losses) on every shape -- and the split form is itself pinned to the
oracle and the reference fixtures (test_gpu_parity.py).  Reference: train_loop,
/root/reference/functions/tools.py:177-215, parallel clients.
"""
import numpy as np
import pytest
import torch

from oracle import fedsim_oracle as O
from tests.test_gpu_parity import _rand_clients, _train_via_abi, amd  # noqa: F401 (fixture)

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("mb_off")]


def _pair(amd, G):
    return G | amd.lib.G_PAIR


@pytest.mark.parametrize('G', [2, 4, 8, 16])
@pytest.mark.parametrize('B', [32, 16])
@pytest.mark.parametrize('prox,reg', [(True, True), (False, False)])
def test_pair_bitwise_equals_split(amd, G, B, prox, reg):
    """Pair form == split form at width G, bitwise: D = 512 G - 24 (the last tile ragged, padded
    columns stay 0), C = 10, ragged clients incl. tail batches of 1 and 7 rows and an empty
    client, an odd client count (one lane of a group ends early)."""
    rs = np.random.RandomState(G + B + 7 * prox)
    D, C, E = 512 * G - 24, 10, 2
    sizes = [65, 33, 0, 7, 96, 40, 1, 17, 64]
    Xs, ys = _rand_clients(rs, sizes, D, C)
    W0 = (rs.normal(size=(C, D)) * 0.1).astype(np.float32)
    lr, mu, lam = 0.4, 0.03, 0.002
    Wp, lp = _train_via_abi(amd, Xs, ys, W0, lr, E, B, prox, mu, reg, lam, False, seed=3, split=_pair(amd, G))
    assert _train_via_abi.last_G == _pair(amd, G)
    Ws, ls = _train_via_abi(amd, Xs, ys, W0, lr, E, B, prox, mu, reg, lam, False, seed=3, split=G)
    assert np.array_equal(Wp, Ws), np.abs(Wp - Ws).max()
    assert np.array_equal(lp, ls)


@pytest.mark.parametrize('N,G', [(301, 2), (700, 4), (1000, 8)])
def test_pair_many_clients(amd, N, G):
    """More clients than lanes: every lane walks several clients (LPT order, snake over the
    lanes), the next client's first rows streaming in during the previous client's last
    step; a lane's clients restart from W_start.  Bitwise the split form; a sample of clients
    against the oracle."""
    rs = np.random.RandomState(N)
    D, C, B, E = 512 * G, 6, 32, 2
    sizes = list(rs.randint(0, 90, size=N))
    Xs, ys = _rand_clients(rs, sizes, D, C)
    W0 = (rs.normal(size=(C, D)) * 0.1).astype(np.float32)
    args = (0.3, E, B, True, 0.02, True, 0.001, False)
    Wp, lp = _train_via_abi(amd, Xs, ys, W0, *args, seed=9, split=_pair(amd, G))
    Ws, ls = _train_via_abi(amd, Xs, ys, W0, *args, seed=9, split=G)
    assert np.array_equal(Wp, Ws) and np.array_equal(lp, ls)
    torch.manual_seed(9)
    for j, (X, y) in enumerate(zip(Xs, ys)):
        if j % 97 == 0 or sizes[j] == 0:
            Wr, lref = O.train_client(X, y, W0, 0.3, E, B, True, 0.02, True, 0.001)
            assert np.abs(Wp[j] - Wr).max() <= 2e-5 * max(1.0, np.abs(Wr).max()), j
            assert abs(lp[j] - lref) <= 2e-5 * max(1.0, abs(lref)), j
        else:
            torch.empty(2 * E, dtype=torch.int64).random_()     # the oracle's draws for client j


def test_pair_vs_oracle_benchmark_width(amd):
    """The pair form at config 2's width (D = 2048, C = 10, B = 32, G = 4), every client against
    the oracle (FedProx + ridge)."""
    rs = np.random.RandomState(21)
    D, C, B, E = 2048, 10, 32, 2
    sizes = [512, 100, 33, 1, 64]
    Xs, ys = _rand_clients(rs, sizes, D, C)
    W0 = (rs.normal(size=(C, D)) * 0.1).astype(np.float32)
    lr, mu, lam = 0.4, 0.03, 0.002
    W, loss = _train_via_abi(amd, Xs, ys, W0, lr, E, B, True, mu, True, lam, False, seed=11, split=_pair(amd, 4))
    assert _train_via_abi.last_G == _pair(amd, 4)
    torch.manual_seed(11)
    for j, (X, y) in enumerate(zip(Xs, ys)):
        Wr, lref = O.train_client(X, y, W0, lr, E, B, True, mu, True, lam)
        assert np.abs(W[j] - Wr).max() <= 2e-5 * max(1.0, np.abs(Wr).max()), (j, np.abs(W[j] - Wr).max())
        assert abs(loss[j] - lref) <= 2e-5 * max(1.0, abs(lref))


def test_pair_planner_and_train_form(amd):
    """fs_local_train_plan: parallel clients at ld == 512 G get the pair form when its groups
    walk several clients each (else the split form, which measured faster with one client per
    group); chained clients and other widths the split form; fs_tuning.train_form = 1 turns
    the pair form off, 2 asks for it wherever it fits."""
    import ctypes
    L = amd.lib.lib()

    def plan(N, C, B, ld, chained, want=0, prox=0):
        g, w = ctypes.c_int(want), ctypes.c_int64(0)
        amd.lib.check(L.fs_local_train_plan(N, C, B, 2, ld, 1024, chained, prox, ctypes.byref(g), ctypes.byref(w)),
                      'plan')
        return g.value, w.value

    P = amd.lib.G_PAIR
    assert plan(100, 10, 32, 2048, 0)[0] == 2                        # config 2: one client per group
    assert plan(1250, 10, 32, 2048, 0)[0] == 2 | amd.lib.G_PIPE      # config 4: the pipe form (ABI 14)
    with amd.lib.tuning(split_pipe=-1):
        assert plan(1250, 10, 32, 2048, 0)[0] == 4 | P               # ... the pair form without it
    assert plan(1000, 7, 32, 4096, 0, prox=1)[0] == 4                # config 3 (FedProx: the split form, r05)
    with amd.lib.tuning(train_form=2):
        assert plan(1000, 7, 32, 4096, 0, prox=1)[0] == 8 | P        # ... the pair form when asked for
    assert plan(1000, 7, 32, 4096, 0)[0] == 4 | amd.lib.G_PIPE       # ... its shape without the prox term
    assert plan(300, 10, 32, 1024, 0)[0] == 2 | P
    with amd.lib.tuning(train_form=2):
        assert plan(100, 10, 32, 2048, 0)[0] == 4 | P
    assert plan(10, 2, 32, 2048, 1)[0] in (2, 4, 8, 16)             # chained: split form
    assert plan(1000, 10, 32, 16384, 0)[0] == 16                     # ld > 512 * 16: split form
    assert plan(100, 10, 32, 2048, 0, want=2)[0] == 2                # explicit split width
    with amd.lib.tuning(train_form=1):
        assert plan(1250, 10, 32, 2048, 0)[0] == 2
    g, ws = plan(100, 10, 32, 2048, 0, want=4 | P)
    assert g == 4 | P and ws > amd.lib.ERR_BLOCK


@pytest.mark.parametrize('G', [2, 4])
@pytest.mark.parametrize('B', [32, 16])
def test_pair_c14_boundary(amd, G, B):
    """C = 14, the widest the pair form takes: the last real class (13) sits beside the two
    granules that carry ||W - W_a||^2 and ||W||^2 (row 0, classes 14 and 15), with the prox and
    ridge terms on (both norms read).  Bitwise the split form, a client against the oracle; the
    planner never gives the pair form at C = 15 (not even when asked for it)."""
    import ctypes
    rs = np.random.RandomState(140 + G + B)
    D, C, E = 512 * G, 14, 2
    sizes = [70, 33, 1, 64, 17]
    Xs, ys = _rand_clients(rs, sizes, D, C)
    W0 = (rs.normal(size=(C, D)) * 0.1).astype(np.float32)
    lr, mu, lam = 0.4, 0.03, 0.002
    Wp, lp = _train_via_abi(amd, Xs, ys, W0, lr, E, B, True, mu, True, lam, False, seed=5, split=_pair(amd, G))
    assert _train_via_abi.last_G == _pair(amd, G)
    Ws, ls = _train_via_abi(amd, Xs, ys, W0, lr, E, B, True, mu, True, lam, False, seed=5, split=G)
    assert np.array_equal(Wp, Ws), np.abs(Wp - Ws).max()
    assert np.array_equal(lp, ls)
    torch.manual_seed(5)
    Wr, lref = O.train_client(Xs[0], ys[0], W0, lr, E, B, True, mu, True, lam)
    assert np.abs(Wp[0] - Wr).max() <= 2e-5 * max(1.0, np.abs(Wr).max())
    assert abs(lp[0] - lref) <= 2e-5 * max(1.0, abs(lref))
    L = amd.lib.lib()
    for want in (0, _pair(amd, G)):
        g, w = ctypes.c_int(want), ctypes.c_int64(0)
        amd.lib.check(L.fs_local_train_plan(1250, 15, B, 2, D, 1024, 0, 1, ctypes.byref(g), ctypes.byref(w)), 'plan')
        assert not (g.value & amd.lib.G_PAIR), (want, g.value)


def test_pair_handoff_timeout_raises(amd):
    """fs_tuning.inject_timeout: the pair launch reports a timeout through its workspace error
    word; check_errors raises and clears it, and the next launch is clean."""
    rs = np.random.RandomState(1)
    Xs, ys = _rand_clients(rs, [40, 70, 9], 1024, 4)
    W0 = (rs.normal(size=(4, 1024)) * 0.1).astype(np.float32)
    G = _pair(amd, 2)
    with amd.lib.tuning(inject_timeout=1):
        with pytest.raises(amd.lib.FedsimError, match='timed out'):
            _train_via_abi(amd, Xs, ys, W0, 0.3, 2, 32, False, 0.0, False, 0.0, False, seed=1, split=G)
    _train_via_abi(amd, Xs, ys, W0, 0.3, 2, 32, False, 0.0, False, 0.0, False, seed=1, split=G)


def test_pair_repeated_launches_generation_tags(amd):
    """Back-to-back launches on one workspace (generation-tagged hand-offs, no clearing between
    launches) give the same bits every time."""
    rs = np.random.RandomState(4)
    D, C, B, E = 1024, 10, 32, 2
    sizes = list(rs.randint(1, 80, size=40))
    Xs, ys = _rand_clients(rs, sizes, D, C)
    dev = torch.device('cuda')
    feats = amd.engine.Features([torch.from_numpy(x) for x in Xs], [torch.from_numpy(y) for y in ys], D, dev)
    tr = amd.engine.LocalTrainer(feats, C, B, E, split=_pair(amd, 2))
    torch.manual_seed(2)
    tr.upload_perms(amd.rng.draw_pass_seeds(len(Xs) * E))
    Wg = torch.zeros(C, feats.ld, device=dev)
    Wg[:, :D] = torch.from_numpy((rs.normal(size=(C, D)) * 0.1).astype(np.float32))
    outs = []
    for _ in range(5):
        W, loss = tr.run(Wg, 0.3, True, 0.01, False, 0.0, False)
        outs.append((W.clone(), loss.clone()))
    torch.cuda.synchronize()
    tr.check_errors()
    for W, loss in outs[1:]:
        assert torch.equal(W, outs[0][0]) and torch.equal(loss, outs[0][1])
