"""The team form of fs_local_train (csrc/local_train_split.hip TEAMS = 2, ABI 13: G | G_TEAMS).

Each workgroup's 8 waves are two teams of 4, training two clients at once with team-local
barriers.  Per client the arithmetic is the split form's with 4 waves per slice (each wave
accumulates two tiles' partial logits before the wave partials are summed), so it matches the
split form at the same width to fp32 summation-order noise and the oracle within the split
form's tolerance.  Reference: train_loop, /root/reference/functions/tools.py:177-215, parallel
clients.
"""
import numpy as np
import pytest
import torch

from oracle import fedsim_oracle as O
from tests.test_gpu_parity import _rand_clients, _train_via_abi, amd  # noqa: F401 (fixture)

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("mb_off")]


def _teams(amd, G):
    return G | amd.lib.G_TEAMS


@pytest.mark.parametrize('G', [4, 8])
@pytest.mark.parametrize('B', [32, 16])
@pytest.mark.parametrize('prox,reg', [(True, True), (False, False)])
def test_teams_match_split(amd, G, B, prox, reg):
    """Team form vs split form at width G: D = 512 G - 24 (the last tile ragged), C = 10, ragged
    clients incl. tail batches of 1 and 7 rows and an empty client, an odd client count (one
    team of a group ends early); every client also against the oracle."""
    rs = np.random.RandomState(G + B + 7 * prox + 100)
    D, C, E = 512 * G - 24, 10, 2
    sizes = [65, 33, 0, 7, 96, 40, 1, 17, 64]
    Xs, ys = _rand_clients(rs, sizes, D, C)
    W0 = (rs.normal(size=(C, D)) * 0.1).astype(np.float32)
    lr, mu, lam = 0.4, 0.03, 0.002
    Wt, lt = _train_via_abi(amd, Xs, ys, W0, lr, E, B, prox, mu, reg, lam, False, seed=5, split=_teams(amd, G))
    assert _train_via_abi.last_G == _teams(amd, G)
    Ws, ls = _train_via_abi(amd, Xs, ys, W0, lr, E, B, prox, mu, reg, lam, False, seed=5, split=G)
    assert np.abs(Wt - Ws).max() <= 1e-5 * max(1.0, np.abs(Ws).max()), np.abs(Wt - Ws).max()
    np.testing.assert_allclose(lt, ls, rtol=1e-5, atol=1e-6)
    torch.manual_seed(5)
    for j, (X, y) in enumerate(zip(Xs, ys)):
        Wr, lref = O.train_client(X, y, W0, lr, E, B, prox, mu, reg, lam)
        assert np.abs(Wt[j] - Wr).max() <= 2e-5 * max(1.0, np.abs(Wr).max()), (j, np.abs(Wt[j] - Wr).max())
        assert abs(lt[j] - lref) <= 2e-5 * max(1.0, abs(lref)), j


@pytest.mark.parametrize('N,G', [(301, 4), (700, 8)])
def test_teams_many_clients(amd, N, G):
    """More clients than lanes: each team walks several clients (LPT order, snake over the
    lanes), restarting from W_start; against the split form and a sample against the oracle."""
    rs = np.random.RandomState(N + 1)
    D, C, B, E = 512 * G, 6, 32, 2
    sizes = list(rs.randint(0, 90, size=N))
    Xs, ys = _rand_clients(rs, sizes, D, C)
    W0 = (rs.normal(size=(C, D)) * 0.1).astype(np.float32)
    args = (0.3, E, B, True, 0.02, True, 0.001, False)
    Wt, lt = _train_via_abi(amd, Xs, ys, W0, *args, seed=9, split=_teams(amd, G))
    Ws, ls = _train_via_abi(amd, Xs, ys, W0, *args, seed=9, split=G)
    assert np.abs(Wt - Ws).max() <= 1e-5 * max(1.0, np.abs(Ws).max())
    np.testing.assert_allclose(lt, ls, rtol=1e-5, atol=1e-6)
    torch.manual_seed(9)
    for j, (X, y) in enumerate(zip(Xs, ys)):
        if j % 97 == 0 or sizes[j] == 0:
            Wr, lref = O.train_client(X, y, W0, 0.3, E, B, True, 0.02, True, 0.001)
            assert np.abs(Wt[j] - Wr).max() <= 2e-5 * max(1.0, np.abs(Wr).max()), j
            assert abs(lt[j] - lref) <= 2e-5 * max(1.0, abs(lref)), j
        else:
            torch.empty(2 * E, dtype=torch.int64).random_()     # the oracle's draws for client j


def test_teams_planner(amd):
    """fs_local_train_plan: an explicit G | G_TEAMS request is granted for parallel clients at
    G = 4 or 8 where the slice fits; chained clients and other widths fall back;
    fs_tuning.split_teams = 1 picks the team form at the narrowest width that fits."""
    import ctypes
    L = amd.lib.lib()

    def plan(N, C, B, ld, chained, want=0):
        g, w = ctypes.c_int(want), ctypes.c_int64(0)
        amd.lib.check(L.fs_local_train_plan(N, C, B, 2, ld, 1024, chained, 0, ctypes.byref(g), ctypes.byref(w)),
                      'plan')
        return g.value, w.value

    T = amd.lib.G_TEAMS
    g, w = plan(100, 10, 32, 2048, 0, 4 | T)
    assert g == 4 | T and w > 0
    g, _ = plan(100, 10, 32, 2048, 1, 4 | T)
    assert not (g & T)                                    # chained: no team form
    g, _ = plan(100, 10, 32, 2048, 0, 2 | T)
    assert not (g & T)                                    # G = 2: no team instance
    with amd.lib.tuning(split_teams=1):
        g, _ = plan(100, 10, 32, 2048, 0)
        assert g == 4 | T
    with amd.lib.tuning(split_teams=-1):
        g, _ = plan(100, 10, 32, 2048, 0)
        assert not (g & T)
