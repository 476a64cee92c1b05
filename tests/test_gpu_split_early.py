"""The split form's early row issue (csrc/local_train_split.hip, ABI 11 fs_tuning.split_early).

On full slices (FedAvg, FedAMW's local training; since round 5 FedProx too) each wave issues the first
SP_E1 of its next-step row loads right after the hand-off, so they stream through the softmax
instead of waiting for the backward.  Only the time a load is issued moves: the weights and
losses must be BITWISE those of the late form (split_early = -1), which is itself pinned to the
oracle and the reference fixtures (test_gpu_parity.py).  Reference: train_loop,
/root/reference/functions/tools.py:177-215.
"""
import numpy as np
import pytest
import torch

from oracle import fedsim_oracle as O
from tests.test_gpu_parity import _rand_clients, _train_via_abi, amd  # noqa: F401 (fixture)

pytestmark = pytest.mark.gpu


def _both(amd, Xs, ys, W0, args, seed, G):
    out = []
    for early in (0, -1):
        with amd.lib.tuning(split_early=early):
            out.append(_train_via_abi(amd, Xs, ys, W0, *args, seed=seed, split=G))
            assert _train_via_abi.last_G == G
    return out


@pytest.mark.parametrize('G', [2, 4, 8, 16])
@pytest.mark.parametrize('B', [32, 16])
@pytest.mark.parametrize('chained', [False, True])
@pytest.mark.parametrize('prox', [False, True])
def test_split_early_bitwise(amd, G, B, chained, prox):
    """Early == late issue, bitwise, on full slices (D = 1024 G - 24: the last tile ragged, its
    padded columns stay 0), ridge on, ragged clients incl. tail batches of 1 and 7 rows and an
    empty client; chained clients carry the weights (and the row stream) across clients.  With
    the prox term (round 5) the early form loads the anchor's whole slice ahead of its early rows
    (W_start, or in a chain the previous client's result)."""
    rs = np.random.RandomState(G + B + 31 * chained + 7 * prox)
    D, C, E = 1024 * G - 24, 7 if prox else 10, 2
    sizes = [65, 33, 0, 7, 96, 1, 40]
    Xs, ys = _rand_clients(rs, sizes, D, C)
    W0 = (rs.normal(size=(C, D)) * 0.1).astype(np.float32)
    args = (0.4, E, B, prox, 0.05 if prox else 0.0, True, 0.002, chained)
    (We, le), (Wl, ll) = _both(amd, Xs, ys, W0, args, 5, G)
    assert np.array_equal(We, Wl), np.abs(We - Wl).max()
    assert np.array_equal(le, ll)


def test_split_early_persistent_groups_vs_oracle(amd):
    """More clients than groups (N = 300 at G = 2: 128 groups walk 2-3 clients each, the next
    client's first rows issued early inside the previous client's last step): bitwise the late
    form; a sample of clients against the oracle."""
    rs = np.random.RandomState(300)
    D, C, B, E, G = 2048, 10, 32, 2, 2
    sizes = list(rs.randint(0, 70, size=300))
    Xs, ys = _rand_clients(rs, sizes, D, C)
    W0 = (rs.normal(size=(C, D)) * 0.1).astype(np.float32)
    args = (0.3, E, B, False, 0.0, False, 0.0, False)
    (We, le), (Wl, ll) = _both(amd, Xs, ys, W0, args, 8, G)
    assert np.array_equal(We, Wl) and np.array_equal(le, ll)
    torch.manual_seed(8)
    for j, (X, y) in enumerate(zip(Xs, ys)):
        if j % 61 == 0 or sizes[j] == 0:
            Wr, lref = O.train_client(X, y, W0, 0.3, E, B, False, 0.0, False, 0.0)
            assert np.abs(We[j] - Wr).max() <= 2e-5 * max(1.0, np.abs(Wr).max()), j
            assert abs(le[j] - lref) <= 2e-5 * max(1.0, abs(lref)), j
        else:
            torch.empty(2 * E, dtype=torch.int64).random_()     # the oracle's draws for client j


@pytest.mark.parametrize('G', [4, 8, 16])
@pytest.mark.parametrize('per', [4, 8])
@pytest.mark.parametrize('prox', [False, True])
def test_split_narrow_chained_bitwise(amd, G, per, prox):
    """The narrow chained instances (round 5, session 2): slices of exactly ``per`` tiles, one tile
    per wave -- 4-wave workgroups at 4 tiles (exp.py's config 1: D = 2000 at G = 8), 8 waves at 8
    -- with every next-step row load early.  Same weights, bitwise, as the late 8-wave form
    (split_early = -1), whose waves 4-7 hold no tile at 4 tiles per slice; the losses too, up to the
    order of the cross-entropy partials (4 waves sum 2 rows each where 8 sum one)."""
    rs = np.random.RandomState(7 * G + per + 3 * prox)
    D, C, E, B = 64 * per * G - 24, 7 if prox else 2, 2, 32
    sizes = [65, 33, 0, 7, 96, 1, 40]
    Xs, ys = _rand_clients(rs, sizes, D, C)
    W0 = (rs.normal(size=(C, D)) * 0.1).astype(np.float32)
    args = (0.4, E, B, prox, 0.05 if prox else 0.0, True, 0.002, True)
    (We, le), (Wl, ll) = _both(amd, Xs, ys, W0, args, 11, G)
    assert np.array_equal(We, Wl), np.abs(We - Wl).max()
    assert np.allclose(le, ll, rtol=1e-6, atol=0), np.abs(le - ll).max()
