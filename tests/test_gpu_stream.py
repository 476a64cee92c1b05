"""The stream form of split-client local training (csrc/local_train_stream.hip, ABI 12,
fs_tuning.stream_form): four waves per workgroup, the batch rows in three rotating register
banks so the next step's rows stream during the forward and the hand-off.  It runs the split
form's arithmetic in the split form's order, so the two must agree BITWISE (weights, losses,
the fused evaluation) -- and the split form is pinned to the oracle and the reference fixtures
(test_gpu_parity.py).  Reference: train_loop, /root/reference/functions/tools.py:177-215,
parallel clients without the prox term (FedAvg; FedAMW's local training with ridge).
"""
import numpy as np
import pytest
import torch

from oracle import fedsim_oracle as O
from tests.test_gpu_parity import _rand_clients, _train_via_abi, amd  # noqa: F401 (fixture)

pytestmark = pytest.mark.gpu


def _both(amd, Xs, ys, W0, lr, E, B, reg, lam, G, seed):
    with amd.lib.tuning(stream_form=1):
        Ws, ls = _train_via_abi(amd, Xs, ys, W0, lr, E, B, False, 0.0, reg, lam, False, seed=seed, split=G)
    assert _train_via_abi.last_G == G
    with amd.lib.tuning(stream_form=-1):
        Wr, lr_ = _train_via_abi(amd, Xs, ys, W0, lr, E, B, False, 0.0, reg, lam, False, seed=seed, split=G)
    return Ws, ls, Wr, lr_


@pytest.mark.parametrize('G', [2, 4, 8, 16])
@pytest.mark.parametrize('reg', [False, True])
def test_stream_bitwise_equals_split(amd, G, reg):
    """Stream form == split form at width G, bitwise: D = 1024 G (full slices), C = 10, B = 32,
    ragged clients with tail batches of 1 and 7 rows, an empty client, more clients than groups
    at G = 16 (persistent groups walk several clients: W_start reloads at client starts)."""
    rs = np.random.RandomState(G + 31 * reg)
    D, C, B, E = 1024 * G, 10, 32, 2
    sizes = [65, 33, 0, 7, 96, 40, 1, 17, 64] + ([29] * 12 if G == 16 else [])
    Xs, ys = _rand_clients(rs, sizes, D, C)
    W0 = (rs.normal(size=(C, D)) * 0.1).astype(np.float32)
    Ws, ls, Wr, lr_ = _both(amd, Xs, ys, W0, 0.4, E, B, reg, 0.002, G, seed=3)
    assert np.array_equal(Ws, Wr), np.abs(Ws - Wr).max()
    assert np.array_equal(ls, lr_)


@pytest.mark.parametrize('C', [2, 7, 16])
def test_stream_classes(amd, C):
    """Other class counts (2, 7 and the widest, 16) at G = 2, ridge on: bitwise the split form,
    and the first client against the oracle."""
    rs = np.random.RandomState(100 + C)
    D, B, E, G = 2048, 32, 2, 2
    sizes = [70, 32, 5, 64]
    Xs, ys = _rand_clients(rs, sizes, D, C)
    W0 = (rs.normal(size=(C, D)) * 0.1).astype(np.float32)
    Ws, ls, Wr, lr_ = _both(amd, Xs, ys, W0, 0.4, E, B, True, 0.002, G, seed=8)
    assert np.array_equal(Ws, Wr) and np.array_equal(ls, lr_)
    torch.manual_seed(8)
    Wo, lo = O.train_client(Xs[0], ys[0], W0, 0.4, E, B, False, 0.0, True, 0.002)
    assert np.abs(Ws[0] - Wo).max() <= 2e-5 * max(1.0, np.abs(Wo).max())
    assert abs(ls[0] - lo) <= 2e-5 * max(1.0, abs(lo))


def test_stream_not_taken_outside_its_shapes(amd):
    """The stream form only takes parallel clients without a prox anchor on full slices with
    16 < B <= 32; anything else runs the split form unchanged (same results as stream off)."""
    rs = np.random.RandomState(7)
    for (D, B, prox) in ((2048, 16, False), (2048, 32, True), (1500, 32, False)):
        Xs, ys = _rand_clients(rs, [40, 33], D, 6)
        W0 = (rs.normal(size=(6, D)) * 0.1).astype(np.float32)
        with amd.lib.tuning(stream_form=1):
            Wa, la = _train_via_abi(amd, Xs, ys, W0, 0.3, 2, B, prox, 0.02, True, 0.001, False, seed=2, split=2)
        with amd.lib.tuning(stream_form=-1):
            Wb, lb = _train_via_abi(amd, Xs, ys, W0, 0.3, 2, B, prox, 0.02, True, 0.001, False, seed=2, split=2)
        assert np.array_equal(Wa, Wb) and np.array_equal(la, lb)


def test_stream_rounds_with_deferred_eval(amd):
    """Three FedAvg rounds through the round plan, the evaluation deferred into the next
    training launch (the stream kernel's fused evaluation blocks run the 8-wave evaluation body
    on 4 waves): every return and the global model bitwise equal with the stream form on and
    off."""
    from fedamw_amd import data as fdata
    from fedamw_amd.functions import tools
    dev = torch.device('cuda')
    out = {}
    for form in (1, -1):
        d = fdata.federated(24, 96, 2048, 10, 1000, shape='a9a', seed=5, device=dev)
        with amd.lib.tuning(stream_form=form):
            torch.manual_seed(4)
            stats = {'trace': True}
            res = tools.FedAvg(d['X_train'], d['y_train'], d['X_test'], d['y_test'], 'classification', 10, 2048, 0.5,
                               2, 32, False, 0.0, False, 0.0, 3, clients='parallel', stats=stats, verbose=False)
        out[form] = ([r.numpy() for r in res], stats['W_rounds'])
    for a, b in zip(out[1][0], out[-1][0]):
        assert np.array_equal(a, b), (a, b)
    assert np.array_equal(out[1][1], out[-1][1])
