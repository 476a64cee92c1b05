"""Diagnostic: where the stream form and the split form differ (G, reg, lam from argv).
    python scripts/stream_diff.py G reg lam"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_gpu_parity import _rand_clients, _train_via_abi  # noqa: E402
import fedamw_amd  # noqa: E402,F401
from fedamw_amd import _lib, engine, rng  # noqa: E402

amd = type('amd', (), dict(lib=_lib, engine=engine, rng=rng))
G, reg, lam = int(sys.argv[1]), bool(int(sys.argv[2])), float(sys.argv[3])
rs = np.random.RandomState(G + 31 * reg)
D, C, B, E = 1024 * G, 10, 32, int(sys.argv[4]) if len(sys.argv) > 4 else 2
sizes = [65, 33, 0, 7, 96, 40, 1, 17, 64]
Xs, ys = _rand_clients(rs, sizes, D, C)
W0 = (rs.normal(size=(C, D)) * 0.1).astype(np.float32)
out = {}
for f in (1, -1):
    with _lib.tuning(stream_form=f):
        out[f] = _train_via_abi(amd, Xs, ys, W0, 0.4, E, B, False, 0.0, reg, lam, False, seed=3, split=G)
Ws, ls = out[1]
Wr, lr_ = out[-1]
bad = np.argwhere(Ws != Wr)
print('G=%d reg=%d lam=%g E=%d: %d of %d weights differ, max %.3g; losses equal %s' % (
    G, reg, lam, E, len(bad), Ws.size, np.abs(Ws - Wr).max(), np.array_equal(ls, lr_)))
if len(bad):
    cl = np.unique(bad[:, 0], return_counts=True)
    print('  by client', dict(zip(cl[0].tolist(), cl[1].tolist())))
    tiles = np.unique(bad[:, 2] // 64, return_counts=True)
    print('  by 64-col tile', dict(zip(tiles[0].tolist(), tiles[1].tolist())))
    print('  by class', np.unique(bad[:, 1]).tolist())
    print('  loss diff', (ls - lr_).tolist())
