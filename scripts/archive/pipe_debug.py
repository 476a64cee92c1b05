"""Diagnostic: per-client differences between the pipe and split forms (ridge on)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fedamw_amd  # noqa: E402,F401
from fedamw_amd import _lib, engine, rng  # noqa: E402
from tests.test_gpu_parity import _rand_clients, _train_via_abi  # noqa: E402

amd = type('amd', (), dict(lib=_lib, engine=engine, rng=rng))
for sizes, reg, lam, chained in [([65, 33, 0, 7, 96, 40, 1, 17, 64], True, 0.002, False), ([65], True, 0.002, False),
                                 ([32], True, 0.002, False), ([32, 32], True, 0.002, False),
                                 ([65], True, 0.0, False), ([65, 33], True, 0.002, True)]:
    rs = np.random.RandomState(1)
    G, C, B, D = 2, 10, 32, 2024
    Xs, ys = _rand_clients(rs, sizes, D, C)
    W0 = (rs.normal(size=(C, D)) * 0.1).astype(np.float32)
    Wp, lp = _train_via_abi(amd, Xs, ys, W0, 0.4, 2, B, False, 0.0, reg, lam, chained, seed=3, split=G | _lib.G_PIPE)
    Ws, ls = _train_via_abi(amd, Xs, ys, W0, 0.4, 2, B, False, 0.0, reg, lam, chained, seed=3, split=G)
    print(sizes, 'lam', lam, 'chained', chained, 'W diff per client', [float(np.abs(a - b).max()) for a, b in zip(Wp, Ws)],
          'loss diff', (lp - ls).tolist(), flush=True)
    for E in (1,):
        Wp, lp = _train_via_abi(amd, Xs, ys, W0, 0.4, E, B, False, 0.0, reg, lam, chained, seed=3, split=G | _lib.G_PIPE)
        Ws, ls = _train_via_abi(amd, Xs, ys, W0, 0.4, E, B, False, 0.0, reg, lam, chained, seed=3, split=G)
        print('  E=1', [float(np.abs(a - b).max()) for a, b in zip(Wp, Ws)], (lp - ls).tolist(), flush=True)

# determinism: each form against itself
rs = np.random.RandomState(1)
sizes = [65, 33, 0, 7, 96, 40, 1, 17, 64]
Xs, ys = _rand_clients(rs, sizes, 2024, 10)
W0 = (rs.normal(size=(10, 2024)) * 0.1).astype(np.float32)
for form, sp in (('pipe', 2 | _lib.G_PIPE), ('split', 2)):
    ref = None
    for k in range(4):
        W, l = _train_via_abi(amd, Xs, ys, W0, 0.4, 2, 32, False, 0.0, True, 0.002, False, seed=3, split=sp)
        if ref is None:
            ref = (W, l)
        else:
            print(form, 'repeat', k, 'W diff per client', [float(np.abs(a - b).max()) for a, b in zip(W, ref[0])],
                  flush=True)
