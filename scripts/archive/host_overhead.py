"""Diagnostic: host-side cost of Federation.round() at config 2 (GPU box)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fedamw_amd  # noqa: E402,F401
from fedamw_amd import data  # noqa: E402
from fedamw_amd.functions import tools  # noqa: E402

dev = torch.device('cuda')
d = data.federated(100, 512, 2048, 10, 10000, device=dev)
torch.manual_seed(100)
R = 60
fed = tools.Federation('fedavg', d['X_train'], d['y_train'], d['X_test'], d['y_test'], None, 'classification', 10,
                       2048, 0.5, 2, 32, False, 0.0, False, 1e-5, R, 1e-3, 'parallel', verbose=False)
for _ in range(5):
    fed.round()
torch.cuda.synchronize()
# host-only cost: time to ENQUEUE rounds (the GPU queue absorbs them)
t0 = time.perf_counter()
n = 0
times = []
for _ in range(30):
    a = time.perf_counter()
    fed.round()
    times.append(time.perf_counter() - a)
    n += 1
enq = time.perf_counter() - t0
torch.cuda.synchronize()
tot = time.perf_counter() - t0
times.sort()
print('per round: enqueue %.1f us (median %.1f, max %.1f), wall incl. drain %.1f us' %
      (1e6 * enq / n, 1e6 * times[len(times) // 2], 1e6 * times[-1], 1e6 * tot / n))
import cProfile, pstats
pr = cProfile.Profile()
pr.enable()
for _ in range(10):
    fed.round()
pr.disable()
torch.cuda.synchronize()
pstats.Stats(pr).sort_stats('tottime').print_stats(12)
