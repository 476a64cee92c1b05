"""Diagnostic: host time of each native call of Federation.round() at config 2 (GPU box).
    python scripts/host_calls.py"""
import collections
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fedamw_amd  # noqa: E402,F401
from fedamw_amd import data  # noqa: E402
from fedamw_amd.functions import tools  # noqa: E402

dev = torch.device('cuda')
d = data.federated(100, 512, 2048, 10, 10000, device=dev)
torch.manual_seed(100)
R = 80
fed = tools.Federation('fedavg', d['X_train'], d['y_train'], d['X_test'], d['y_test'], None, 'classification', 10,
                       2048, 0.5, 2, 32, False, 0.0, False, 1e-5, R, 1e-3, 'parallel', verbose=False)
acc = collections.defaultdict(list)


def wrap(obj, name):
    fn = getattr(obj, name)

    def w(*a, **k):
        t = time.perf_counter()
        out = fn(*a, **k)
        acc['%s%s' % (name, '' if name != 'round' else '(phases=%d)' % a[2])].append(time.perf_counter() - t)
        return out
    setattr(obj, name, w)


for _ in range(5):
    fed.round()
torch.cuda.synchronize()
wrap(fed.plan, 'shuffle')
wrap(fed.plan, 'round')
t0 = time.perf_counter()
rt = []
for _ in range(60):
    a = time.perf_counter()
    fed.round()
    rt.append(time.perf_counter() - a)
torch.cuda.synchronize()
print('wall per round %.1f us; round() host mean %.1f us' % (1e6 * (time.perf_counter() - t0) / 60, 1e6 * np.mean(rt)))
for k, v in sorted(acc.items()):
    print('  %-22s n=%3d mean %7.1f us  median %7.1f  max %7.1f' % (k, len(v), 1e6 * np.mean(v), 1e6 * np.median(v),
                                                                    1e6 * np.max(v)))
