"""Diagnostic: event-timed fs_aggregate at a shape, the automatic form (chunks = 0) against
explicit chunk counts (the two-launch fold).      python scripts/agg_time.py [N] [C] [D]  (GPU box)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fedamw_amd  # noqa: E402,F401
from fedamw_amd import engine  # noqa: E402

a = [int(x) for x in sys.argv[1:]]
N, C, D = (a + [100, 10, 2048][len(a):])[:3]
dev = torch.device('cuda')
W = torch.randn(N, C, D, device=dev)
p = torch.rand(N, device=dev)
p /= p.sum()
out = torch.empty(C, D, device=dev)
for chunks in (0, 4, 8, 12, 16, 32):
    if chunks > N:
        continue
    agg = engine.Aggregator(N, C, D, dev, chunks=chunks)
    for _ in range(5):
        agg.run(W, p, out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 200
    e0.record()
    for _ in range(reps):
        agg.run(W, p, out)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    print('N=%d C=%d D=%d chunks=%-3d %7.2f us per call (%.0f GB/s)' % (N, C, D, chunks, us,
                                                                          4.0 * N * C * D / us / 1e3), flush=True)
