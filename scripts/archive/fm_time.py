"""Diagnostic: fs_feature_map time at the configs' shapes (GPU box).
    python scripts/fm_time.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fedamw_amd  # noqa: E402,F401
from fedamw_amd import engine  # noqa: E402

for name, n, d, D in (('config 1 (a9a train)', 32561, 123, 2000), ('config 2 (a9a, 100 x 640 rows)', 64000, 123, 2048),
                      ('config 3 (covtype pool)', 581012, 54, 4096), ('config 5 (a9a, 1000 x 160 rows)', 160000, 123, 16384)):
    g = torch.Generator().manual_seed(0)
    X = (torch.rand(n, d, generator=g) < 0.12).float().cuda()
    W = (torch.randn(d, D, generator=g) * 0.1).cuda()
    b = (torch.rand(1, D, generator=g) * 6.28).cuda()
    ldo = engine.pad_ld(D)
    out = torch.empty(n, ldo, device='cuda')
    engine.feature_map(X, W, b, D, out=out, ldo=ldo)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 5
    e0.record()
    for _ in range(reps):
        engine.feature_map(X, W, b, D, out=out, ldo=ldo)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    by = 4.0 * n * ldo + 4.0 * n * d + 4.0 * d * D
    fl = 2.0 * n * d * D
    print('%-32s n=%d d=%d D=%d: %.3f ms  %.0f GB/s (%.1f%% of 8 TB/s)  %.1f TFLOP/s (%.1f%% of 157.3)'
          % (name, n, d, D, ms, by / ms / 1e6, by / ms / 1e6 / 80, fl / ms / 1e9, fl / ms / 1e9 / 1.573), flush=True)
    del X, W, b, out
