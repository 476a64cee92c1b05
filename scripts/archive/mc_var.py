"""Diagnostic: run-to-run spread of the multi-CU p-solve at config 5's shape (GPU box)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fedamw_amd  # noqa: E402,F401
from fedamw_amd import _lib, engine, rng  # noqa: E402

N, C, nv, ep, D = 1000, 10, 12800, 2, 256
dev = torch.device('cuda')
g = torch.Generator().manual_seed(0)
Xv = torch.cos(torch.randn(nv, D, generator=g)) / D ** 0.5
yv = torch.randint(0, C, (nv,), generator=g)
mix = engine.Mixture(Xv, yv, D, C, N, 16, torch.full((N,), 1.0 / N), dev)
W = torch.randn(N, C, mix.f.ld, generator=g).to(dev) * 0.05
torch.manual_seed(1)
mix.solve(W, rng.draw_pass_seeds(ep), 1e-3)
steps = ep * ((nv + 15) // 16)
ts = []
for rep in range(12):
    torch.manual_seed(2 + rep)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    mix.prepare(rng.draw_pass_seeds(ep), 0)
    torch.cuda.synchronize()
    e0.record()
    mix.solve(None, None, 1e-3, slot=0, z=False)
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) * 1e3 / steps)
mix.check_errors()
print('us/step over %d launches: %s' % (len(ts), ' '.join('%.2f' % t for t in ts)), flush=True)
