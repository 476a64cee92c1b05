"""Diagnostic: mean fs_local_train launch time at config 2 for each split choice.
    python scripts/lt_time.py [N] [splits...]     (GPU box)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fedamw_amd  # noqa: E402,F401
from fedamw_amd import data, engine, rng  # noqa: E402

dev = torch.device('cuda')
N = int(sys.argv[1]) if len(sys.argv) > 1 else 100
splits = [int(a) for a in sys.argv[2:]] or [None]
D, C, E, B = 2048, 10, 2, 32
d = data.federated(N, 512, D, C, 1000, device=dev)
feats = engine.Features(d['X_train'], d['y_train'], D, dev)
alg = 4.0 * E * feats.rows * D + 8.0 * E * feats.rows + 8.0 * N * C * D
for sp in splits:
    tr = engine.LocalTrainer(feats, C, B, E, split=sp)
    if os.environ.get('FEDSIM_LIB', '').endswith('stamps.so'):
        tr.ws = torch.zeros(tr.ws.numel() + N * tr.G * 16 * 8, dtype=torch.uint8, device=dev)
    torch.manual_seed(0)
    tr.upload_perms(rng.draw_pass_seeds(N * E))
    W0 = torch.zeros(C, feats.ld, device=dev)
    for _ in range(3):
        tr.run(W0, 0.5, False, 0, False, 0, False)
    torch.cuda.synchronize()
    ts = []
    for _ in range(20):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        tr.run(W0, 0.5, False, 0, False, 0, False)
        b.record()
        ts.append((a, b))
    torch.cuda.synchronize()
    tr.check_errors()
    ms = sum(a.elapsed_time(b) for a, b in ts) / len(ts)
    print('split=%s G=%d: %.1f us/launch, %.0f GB/s algorithmic' % (sp, tr.G, ms * 1e3, alg / ms / 1e6), flush=True)
