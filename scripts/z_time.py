"""Diagnostic: fs_mix_z (the FedAMW Z GEMM) time and TFLOP/s at a shape, plus a sampled check
against fp64.   python scripts/z_time.py [N] [C] [D] [n_val] [reps]   (GPU box; default config 5)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fedamw_amd  # noqa: E402,F401
from fedamw_amd import _lib as L  # noqa: E402
a = [int(x) for x in sys.argv[1:]]
N, C, D, nv, reps = (a + [1000, 10, 16384, 32000, 5][len(a):])[:5]
dev = torch.device('cuda')
torch.manual_seed(0)
ld = (D + 63) // 64 * 64
X = torch.zeros(nv, ld, device=dev)
X[:, :D] = torch.randn(nv, D, device=dev).cos_().mul_(D ** -0.5)
W = torch.zeros(N, C, ld, device=dev)
W[:, :, :D] = torch.randn(N, C, D, device=dev) * 0.05
ldN = (N + 3) // 4 * 4
Z = torch.empty(nv, C * ldN, device=dev)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
st = L.stream_ptr()
L.check(L.lib().fs_mix_z(L.ptr(W), L.ptr(X), ld, N, C, nv, L.ptr(Z), st), 'z')
torch.cuda.synchronize()
ev[0].record()
for r in range(reps):
    L.check(L.lib().fs_mix_z(L.ptr(W), L.ptr(X), ld, N, C, nv, L.ptr(Z), st), 'z')
    ev[r + 1].record()
torch.cuda.synchronize()
ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(reps)]
fl = 2.0 * N * C * D * nv
best = min(ms)
print('mix_z N=%d C=%d D=%d n_val=%d: %s ms; best %.3f ms = %.1f TFLOP/s (%.1f %% of 157.3)'
      % (N, C, D, nv, ' '.join('%.3f' % m for m in ms), best, fl / best / 1e9, fl / best / 1e9 / 1.573), flush=True)
# sampled check: 256 random rows against fp64
rows = torch.randint(0, nv, (256,), device=dev)
ref = torch.einsum('vd,ncd->vcn', X[rows, :D].double(), W[:, :, :D].double())
got = Z[rows].view(-1, C, ldN)
err = (got[:, :, :N].double() - ref).abs().max().item()
scale = torch.einsum('vd,ncd->vcn', X[rows, :D].double().abs(), W[:, :, :D].double().abs()).max().item()
pad = got[:, :, N:].abs().max().item() if ldN > N else 0.0
print('  max |Z - Z64| = %.3e, max sum|x||w| = %.3e, ratio %.2e; padding max %.1f' % (err, scale, err / scale, pad),
      flush=True)
assert err <= 2e-6 * scale and pad == 0.0
