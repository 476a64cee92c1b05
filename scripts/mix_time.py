"""Diagnostic: fs_mix_solve time per dependent p-SGD step (and fs_mix_z) at a given shape.
    [FS_MIX_SOLVER=name] [FS_MIX_EXACT=1] [FS_MIX_PF_H=h] [FS_MIX_PF_LEAD=l] [FS_MIX_QMC_LC=4|8] [FS_MIX_QUAD_LOADERS=-1] [FS_MIX_POLL_DELAY=n]
    [FS_MIX_DUMP=file.npy (p and buf after the run, for bitwise A/B of two builds)] python scripts/mix_time.py
        [N] [C] [n_val] [epochs] [D]
(GPU box; default config 2; the variables only select fs_tuning fields for this run)"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fedamw_amd  # noqa: E402,F401
from fedamw_amd import engine, rng  # noqa: E402

SOLVER = os.environ.get('FS_MIX_SOLVER', 'auto')
fedamw_amd._lib.set_tuning(mix_solver=SOLVER, mix_exact_softmax=int(os.environ.get('FS_MIX_EXACT', '0')),
                           mix_prefetch=int(os.environ.get('FS_MIX_PF_H', '0')),
                           mix_prefetch_lead=int(os.environ.get('FS_MIX_PF_LEAD', '0')),
                           mix_qmc_lane_clients=int(os.environ.get('FS_MIX_QMC_LC', '0')),
                           mix_quad_loaders=int(os.environ.get('FS_MIX_QUAD_LOADERS', '0')),
                           mix_poll_delay=int(os.environ.get('FS_MIX_POLL_DELAY', '0')))
a = [int(x) for x in sys.argv[1:]]
N, C, nv, ep, D = (a + [100, 10, 12800, 10, 2048][len(a):])[:5]
dev = torch.device('cuda')
g = torch.Generator().manual_seed(0)
Xv = torch.cos(torch.randn(nv, D, generator=g)) / D ** 0.5
yv = torch.randint(0, C, (nv,), generator=g)
p0 = torch.full((N,), 1.0 / N)
mix = engine.Mixture(Xv, yv, D, C, N, 16, p0, dev)
STAMPS = os.environ.get('FEDSIM_LIB', '').endswith('stamps.so')
if STAMPS:                       # room after buf[N] for the stamp build's phase counters
    mix.buf = torch.zeros(N + 64, dtype=torch.float32, device=dev)
W = torch.randn(N, C, mix.f.ld, generator=g).to(dev) * 0.05
torch.manual_seed(1)
mix.solve(W, rng.draw_pass_seeds(1), 1e-3)
torch.cuda.synchronize()
L = fedamw_amd._lib
ts = []
for rep in range(3):
    mix.prepare(rng.draw_pass_seeds(ep), 0)
    perms = mix.shuffler.acquire(0)
    torch.cuda.synchronize()
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    e0.record()
    L.check(L.lib().fs_mix_z(L.ptr(W), L.ptr(mix.f.phi), mix.f.ld, N, C, nv, L.ptr(mix.Z), L.stream_ptr()), 'z')
    e1.record()
    L.check(L.lib().fs_mix_solve(L.ptr(mix.Z), L.ptr(mix.f.labels), L.ptr(perms), N, C, nv, ep, 16, 1e-3, 0.9,
                                 L.ptr(mix.p), L.ptr(mix.buf), L.ptr(mix.first), L.ptr(mix.ws), mix.ws.numel(),
                                 L.stream_ptr()), 'solve')
    e2.record()
    torch.cuda.synchronize()
    ts.append((e0.elapsed_time(e1), e1.elapsed_time(e2)))
steps = ep * ((nv + 15) // 16)
zms, sms = ts[-1]
print('N=%d C=%d n_val=%d epochs=%d: mix_z %.1f us (%.1f TFLOP/s), mix_solve %.2f ms = %.3f us/step over %d steps; '
      'p finite: %s' % (N, C, nv, ep, zms * 1e3, 2.0 * N * C * D * nv / zms / 1e9, sms, sms * 1e3 / steps, steps,
                        bool(torch.isfinite(mix.p).all())), flush=True)
mix.check_errors()
if os.environ.get('FS_MIX_DUMP'):
    np.save(os.environ['FS_MIX_DUMP'], np.stack([mix.p[:N].cpu().numpy(), mix.buf[:N].cpu().numpy()]))
print('  solver requested %s, ran %s' % (SOLVER,
                                         L.SOLVER_NAMES[L.lib().fs_mix_solve_last_mode()]), flush=True)
if STAMPS:
    acc = mix.buf[N + 8:N + 20].cpu().numpy().view(np.uint64)
    ran = L.SOLVER_NAMES[L.lib().fs_mix_solve_last_mode()]
    names = {'quad': ['wait+logits', 'rs+softmax+grad', 'fold', 'barrier', 'update+gather', 'issue'],
             'qmc': ['wait ring+logits+rs', 'hop (publish+polls)', 'late issue+softmax+grad', 'issue+fold+lds',
                     'barrier', 'update+gather']}.get(ran, ['wait ring', 'logits+softmax+grad', 'gpart+issue',
                                                           'barrier', 'update'])
    print('wave-0 s_memtime ticks per step (last call): ' +
          ', '.join('%s %.0f' % (nm, a / steps) for nm, a in zip(names, acc)), flush=True)
