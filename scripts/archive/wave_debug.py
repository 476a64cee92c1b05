"""Diagnostic: the one-wave p-solver after 1, 2, 3, 8 steps vs a numpy emulation (GPU box).

    python scripts/wave_debug.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fedamw_amd  # noqa: E402,F401
from fedamw_amd import _lib  # noqa: E402


def emulate(Z, yv, perms, N, C, nv, epochs, Bv, lr, mom, p0):
    ldN = (N + 3) & ~3
    nbat = (nv + Bv - 1) // Bv
    pr = np.zeros(16, np.float32)
    pr[:N] = p0
    br = np.zeros(16, np.float32)
    first = True
    for st in range(epochs * nbat):
        ep, sb = divmod(st, nbat)
        bc = min(Bv, nv - sb * Bv)
        gp = np.zeros(16, np.float32)
        for b in range(16):
            row = perms[ep * nv + sb * Bv + (b if b < bc else 0)]
            zs = []
            for c in range(4):
                cc = min(c, C - 1)
                z = np.concatenate([Z[row, cc * ldN + min(4 * k, ldN - 4):cc * ldN + min(4 * k, ldN - 4) + 4]
                                    for k in range(4)])
                zs.append(z)
            os_ = [float(np.dot(z, pr)) for z in zs]
            m = max(os_[c] for c in range(C))
            e = sum(np.exp(os_[c] - m) for c in range(C))
            for c in range(C):
                if b < bc:
                    g = (-1.0 / bc if c == yv[row] else 0.0) + np.exp(os_[c] - m - np.log(e)) / bc
                    gp += np.float32(g) * zs[c]
        br = (gp if first else mom * br + gp).astype(np.float32)
        pr = (pr - lr * br).astype(np.float32)
        pr[N:] = 0
        first = False
    return pr[:N], br[:N]


def main():
    dev = torch.device('cuda')
    rs = np.random.RandomState(3)
    N, C, Bv = 10, 2, 16
    ldN = (N + 3) & ~3
    for nv, ep in ((16, 1), (32, 1), (48, 1), (128, 1), (203, 2)):
        Z = np.zeros((nv, C * ldN), np.float32)
        for c in range(C):
            Z[:, c * ldN:c * ldN + N] = rs.normal(size=(nv, N)).astype(np.float32) * 0.3
        yv = rs.randint(0, C, size=nv).astype(np.int32)
        perms = np.concatenate([rs.permutation(nv) for _ in range(ep)]).astype(np.int32)
        p0 = np.full(N, 0.1, np.float32)
        pe, be = emulate(Z, yv, perms, N, C, nv, ep, Bv, 0.5, 0.9, p0)
        Zd, yd, pd = torch.from_numpy(Z).to(dev), torch.from_numpy(yv).to(dev), torch.from_numpy(perms).to(dev)
        p = torch.from_numpy(p0).to(dev)
        b = torch.zeros(N, device=dev)
        first = torch.ones(1, dtype=torch.int32, device=dev)
        ws = torch.zeros(_lib.lib().fs_mix_solve_ws_bytes(N, C, Bv), dtype=torch.uint8, device=dev)
        _lib.check(_lib.lib().fs_mix_solve(_lib.ptr(Zd), _lib.ptr(yd), _lib.ptr(pd), N, C, nv, ep, Bv, 0.5, 0.9,
                                           _lib.ptr(p), _lib.ptr(b), _lib.ptr(first), _lib.ptr(ws), ws.numel(),
                                           _lib.stream_ptr()), 'solve')
        torch.cuda.synchronize()
        pg = p.cpu().numpy()
        print('nv %d ep %d solver %s: max|dp| %.3g  max|db| %.3g' % (
            nv, ep, _lib.SOLVER_NAMES[_lib.lib().fs_mix_solve_last_mode()], np.abs(pg - pe).max(),
            np.abs(b.cpu().numpy() - be).max()), flush=True)
        if nv == 16:
            print('  gpu', pg, '\n  emu', pe, flush=True)


if __name__ == '__main__':
    main()
