"""Diagnostic: fs_local_train launch time back to back vs after an idle gap (clock ramp).

    python scripts/lt_idle_gap.py --config 5 [--gap 0.5] [--reps 6]      (GPU box)

Times the planner's form at a BASELINE config shape (scripts/lt_sweep.py SHAPES) with HIP
events: first ``reps`` launches back to back, then ``reps`` launches each preceded by ``gap``
seconds with the GPU idle (host sleep after a synchronize)."""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fedamw_amd  # noqa: E402,F401
from fedamw_amd import data, engine, rng  # noqa: E402
from scripts.lt_sweep import SHAPES  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', type=int, default=5, choices=sorted(SHAPES))
    ap.add_argument('--gap', type=float, default=0.5)
    ap.add_argument('--reps', type=int, default=6)
    a = ap.parse_args()
    sh = SHAPES[a.config]
    dev = torch.device('cuda')
    N, D, C, E, B = sh['clients'], sh['D'], sh['C'], 2, 32
    d = data.federated(N, sh['rows'], D, C, 1000, shape=sh['shape'], device=dev)
    feats = engine.Features(d['X_train'], d['y_train'], D, dev)
    del d
    tr = engine.LocalTrainer(feats, C, B, E, chained=sh.get('chained', False))
    torch.manual_seed(0)
    tr.upload_perms(rng.draw_pass_seeds(N * E))
    W0 = torch.zeros(C, feats.ld, device=dev)
    W0.normal_(0, 0.01)

    def one():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        tr.run(W0, 0.5, False, 0.0, True, 1e-5, sh.get('chained', False))
        e1.record()
        return e0, e1
    for _ in range(3):
        one()
    torch.cuda.synchronize()
    bb = [one() for _ in range(a.reps)]
    torch.cuda.synchronize()
    gapped = []
    for _ in range(a.reps):
        torch.cuda.synchronize()
        time.sleep(a.gap)
        gapped.append(one())
    torch.cuda.synchronize()
    f = lambda ev: [x.elapsed_time(y) for x, y in ev]
    print('config %d: back to back %s ms; after %.2f s idle %s ms' % (
        a.config, np.round(f(bb), 3).tolist(), a.gap, np.round(f(gapped), 3).tolist()), flush=True)


if __name__ == '__main__':
    main()
