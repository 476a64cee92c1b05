"""Diagnostic: fs_local_train launch time at a BASELINE config shape under fs_tuning overrides.

    python scripts/lt_tuning_sweep.py --config 2 --field split_poll_delay --values -1,2,4,8   (GPU box)

Event-timed mean of --reps launches of the planner's form after 3 warm-up launches, one line per value."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fedamw_amd  # noqa: E402,F401
import fedamw_amd._lib as L  # noqa: E402
from fedamw_amd import data, engine, rng  # noqa: E402
from scripts.lt_sweep import SHAPES  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', type=int, default=2, choices=sorted(SHAPES))
    ap.add_argument('--field', default='split_poll_delay')
    ap.add_argument('--values', default='-1,2,4,8')
    ap.add_argument('--reps', type=int, default=20)
    a = ap.parse_args()
    sh = SHAPES[a.config]
    dev = torch.device('cuda')
    N, D, C, E, B = sh['clients'], sh['D'], sh['C'], 2, 32
    d = data.federated(N, sh['rows'], D, C, 1000, shape=sh['shape'], device=dev)
    feats = engine.Features(d['X_train'], d['y_train'], D, dev)
    del d
    ch = sh.get('chained', False)
    tr = engine.LocalTrainer(feats, C, B, E, chained=ch)
    torch.manual_seed(0)
    tr.upload_perms(rng.draw_pass_seeds(N * E))
    W0 = torch.zeros(C, feats.ld, device=dev)
    W0.normal_(0, 0.01)
    alg = 4.0 * E * feats.rows * D + 8.0 * E * feats.rows + 8.0 * N * C * D
    for v in [int(x) for x in a.values.split(',')]:
        with L.tuning(**{a.field: v}):
            for _ in range(3):
                tr.run(W0, 0.5, False, 0.0, False, 0.0, ch)
            ts = []
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                tr.run(W0, 0.5, False, 0.0, False, 0.0, ch)
                e1.record()
                ts.append((e0, e1))
            torch.cuda.synchronize()
        tr.check_errors()
        ms = float(np.mean([x.elapsed_time(y) for x, y in ts]))
        print('config %d %s=%d: %.1f us/launch (%.1f%% of 8 TB/s)' % (a.config, a.field, v, ms * 1e3,
                                                                     alg / ms / 1e6 / 80), flush=True)


if __name__ == '__main__':
    main()
