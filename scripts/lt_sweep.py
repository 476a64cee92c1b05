"""Diagnostic: mean fs_local_train launch time per group width G at a BASELINE config shape.

    python scripts/lt_sweep.py --config 5 --G 1,8,16 [--chained] [--prox]      (GPU box)

G = 1 is the one-workgroup-per-client kernel, G >= 2 the split-client group kernel
(FS_SPLIT_G semantics); 0 = the planner's choice.  Prints one line per G: microseconds per
launch and the algorithmic HBM rate (4*E*sum(n_j)*D + 8*E*sum(n_j) + 8*N*C*D
bytes per launch)."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fedamw_amd  # noqa: E402,F401
import fedamw_amd._lib  # noqa: E402
from fedamw_amd import data, engine, rng  # noqa: E402

# per-GPU shapes of the BASELINE configs (bench.py PRESETS); config 1 = exp.py's a9a chain
CONFIG1_SIZES = [11434, 5200, 3100, 2400, 1500, 1000, 700, 400, 375, 346]
SHAPES = {
    1: dict(clients=10, rows=CONFIG1_SIZES, D=2000, C=2, shape='a9a', chained=True),
    2: dict(clients=100, rows=512, D=2048, C=10, shape='a9a'),
    3: dict(clients=1000, rows=465, D=4096, C=7, shape='covtype'),
    4: dict(clients=1250, rows=64, D=2048, C=10, shape='a9a'),
    5: dict(clients=1000, rows=128, D=16384, C=10, shape='a9a'),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', type=int, default=2, choices=sorted(SHAPES))
    ap.add_argument('--G', default='0')
    ap.add_argument('--chained', action='store_true')
    ap.add_argument('--prox', action='store_true')
    ap.add_argument('--reps', type=int, default=10)
    ap.add_argument('--reg', type=int, default=1, help='ridge term on (FedAMW local training) or off (FedAvg)')
    ap.add_argument('--early', choices=['auto', 'off'], default='auto', help="fs_tuning.split_early (the split form's early row issue)")
    ap.add_argument('--dbuf', choices=['auto', 'on', 'off'], default='auto',
                    help="fs_tuning.split_dbuf (the split form's double-buffered instance, round 6)")
    ap.add_argument('--mb', choices=['auto', 'on', 'off'], default='auto',
                    help="fs_tuning.split_mb (the split form's 4x4x1 multi-block MFMA instances, round 6)")
    a = ap.parse_args()
    fedamw_amd._lib.set_tuning(split_early={'auto': 0, 'off': -1}[a.early],
                               split_dbuf={'auto': 0, 'on': 1, 'off': -1}[a.dbuf],
                               split_mb={'auto': 0, 'on': 1, 'off': -1}[a.mb])
    sh = SHAPES[a.config]
    chained = a.chained or sh.get('chained', False)
    dev = torch.device('cuda')
    N, D, C, E, B = sh['clients'], sh['D'], sh['C'], 2, 32
    d = data.federated(N, sh['rows'], D, C, 1000, shape=sh['shape'], device=dev)
    feats = engine.Features(d['X_train'], d['y_train'], D, dev)
    del d
    alg = 4.0 * E * feats.rows * D + 8.0 * E * feats.rows + 8.0 * N * C * D
    steps = int(np.sum(E * ((feats.ns + B - 1) // B)))
    for G in [int(g) for g in a.G.split(',')]:
        try:
            tr = engine.LocalTrainer(feats, C, B, E, split=(G or None), chained=chained, prox=a.prox)
        except fedamw_amd._lib.FedsimError as ex:
            print('config %d G=%d: n/a (%s)' % (a.config, G, ex), flush=True)
            continue
        torch.manual_seed(0)
        tr.upload_perms(rng.draw_pass_seeds(N * E))
        W0 = torch.zeros(C, feats.ld, device=dev)
        W0.normal_(0, 0.01)
        for _ in range(2):
            tr.run(W0, 0.5, a.prox, 1e-3, bool(a.reg), 1e-5, chained)
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            tr.run(W0, 0.5, a.prox, 1e-3, bool(a.reg), 1e-5, chained)
            e1.record()
            ts.append((e0, e1))
        torch.cuda.synchronize()
        tr.check_errors()
        ms = float(np.mean([x.elapsed_time(y) for x, y in ts]))
        print('config %d %s G=%d: %.1f us/launch, %.0f GB/s algorithmic (%.1f%% of 8 TB/s), %.2f us/step-chain%s'
              % (a.config, 'chained' if chained else 'parallel', tr.G, ms * 1e3, alg / ms / 1e6,
                 alg / ms / 1e6 / 80, ms * 1e3 / (steps if chained else 1), ' prox' if a.prox else ''), flush=True)
        del tr


if __name__ == '__main__':
    main()
