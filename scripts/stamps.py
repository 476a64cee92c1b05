"""Diagnostic: per-phase cycle split of the split-client group kernel (stamp build).

    make -C <pkg>/csrc stamps
    FEDSIM_LIB=<pkg>/libfedsim_stamps.so python scripts/stamps.py --config 5 [--G 16] [--chained]

Wave 0 of every workgroup sums s_memtime deltas per phase over its steps (the stamps cost
~40 cycles each); printed as cycles per step (mean / min / max over workgroups)."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fedamw_amd  # noqa: E402,F401
from fedamw_amd import data, engine, rng  # noqa: E402
from scripts.lt_sweep import SHAPES  # noqa: E402

NAMES = ['fwd', 'S1', 'sum+publish', 'poll+sum', 'next(early)', 'S2', 'softmax+S3+next', 'bwd+update']
PAIR_NAMES = ['wait rows', 'fwd', 'S1', 'publish+img', 'wait polls', 'check', 'sum+S2', 'softmax+S3',
              'issue', 'bwd+update']
PIPE_NAMES = ['wait rows0', 'fwd0', 'B1a', 'own0+pub0', 'wait rows1', 'fwd1', 'B1b', 'own1+pub1+poll0+idx',
              'img', 'wait poll0', 'smax0+poll1+issue0', 'K0', 'wait poll1+issue1', 'smax1+K1+upd+end']


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', type=int, default=2, choices=sorted(SHAPES))
    ap.add_argument('--G', type=int, default=0)
    ap.add_argument('--chained', action='store_true')
    ap.add_argument('--pair', action='store_true', help='the pair form at width --G (or the planner\'s)')
    ap.add_argument('--teams', action='store_true', help='the team form at width --G (team 0 stamped)')
    ap.add_argument('--pipe', action='store_true', help='the pipe form at width --G')
    ap.add_argument('--prox', action='store_true', help="FedProx's prox term (mu = 1e-3), ridge off")
    ap.add_argument('--dbuf', choices=['auto', 'on', 'off'], default='auto',
                    help="fs_tuning.split_dbuf: the split form's double-buffered instance (round 6)")
    ap.add_argument('--mb', choices=['auto', 'on', 'off'], default='auto',
                    help="fs_tuning.split_mb: the split form's 4x4x1 multi-block MFMA instances (round 6)")
    a = ap.parse_args()
    assert os.environ.get('FEDSIM_LIB', '').endswith('stamps.so'), 'run with FEDSIM_LIB=.../libfedsim_stamps.so'
    fedamw_amd._lib.set_tuning(split_dbuf={'auto': 0, 'on': 1, 'off': -1}[a.dbuf],
                               split_mb={'auto': 0, 'on': 1, 'off': -1}[a.mb])
    sh = SHAPES[a.config]
    chained = a.chained or sh.get('chained', False)
    dev = torch.device('cuda')
    N, D, C, E, B = sh['clients'], sh['D'], sh['C'], 2, 32
    d = data.federated(N, sh['rows'], D, C, 1000, shape=sh['shape'], device=dev)
    feats = engine.Features(d['X_train'], d['y_train'], D, dev)
    L = fedamw_amd._lib
    split = (a.G | L.G_PAIR if a.pair else (a.G | L.G_TEAMS if a.teams else (a.G | L.G_PIPE if a.pipe else a.G))) or None
    tr = engine.LocalTrainer(feats, C, B, E, split=split, chained=chained, prox=a.prox)
    names = PAIR_NAMES if tr.pair else (PIPE_NAMES if tr.pipe else NAMES)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    grid = 8 * tr.width if chained else tr.groups(cus) * tr.width
    per_wave = 8 if tr.pipe else 1                              # the pipe form stamps every wave
    extra = grid * per_wave * 16 * 8
    base = tr.ws.numel() - fedamw_amd._lib.ERR_BLOCK          # exchange granules; stamps go right after
    tr.ws = torch.zeros(tr.ws.numel() + extra, dtype=torch.uint8, device=dev)
    torch.manual_seed(0)
    tr.upload_perms(rng.draw_pass_seeds(N * E))
    W0 = torch.zeros(C, feats.ld, device=dev)
    for _ in range(3):
        tr.run(W0, 0.5, a.prox, 1e-3, not a.prox, 1e-5, chained)
    torch.cuda.synchronize()
    tr.check_errors()
    st = tr.ws[base:base + extra].view(torch.int64).view(-1, 16).cpu().numpy().astype(np.float64)
    if per_wave > 1:
        allw = st.reshape(-1, per_wave, 16)
        allw = allw[allw[:, 0, 15] > 0]
        pw = allw[:, :, :14] / allw[:, :, 15:16]
        print('per wave (mean over workgroups), cycles/step:')
        for k, nm in enumerate(PIPE_NAMES):
            print('  %-22s' % nm + ' '.join('%6.0f' % pw[:, wv, k].mean() for wv in range(per_wave)))
        st = allw[:, 0, :]
    st = st[st[:, 15] > 0]
    steps = st[:, 15]
    per = st[:, :len(names)] / steps[:, None]
    print('config %d G %s (%s): %d workgroups, %.0f steps each' % (a.config, ('pair %d' % tr.width) if tr.pair else tr.width, 'chained' if chained else
                                                                   'parallel', len(st), steps.mean()))
    for k, nm in enumerate(names):
        print('%-16s mean %8.0f  min %8.0f  max %8.0f cycles/step' % (nm, per[:, k].mean(), per[:, k].min(),
                                                                       per[:, k].max()))
    print('total            mean %8.0f cycles/%s' % (per.sum(1).mean(), 'half-step' if tr.pair else 'step'),
          flush=True)


if __name__ == '__main__':
    main()
