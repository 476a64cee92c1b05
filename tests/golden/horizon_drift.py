"""The fp32 arithmetic's own drift at each FedAMW solver horizon -- the derived tolerance of
the horizon parity checks.

    python tests/golden/horizon_drift.py            (CPU, a few minutes; writes horizon_drift.json)

For every horizon case (``horizon_<solver>_<mode>.npz``, make_golden.py run_horizon) the CPU
restatement (oracle/fedsim_oracle.py) runs the case twice on the same inputs and the same
torch RNG stream: once in float32 (as the reference computes) and once in float64 (the module's
working type ``F32`` rebound to float64 for the run -- every array and scalar of the
restatement follows it).  The relative distance of the two after every round,

    delta_W(t) = max|W32(t) - W64(t)| / max|W64(t)|,   delta_p(t) likewise for p,

is how far ANY correct float32 evaluation of the round may sit from the exact one at that
horizon -- summation order alone moves an fp32 result by about this much (the reference's
torch kernels and ours sum in different orders).  Two fp32 evaluations may then differ by up to
about twice it, so the parity bounds of a case are rtol_W = max(1e-5, 2 max_t delta_W) and
rtol_p = max(1e-5, 2 max_t delta_p) (the losses likewise: rtol_loss), stated per case in the JSON and read by tests/fixtures.py
(``horizon_rtol``).  Round 6 (one whole-run bound let a GPU error 100x the real
drift of the early rounds pass): the per-round distances are stored too, and the GPU parity check
of round t uses max(1e-5, 2 max_{s <= t} delta(s)) -- the drift accumulated by round t
(``horizon_rtol_rounds``).  Only the oracle runs here: it is test
infrastructure, and the reference is not imported.
"""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import fedsim_oracle as O  # noqa: E402
from tests.fixtures import HORIZON_CASES, load_horizon, positional, split_clients  # noqa: E402


def run(d, dtype):
    saved = O.F32
    O.F32 = dtype
    try:
        Xs, ys = split_clients(d)
        Xs = [np.asarray(x, dtype) for x in Xs]
        mode = 'parallel' if str(d['mode']) == 'par' else 'sequential'
        torch.manual_seed(int(d['torch_seed']))
        tr, tl, ta, trace = O.FedAMW(Xs, ys, np.asarray(d['X_test'], dtype), d['y_test'],
                                     np.asarray(d['X_val'], dtype), d['y_val'], *positional(d),
                                     lr_p=float(d['lr_p']), clients=mode)
        return trace, tr, tl
    finally:
        O.F32 = saved


def main():
    torch.set_num_threads(1)
    out = {}
    for name in HORIZON_CASES:
        d = load_horizon(name)
        (t32, tr32, tl32), (t64, tr64, tl64) = run(d, np.float32), run(d, np.float64)
        # the losses (train: the p-weighted client losses; test: the global model's CE), as the
        # parity checks scale them: absolute difference / max(1, max|loss|)
        dl = max(float(np.abs(np.asarray(a, np.float64) - b).max() / max(1.0, float(np.abs(b).max())))
                 for a, b in ((tr32, tr64), (tl32, tl64)))
        # per round (round 6): the larger of the train and test loss distances
        dl_t = [max(float(abs(float(a[t]) - float(b[t])) / max(1.0, float(np.abs(b).max())))
                    for a, b in ((tr32, tr64), (tl32, tl64))) for t in range(len(tr64))]
        dW = [float(np.abs(a.astype(np.float64) - b).max() / np.abs(b).max()) for a, b in zip(t32['W'], t64['W'])]
        dp = [float(np.abs(a.astype(np.float64) - b).max() / np.abs(b).max()) for a, b in zip(t32['p'], t64['p'])]
        # the fp32 oracle against the reference (its measured distance, for the record)
        rW = [float(np.abs(a - b).max() / np.abs(b).max()) for a, b in zip(t32['W'], d['W'])]
        rp = [float(np.abs(a - b).max() / np.abs(b).max()) for a, b in zip(t32['p'], d['p'])]
        out[name] = {'delta_W': max(dW), 'delta_p': max(dp), 'delta_W_per_round': dW, 'delta_p_per_round': dp,
                     'oracle_vs_reference_W': max(rW), 'oracle_vs_reference_p': max(rp),
                     'delta_loss': dl, 'delta_loss_per_round': dl_t,
                     'rtol_W': max(1e-5, 2.0 * max(dW)), 'rtol_p': max(1e-5, 2.0 * max(dp)),
                     'rtol_loss': max(1e-5, 2.0 * dl)}
        print('%-24s delta_W %.2e delta_p %.2e | oracle vs reference W %.2e p %.2e | rtol W %.2e p %.2e'
              % (name, max(dW), max(dp), max(rW), max(rp), out[name]['rtol_W'], out[name]['rtol_p']), flush=True)
    with open(os.path.join(HERE, 'horizon_drift.json'), 'w') as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == '__main__':
    main()
