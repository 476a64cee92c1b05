"""Tabulate the GPU's measured distance from the reference on every solver-horizon case.

    python scripts/horizon_margins.py gpurun_out/horizon_margins.jsonl profiles/r06/horizon_margins.json

Input: the JSON lines tests/test_gpu_parity.py::test_dropin_solver_horizon_fedamw appends to
$FS_MARGINS_OUT (one per case: per-round relative W error and bound, final p error and bound,
per-round loss error and bound).  Output: one JSON object per case with the worst round, the
largest fraction of its bound any round used, and the fp32-vs-fp64 drift / oracle-vs-reference
distances of tests/golden/horizon_drift.json beside them; a table on stdout.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(src, dst):
    drift = json.load(open(os.path.join(ROOT, 'tests', 'golden', 'horizon_drift.json')))
    out = {}
    for line in open(src):
        r = json.loads(line)
        name = r.pop('case')
        eW, bW = r['W_rel_err'], r['W_bound']
        el, bl = r['loss_err'], r['loss_bound']
        use = [e / b for e, b in zip(eW, bW)]
        t = max(range(len(use)), key=use.__getitem__)
        dr = drift[name]
        out[name] = dict(r, W_max_rel_err=max(eW), W_worst_round=t, W_bound_used=max(use),
                         W_bound_round0=bW[0], W_bound_last=bW[-1],
                         loss_max_err=max(el), loss_bound_used=max(e / b for e, b in zip(el, bl)),
                         p_bound_used=r['p_rel_err'] / r['p_bound'],
                         fp32_vs_fp64_W=dr['delta_W'], fp32_vs_fp64_p=dr['delta_p'],
                         oracle_vs_reference_W=dr['oracle_vs_reference_W'],
                         oracle_vs_reference_p=dr['oracle_vs_reference_p'])
    os.makedirs(os.path.dirname(os.path.abspath(dst)), exist_ok=True)
    with open(dst, 'w') as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print('| case | GPU max W err | bound (round 0 .. last) | most of a bound used (round) | GPU p err / bound | '
          'GPU loss err / bound | fp32 vs fp64 W | oracle vs ref W |')
    print('|---|---|---|---|---|---|---|---|')
    for name in sorted(out):
        o = out[name]
        print('| %s | %.1e | %.1e .. %.1e | %.2f (%d) | %.1e / %.1e | %.1e / %.2f | %.1e | %.1e |'
              % (name, o['W_max_rel_err'], o['W_bound_round0'], o['W_bound_last'], o['W_bound_used'], o['W_worst_round'],
                 o['p_rel_err'], o['p_bound'], o['loss_max_err'], o['loss_bound_used'], o['fp32_vs_fp64_W'],
                 o['oracle_vs_reference_W']))


if __name__ == '__main__':
    main(*sys.argv[1:3])
