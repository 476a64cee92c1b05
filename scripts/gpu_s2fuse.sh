#!/bin/bash
# Deferred evaluation (FS_PHASE_EVAL_DEFER): drop-in parity tests, then bench A/B at configs 2 and 4
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-s2fuse}; mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step pytest timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "dropin or deferred" > $O/gpu_tests.log 2>&1
tail -1 $O/gpu_tests.log
for c in 2 4; do
  for v in 0 1; do
    step bench_c${c}_d$v env FS_EVAL_DEFER=$v timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $O/bench_c${c}_d$v.json 2> $O/bench_c${c}_d$v.err
    python3 -c "
import json; d=json.loads(open('$O/bench_c${c}_d$v.json').read().strip().splitlines()[-1]); r=d['roofline']
print('c$c defer=$v', round(d['value']), 'ms/step %.4f' % d['ms_per_step'], 'frac %.3f' % r['frac'])"
  done
done
