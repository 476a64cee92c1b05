#!/bin/bash
# GPU suite, smoke, bench lines at configs 2 (default, + CPU baseline) / 3 / 4 / 5, rocprofv3
# kernel stats of the default bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-s2bench}; mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step pytest timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
tail -1 $O/gpu_tests.log
step smoke timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step bench_c2 timeout -k 10 300 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err
step prof_c2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 --output-format csv -- python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_c2.log 2>&1
step bench_c4 timeout -k 10 300 python -u bench.py --config 4 > $O/bench_c4.json 2> $O/bench_c4.err
step bench_c3 timeout -k 10 300 python -u bench.py --config 3 --steps 5 --warmup 2 > $O/bench_c3.json 2> $O/bench_c3.err
step bench_c5 timeout -k 10 400 python -u bench.py --config 5 --steps 2 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err
for c in 2 3 4 5; do python3 -c "
import json; d=json.loads(open('$O/bench_c$c.json').read().strip().splitlines()[-1]); r=d['roofline']
print('c$c', round(d['value']), 'ms/step %.4f' % d['ms_per_step'], 'frac %.3f' % r['frac'], 'traffic', r['traffic'], r.get('traffic_note'), d.get('fedamw', {}).get('p_solve_us_per_step'))"; done
