#!/bin/bash
# team form: tests, then bench A/B (auto form vs --train-form teams) at configs 2, 4, 3
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-teams}
mkdir -p gpurun_out/$TAG
timeout -k 10 500 python -u -m pytest tests/test_gpu_teams.py tests/test_gpu_split_early.py -m gpu -x -v --timeout 150 \
  --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/$TAG/tests.log; exit 1; }
tail -2 gpurun_out/$TAG/tests.log
OUT=gpurun_out/$TAG/ab.txt
: > $OUT
for c in 2 4 3; do
  for f in auto teams auto teams; do
    timeout -k 10 200 python -u bench.py --config $c --no-legs --no-fedamw-leg --no-cpu-baseline --steps 20 --warmup 3 \
      --train-form $f > gpurun_out/$TAG/b.json 2> gpurun_out/$TAG/b.err || { echo "bench rc=$? c$c $f"; tail -20 gpurun_out/$TAG/b.err; exit 1; }
    python -c "import json; d = json.loads(open('gpurun_out/$TAG/b.json').read().strip().splitlines()[-1]); r = d['roofline']; print('config $c $f', round(d['value']), 'cr/s', round(d['ms_per_step'], 4), 'ms/round, launch', round(r['launch_ms'], 4), 'frac', round(r['frac'], 4), r['form'], r['group_width'])" >> $OUT
  done
done
cat $OUT
