#!/bin/bash
# one-launch aggregation at every N: tests, launch times, then bench length A/B (20 / 100 / 200 rounds)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-agg2}
mkdir -p gpurun_out/$R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "aggregate or deferred or dropin_fedavg or round" > gpurun_out/$R/tests.log 2>&1 \
  || { echo "tests rc=$?"; tail -30 gpurun_out/$R/tests.log; exit 1; }
tail -1 gpurun_out/$R/tests.log
for s in "1000 7 4096" "1250 10 2048" "1000 10 16384" "100 10 2048"; do
  timeout -k 10 120 python -u scripts/agg_time.py $s 2>&1 | grep -v amdgpu.ids >> gpurun_out/$R/agg_time.txt \
    || { echo "agg_time rc=$?"; exit 1; }
done
cat gpurun_out/$R/agg_time.txt
for k in 1 2; do
  for st in 20 100 200; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-legs --no-fedamw-leg --steps $st \
      > gpurun_out/$R/steps$st.$k.json 2>/dev/null || { echo "ab rc=$?"; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/$R/steps$st.$k.json')); print('steps=$st', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['launch_ms'],4))"
  done
done
