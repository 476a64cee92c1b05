#!/bin/bash
# aggregation auto rule re-check, then bench warm-up A/B at the driver's --steps 20 (warmup 5 vs 50)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-warm}
mkdir -p gpurun_out/$R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "aggregate or deferred or dropin_fedavg or round" > gpurun_out/$R/tests.log 2>&1 \
  || { echo "tests rc=$?"; tail -30 gpurun_out/$R/tests.log; exit 1; }
tail -1 gpurun_out/$R/tests.log
for s in "1000 7 4096" "1250 10 2048"; do
  timeout -k 10 120 python -u scripts/agg_time.py $s 2>&1 | grep -v amdgpu.ids | head -2 >> gpurun_out/$R/agg_time.txt \
    || { echo "agg_time rc=$?"; exit 1; }
done
cat gpurun_out/$R/agg_time.txt
for k in 1 2; do
  for w in 5 50 200; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-legs --no-fedamw-leg --steps 20 --warmup $w \
      > gpurun_out/$R/w$w.$k.json 2>/dev/null || { echo "ab rc=$?"; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/$R/w$w.$k.json')); print('warmup=$w', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['launch_ms'],4))"
  done
done
