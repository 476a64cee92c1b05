#!/bin/bash
# one-launch aggregation: its GPU tests, launch times against the chunked form, then the bench line
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-agg}
mkdir -p gpurun_out/$R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "aggregate or deferred or dropin_fedavg or round" > gpurun_out/$R/tests.log 2>&1 \
  || { echo "tests rc=$?"; tail -30 gpurun_out/$R/tests.log; exit 1; }
tail -2 gpurun_out/$R/tests.log
for s in "100 10 2048" "1000 7 4096" "1250 10 2048" "300 10 2048"; do
  timeout -k 10 120 python -u scripts/agg_time.py $s 2>&1 | grep -v amdgpu.ids >> gpurun_out/$R/agg_time.txt \
    || { echo "agg_time rc=$?"; exit 1; }
done
cat gpurun_out/$R/agg_time.txt
for k in 1 2; do
  for ev in 0 1; do
    FS_BENCH_NO_EVENTS=$ev timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-legs --no-fedamw-leg --steps 200 \
      > gpurun_out/$R/ab_ev$ev.$k.json 2>/dev/null || { echo "ab rc=$?"; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/$R/ab_ev$ev.$k.json')); print('no-events=$ev', round(d['value']), round(d['ms_per_step'],4))"
  done
done
for k in a; do
  timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/$R/bench_$k.json 2> gpurun_out/$R/bench_$k.err \
    || { echo "bench rc=$?"; tail -30 gpurun_out/$R/bench_$k.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/$R/bench_$k.json')); r=d['roofline']; print('c2', round(d['value']), round(d['ms_per_step'],4), round(r['frac'],4), round(r['launch_ms'],4), r['traffic'] is not None); [print(c, round(d[c]['value']), round(d[c]['ms_per_round'],4)) for c in ('config3','config4','config5','config1')]; print('fedamw', d['fedamw']['ms_per_round'])"
done
