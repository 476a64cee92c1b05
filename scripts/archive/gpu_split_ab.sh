#!/bin/bash
# split-form timing at configs 2 and 5 (+ its GPU tests), for A/B against the previous sources
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r03}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "split or unit_golden or vs_oracle or persistent or golden" \
  > gpurun_out/$TAG/split_tests.log 2>&1 || { echo "split tests rc=$?"; tail -30 gpurun_out/$TAG/split_tests.log; exit 1; }
tail -1 gpurun_out/$TAG/split_tests.log
for cfg in 2 5; do
  timeout -k 10 300 python -u bench.py --config $cfg --train-form split --no-legs --no-fedamw-leg --no-cpu-baseline \
    --steps 6 --warmup 2 > gpurun_out/$TAG/bench_c${cfg}_split.json 2> gpurun_out/$TAG/bench_c${cfg}_split.err \
    || { echo "bench c$cfg rc=$?"; tail -20 gpurun_out/$TAG/bench_c${cfg}_split.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/$TAG/bench_c${cfg}_split.json')); r=d['roofline']; print('config $cfg split', round(d['value']), 'ms/round %.4f' % d['ms_per_step'], 'launch %.4f ms' % r['launch_ms'], 'frac %.3f' % r['frac'])"
done
