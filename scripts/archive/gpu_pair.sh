#!/bin/bash
# Pair-form bring-up: its GPU tests, then config-2/3/4 bench lines with each form.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r03b}
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests/test_gpu_pair.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/$TAG/pair_tests.log 2>&1 || { echo "pair tests rc=$?"; tail -40 gpurun_out/$TAG/pair_tests.log; exit 1; }
tail -3 gpurun_out/$TAG/pair_tests.log
for cfg in 2 4 3; do
  for form in split pair; do
    timeout -k 10 200 python -u bench.py --config $cfg --train-form $form --no-legs --no-fedamw-leg --no-cpu-baseline \
      --steps 10 --warmup 2 > gpurun_out/$TAG/bench_c${cfg}_$form.json 2> gpurun_out/$TAG/bench_c${cfg}_$form.err \
      || { echo "bench c$cfg $form rc=$?"; tail -20 gpurun_out/$TAG/bench_c${cfg}_$form.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/$TAG/bench_c${cfg}_$form.json')); r=d['roofline']; print('config $cfg $form', round(d['value']), 'ms/round %.4f' % d['ms_per_step'], 'launch %.4f ms' % r['launch_ms'], 'frac %.3f' % r['frac'], r['form'], r['group_width'])"
  done
done
