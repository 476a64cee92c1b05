#!/bin/bash
# The 4-wave stream form of local training: its bitwise tests, the bench A/B (stream on / off)
# at configs 2 and 5, and the phase stamps of both forms.   scripts/gpu_stream.sh <tag>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-stream}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/$TAG/stream_tests.log 2>&1 || { echo "stream tests rc=$?"; tail -30 gpurun_out/$TAG/stream_tests.log; exit 1; }
tail -1 gpurun_out/$TAG/stream_tests.log
for cfg in 2 5; do
  for form in on off; do
    timeout -k 10 300 python -u bench.py --config $cfg --stream-form $form --no-legs --no-fedamw-leg --no-cpu-baseline \
      --steps 6 --warmup 2 > gpurun_out/$TAG/bench_c${cfg}_$form.json 2> gpurun_out/$TAG/bench_c${cfg}_$form.err \
      || { echo "bench c$cfg $form rc=$?"; tail -20 gpurun_out/$TAG/bench_c${cfg}_$form.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/$TAG/bench_c${cfg}_$form.json')); r=d['roofline']; print('config $cfg stream $form', r['form'], round(d['value']), 'ms/round %.4f' % d['ms_per_step'], 'launch %.4f ms' % r['launch_ms'], 'frac %.3f' % r['frac'])"
  done
done
bash scripts/gpu_stamps.sh $TAG/st "--config 2 --stream" "--config 2" "--config 5 --stream" "--config 5"
