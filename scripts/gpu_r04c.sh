#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04d
for a in "4 1 0.002" "4 1 0" "4 1 0.002 1" "8 1 0.002" "16 1 0.002" "2 1 0.002"; do
  timeout -k 10 120 python -u scripts/stream_diff.py $a >> gpurun_out/r04d/diff.txt 2>&1 || { echo "diff rc=$?"; tail gpurun_out/r04d/diff.txt; exit 1; }
done
grep -v amdgpu gpurun_out/r04d/diff.txt
TAG=r04st2
mkdir -p gpurun_out/$TAG
for cfg in 2 5; do
  for form in on off; do
    timeout -k 10 300 python -u bench.py --config $cfg --stream-form $form --no-legs --no-fedamw-leg --no-cpu-baseline \
      --steps 6 --warmup 2 > gpurun_out/$TAG/bench_c${cfg}_$form.json 2> gpurun_out/$TAG/bench_c${cfg}_$form.err \
      || { echo "bench c$cfg $form rc=$?"; tail -20 gpurun_out/$TAG/bench_c${cfg}_$form.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/$TAG/bench_c${cfg}_$form.json')); r=d['roofline']; print('config $cfg stream $form', r['form'], round(d['value']), 'ms/round %.4f' % d['ms_per_step'], 'launch %.4f ms' % r['launch_ms'], 'frac %.3f' % r['frac'])"
  done
done
bash scripts/gpu_stamps.sh $TAG/st "--config 2 --stream" "--config 2" "--config 5 --stream"
