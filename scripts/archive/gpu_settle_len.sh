#!/bin/bash
# the workload settle's length (config 2 headline only)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/settlelen
mkdir -p $O
for k in 1 2; do
 for ms in 100 300 1000; do
  FS_BENCH_SETTLE_MS=$ms timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-legs --no-fedamw-leg > $O/s${ms}_$k.json 2> $O/s${ms}_$k.err || { echo "bench rc=$?"; tail -30 $O/s${ms}_$k.err; exit 1; }
 done
done
python - <<'P'
import json,glob
for f in sorted(glob.glob('gpurun_out/settlelen/*.json')):
    d=json.load(open(f))
    print('%-14s c2 %.0f %.4f ms/round launch %.4f frac %.4f settle %.0f ms' % (f.split('/')[-1], d['value'], d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac'], d['device_settle_ms']))
P
