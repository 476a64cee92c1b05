#!/bin/bash
# round 6: the default bench line twice (the driver's command), final sources
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-r06_final}
mkdir -p gpurun_out/$R
for k in a b; do
  timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$R/bench_$k.json 2> gpurun_out/$R/bench_$k.err \
    || { echo "bench rc=$?"; tail -30 gpurun_out/$R/bench_$k.err; exit 1; }
  cut -c1-200 gpurun_out/$R/bench_$k.json
done
