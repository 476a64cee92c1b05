#!/bin/bash
# round record: full GPU suite (verbose), smoke(), then the default bench line twice
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-record}
mkdir -p gpurun_out/$R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
  > gpurun_out/$R/gpu_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/$R/gpu_tests.log; exit 1; }
tail -2 gpurun_out/$R/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$R/smoke.log 2>&1 \
  || { echo "smoke rc=$?"; tail -30 gpurun_out/$R/smoke.log; exit 1; }
tail -2 gpurun_out/$R/smoke.log
for k in a b; do
  timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$R/bench_$k.json 2> gpurun_out/$R/bench_$k.err \
    || { echo "bench rc=$?"; tail -30 gpurun_out/$R/bench_$k.err; exit 1; }
  cut -c1-300 gpurun_out/$R/bench_$k.json
done
