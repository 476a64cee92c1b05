#!/bin/bash
# full GPU suite (verbose: every test named), then the default bench line
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-r04i}
mkdir -p gpurun_out/$R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
  > gpurun_out/$R/gpu_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/$R/gpu_tests.log; exit 1; }
tail -2 gpurun_out/$R/gpu_tests.log
timeout -k 10 400 python -u bench.py > gpurun_out/$R/bench.json 2> gpurun_out/$R/bench.err \
  || { echo "bench rc=$?"; tail -30 gpurun_out/$R/bench.err; exit 1; }
cut -c1-400 gpurun_out/$R/bench.json
