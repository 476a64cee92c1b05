#!/bin/bash
# full GPU suite, default bench line, kernel trace of the default bench (round-4 records)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=r04e
mkdir -p gpurun_out/$R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  > gpurun_out/$R/gpu_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/$R/gpu_tests.log; exit 1; }
tail -2 gpurun_out/$R/gpu_tests.log
timeout -k 10 400 python -u bench.py > gpurun_out/$R/bench.json 2> gpurun_out/$R/bench.err \
  || { echo "bench rc=$?"; tail -30 gpurun_out/$R/bench.err; exit 1; }
cat gpurun_out/$R/bench.json | cut -c1-600
