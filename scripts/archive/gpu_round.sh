#!/bin/bash
# One GPU-box session: GPU tests, then the default bench line (configs 2-5), each under its own
# time limit, chained so that the first failure ends the call.
#   scripts/gpu_round.sh <tag> [tests|bench|all] [pytest -k expr]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r03}; WHAT=${2:-all}; K=${3:-}
mkdir -p gpurun_out/$TAG
if [ "$WHAT" = tests ] || [ "$WHAT" = all ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${K:+-k "$K"} \
    > gpurun_out/$TAG/gpu_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/$TAG/gpu_tests.log; exit 1; }
  tail -3 gpurun_out/$TAG/gpu_tests.log
fi
if [ "$WHAT" = bench ] || [ "$WHAT" = all ]; then
  timeout -k 10 400 python -u bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err \
    || { echo "bench rc=$?"; tail -30 gpurun_out/$TAG/bench.err; exit 1; }
  cat gpurun_out/$TAG/bench.json
fi
