#!/bin/bash
# pipe/pair/split bitwise + parity tests after pinning the norm/update rounding; per-wave stamps
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-pipe6}
mkdir -p gpurun_out/$R
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipe.py tests/test_gpu_pair.py tests/test_gpu_split_early.py tests/test_gpu_teams.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/$R/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/$R/tests.log
[ $rc -eq 0 ] || exit 1
bash scripts/gpu_stamps.sh $R "--config 2 --G 2 --pipe"
