#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-pipe7}
mkdir -p gpurun_out/$R
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipe.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/$R/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/$R/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u scripts/lt_time.py 100 2 1026 2 1026 > gpurun_out/$R/lt_time.txt 2>&1 || { echo "lt rc=$?"; tail gpurun_out/$R/lt_time.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/$R/lt_time.txt
bash scripts/gpu_stamps.sh $R "--config 2 --G 2 --pipe"
