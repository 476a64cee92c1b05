#!/bin/bash
# pipe form with the prox term: its GPU tests, then config 3's launch time pair (G = 8) vs pipe (G = 4)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-pipeprox}
mkdir -p gpurun_out/$R
timeout -k 10 900 python -u -m pytest tests/test_gpu_pipe.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/$R/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/$R/tests.log; exit 1; }
tail -3 gpurun_out/$R/tests.log
for i in 1 2; do
  timeout -k 10 300 python -u scripts/lt_sweep.py --config 3 --prox --G 0,2056,1028 >> gpurun_out/$R/sweep3.txt 2>&1 \
    || { echo "sweep rc=$?"; tail -20 gpurun_out/$R/sweep3.txt; exit 1; }
done
grep -v amdgpu.ids gpurun_out/$R/sweep3.txt
