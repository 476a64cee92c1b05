#!/bin/bash
# split form's early row issue with the prox term: bitwise tests, then config 3's launch time early vs late
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-proxearly}
mkdir -p gpurun_out/$R
timeout -k 10 400 python -u -m pytest tests/test_gpu_split_early.py tests/test_gpu_configs.py -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/$R/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/$R/tests.log; exit 1; }
tail -1 gpurun_out/$R/tests.log
for i in 1 2; do
  timeout -k 10 300 python -u scripts/lt_sweep.py --config 3 --prox --reg 0 --G 4,264,4 2>&1 | grep -v amdgpu.ids >> gpurun_out/$R/sweep.txt || exit 1
  timeout -k 10 300 python -u scripts/lt_sweep.py --config 3 --prox --reg 0 --early off --G 4 2>&1 | grep -v amdgpu.ids | sed 's/$/ (late issue)/' >> gpurun_out/$R/sweep.txt || exit 1
done
cat gpurun_out/$R/sweep.txt
