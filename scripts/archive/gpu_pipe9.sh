#!/bin/bash
# pipe vs the planner's form at configs 2, 4, 5 (launch times)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-pipe9}
mkdir -p gpurun_out/$R
for a in "--config 2 --G 0,1026,0,1026 --reg 0" "--config 4 --G 0,1026,0,1026 --reg 0" "--config 5 --G 0,1040,0,1040 --reg 1"; do
  timeout -k 10 300 python -u scripts/lt_sweep.py $a >> gpurun_out/$R/sweep.txt 2>&1 || { echo "sweep rc=$?"; tail gpurun_out/$R/sweep.txt; exit 1; }
done
grep -v amdgpu.ids gpurun_out/$R/sweep.txt
