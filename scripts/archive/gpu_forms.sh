#!/bin/bash
# launch time of every local-training form at configs 3 and 4 (two passes each)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-forms}
mkdir -p gpurun_out/$R
for i in 1 2; do
  timeout -k 10 300 python -u scripts/lt_sweep.py --config 3 --prox --G 0,4,260,1028 2>&1 | grep -v amdgpu.ids >> gpurun_out/$R/sweep.txt || exit 1
  timeout -k 10 300 python -u scripts/lt_sweep.py --config 4 --G 0,2,4,260,1026 2>&1 | grep -v amdgpu.ids >> gpurun_out/$R/sweep.txt || exit 1
done
cat gpurun_out/$R/sweep.txt
