#!/bin/bash
# pipe form diagnostics: determinism / split diffs, then phase stamps (split vs pipe, config 2)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-pipe3}
mkdir -p gpurun_out/$R
timeout -k 10 300 python -u scripts/pipe_debug.py > gpurun_out/$R/debug.txt 2>&1; echo "debug rc=$?"; grep -v amdgpu.ids gpurun_out/$R/debug.txt
bash scripts/gpu_stamps.sh $R "--config 2 --G 2" "--config 2 --G 2 --pipe"
