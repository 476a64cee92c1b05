#!/bin/bash
# Phase stamps of the local-training kernels (diagnostic build, libfedsim_stamps.so).
#   scripts/gpu_stamps.sh <tag> "<stamps.py args>" ["<stamps.py args>" ...]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out/$TAG
i=0
for a in "$@"; do
  i=$((i+1))
  FEDSIM_LIB=$PWD/non-iid-distributed-learning-with-optimal-mixture-weights_amd/libfedsim_stamps.so \
    timeout -k 10 120 python -u scripts/stamps.py $a > gpurun_out/$TAG/stamps_$i.log 2>&1 \
    || { echo "stamps $a rc=$?"; tail -20 gpurun_out/$TAG/stamps_$i.log; exit 1; }
  echo "== $a"; grep -v amdgpu.ids gpurun_out/$TAG/stamps_$i.log
done
