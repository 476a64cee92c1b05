#!/bin/bash
# quad p-solve: stamps with and without its in-loop Z loads (libfedsim_probe_stamps.so: timing
# only, p is wrong), config 2 shape.   scripts/gpu_probe.sh <tag>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-probe}
mkdir -p gpurun_out/$TAG
OUT=gpurun_out/$TAG/quad_noload_probe.txt
: > $OUT
PKG=$PWD/non-iid-distributed-learning-with-optimal-mixture-weights_amd
run() {   # lib H label
  FEDSIM_LIB=$1 FS_MIX_PF_H=$2 timeout -k 10 120 python -u scripts/mix_time.py 100 10 12800 10 64 >> $OUT 2>&1 \
    || { echo "mix_time rc=$? ($3)"; tail -20 $OUT; exit 1; }
  echo "  ^ $3" >> $OUT
}
run $PKG/libfedsim_stamps.so 0 "stamps, default helpers" || exit 1
run $PKG/libfedsim_probe_stamps.so 0 "NO in-loop Z loads, default helpers" || exit 1
run $PKG/libfedsim_probe_stamps.so -1 "NO in-loop Z loads, no helpers" || exit 1
run $PKG/libfedsim.so 0 "shipped" || exit 1
grep -v amdgpu.ids $OUT
