#!/bin/bash
# split local-training stamps with and without the in-loop row stream (libfedsim_split_probe_stamps.so,
# scripts/build_split_probe.sh: timing only), configs 2 and 5.   scripts/gpu_split_probe.sh <tag>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-split_probe}
mkdir -p gpurun_out/$TAG
OUT=gpurun_out/$TAG/split_noload_probe.txt
: > $OUT
PKG=$PWD/non-iid-distributed-learning-with-optimal-mixture-weights_amd
for c in 2 5; do
  for lib in libfedsim_stamps.so libfedsim_split_probe_stamps.so; do
    echo "== config $c, $lib" >> $OUT
    FEDSIM_LIB=$PKG/$lib timeout -k 10 150 python -u scripts/stamps.py --config $c >> $OUT 2>&1 \
      || { echo "stamps rc=$? (config $c $lib)"; tail -20 $OUT; exit 1; }
  done
done
grep -v amdgpu.ids $OUT
