#!/bin/bash
# chained config 1: per-phase stamps at G = 4, 8, 16 and schedules 0 / 1
set -o pipefail
mkdir -p gpurun_out/r02o
T="timeout -k 10"
SL=$PWD/non-iid-distributed-learning-with-optimal-mixture-weights_amd/libfedsim_stamps.so
for G in 4 8 16; do for sc in 0 1; do
  [ $G = 16 ] && [ $sc = 1 ] && continue
  echo "== stamps config 1 chained G $G sched $sc"
  FS_SP_SCHED=$sc FEDSIM_LIB=$SL $T 180 python -u scripts/stamps.py --config 1 --G $G --chained || exit 1
done; done > gpurun_out/r02o/stamps.log 2>&1
echo "stamps rc=$?"; grep -v amdgpu.ids gpurun_out/r02o/stamps.log
