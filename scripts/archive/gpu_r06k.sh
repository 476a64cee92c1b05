#!/bin/bash
# round 6: stamps of the mb instances (read-ahead) vs the 16x16x4 ones at configs 2 and 5
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-r06k}
PKG=non-iid-distributed-learning-with-optimal-mixture-weights_amd
mkdir -p gpurun_out/$R
S=gpurun_out/$R/stamps.txt
L=$PWD/$PKG/libfedsim_stamps.so
for mb in off on; do
  FEDSIM_LIB=$L timeout -k 10 120 python -u scripts/stamps.py --config 2 --mb $mb >> $S 2>&1 || exit 1; echo "^ c2 mb $mb" >> $S
  FEDSIM_LIB=$L timeout -k 10 120 python -u scripts/stamps.py --config 5 --mb $mb >> $S 2>&1 || exit 1; echo "^ c5 mb $mb" >> $S
done
grep -v amdgpu.ids $S
