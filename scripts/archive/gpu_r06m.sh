#!/bin/bash
# round 6: diagnostic -- the mb backward without its image reads / without its g reads (wrong results; timing only)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-r06m}
PKG=non-iid-distributed-learning-with-optimal-mixture-weights_amd
mkdir -p gpurun_out/$R
S=gpurun_out/$R/lt.txt
for k in 1 2; do
  for lib in libfedsim libfedsim_noxread libfedsim_nogread; do
    L=$PWD/$PKG/$lib.so
    FEDSIM_LIB=$L timeout -k 10 120 python -u scripts/lt_sweep.py --config 2 --reg 0 --reps 30 --mb on >> $S 2>&1 || exit 1; echo "^ c2 mb $lib" >> $S
    FEDSIM_LIB=$L timeout -k 10 120 python -u scripts/lt_sweep.py --config 5 --reg 1 --reps 10 --mb on >> $S 2>&1 || exit 1; echo "^ c5 mb $lib" >> $S
  done
done
grep -v amdgpu.ids $S
