#!/bin/bash
# round 6: narrow chained instances with the index / label fetch at the step's top (SP_NARROW_TOP) A/B, config 1
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-r06p}
PKG=non-iid-distributed-learning-with-optimal-mixture-weights_amd
mkdir -p gpurun_out/$R
S=gpurun_out/$R/lt.txt
for k in 1 2; do
  for lib in libfedsim libfedsim_ntop; do
    L=$PWD/$PKG/$lib.so
    FEDSIM_LIB=$L timeout -k 10 120 python -u scripts/lt_sweep.py --config 1 --reg 1 --reps 10 >> $S 2>&1 || exit 1; echo "^ c1 mb $lib" >> $S
    FEDSIM_LIB=$L timeout -k 10 120 python -u scripts/lt_sweep.py --config 1 --reg 1 --reps 10 --mb off >> $S 2>&1 || exit 1; echo "^ c1 16x16x4 $lib" >> $S
  done
done
grep -v amdgpu.ids $S
