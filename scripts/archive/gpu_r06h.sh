#!/bin/bash
# round 6: stamps of the split form's mb instances vs the 16x16x4 ones (configs 2, 3, 1)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-r06h}
PKG=non-iid-distributed-learning-with-optimal-mixture-weights_amd
mkdir -p gpurun_out/$R
S=gpurun_out/$R/stamps.txt
L=$PWD/$PKG/libfedsim_stamps.so
for mb in off on; do
  FEDSIM_LIB=$L timeout -k 10 120 python -u scripts/stamps.py --config 2 --mb $mb >> $S 2>&1 || exit 1; echo "^ c2 mb $mb" >> $S
  FEDSIM_LIB=$L timeout -k 10 120 python -u scripts/stamps.py --config 3 --prox --mb $mb >> $S 2>&1 || exit 1; echo "^ c3 mb $mb" >> $S
  FEDSIM_LIB=$L timeout -k 10 120 python -u scripts/stamps.py --config 1 --mb $mb >> $S 2>&1 || exit 1; echo "^ c1 mb $mb" >> $S
done
grep -v amdgpu.ids $S
# launch A/B: mb with / without the pre-forward (SP_MB_PRE), and the 16x16x4 instances
S2=gpurun_out/$R/lt.txt
for k in 1 2; do
  for lib in libfedsim libfedsim_nopre; do
    L=$PWD/$PKG/$lib.so
    FEDSIM_LIB=$L timeout -k 10 120 python -u scripts/lt_sweep.py --config 2 --reg 0 --reps 30 --mb on >> $S2 2>&1 || exit 1; echo "^ c2 mb $lib" >> $S2
    FEDSIM_LIB=$L timeout -k 10 120 python -u scripts/lt_sweep.py --config 5 --reg 1 --reps 10 --mb on >> $S2 2>&1 || exit 1; echo "^ c5 mb $lib" >> $S2
    FEDSIM_LIB=$L timeout -k 10 120 python -u scripts/lt_sweep.py --config 3 --reg 0 --prox --reps 5 --mb on >> $S2 2>&1 || exit 1; echo "^ c3 mb $lib" >> $S2
  done
  timeout -k 10 120 python -u scripts/lt_sweep.py --config 2 --reg 0 --reps 30 --mb off >> $S2 2>&1 || exit 1; echo "^ c2 16x16x4" >> $S2
  timeout -k 10 120 python -u scripts/lt_sweep.py --config 5 --reg 1 --reps 10 --mb off >> $S2 2>&1 || exit 1; echo "^ c5 16x16x4" >> $S2
done
grep -v amdgpu.ids $S2
