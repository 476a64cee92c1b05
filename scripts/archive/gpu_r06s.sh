#!/bin/bash
# round 6: early-issue depths re-checked on the mb instances -- config 5 (SP_E1 4 / 6 / 8) and config 3 (prox depth SP_EP 1 / 2 / 4)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-r06s}
PKG=non-iid-distributed-learning-with-optimal-mixture-weights_amd
mkdir -p gpurun_out/$R
S=gpurun_out/$R/lt.txt
for k in 1 2; do
  for lib in libfedsim libfedsim_e4 libfedsim_e8; do
    FEDSIM_LIB=$PWD/$PKG/$lib.so timeout -k 10 120 python -u scripts/lt_sweep.py --config 5 --reg 1 --reps 10 >> $S 2>&1 || exit 1; echo "^ c5 $lib" >> $S
  done
  for lib in libfedsim libfedsim_ep4 libfedsim_ep1; do
    FEDSIM_LIB=$PWD/$PKG/$lib.so timeout -k 10 120 python -u scripts/lt_sweep.py --config 3 --reg 0 --prox --reps 5 >> $S 2>&1 || exit 1; echo "^ c3 $lib" >> $S
  done
done
grep -v amdgpu.ids $S
