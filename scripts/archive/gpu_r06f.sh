#!/bin/bash
# round 6: the split form's poll skip (SP_POLL_SKIP) A/B at configs 1, 2, 3, 5 (launch times)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-r06f}
PKG=non-iid-distributed-learning-with-optimal-mixture-weights_amd
mkdir -p gpurun_out/$R
S=gpurun_out/$R/lt.txt
for k in 1 2; do
  for lib in libfedsim_noskip libfedsim; do
    L=$PWD/$PKG/$lib.so
    FEDSIM_LIB=$L timeout -k 10 120 python -u scripts/lt_sweep.py --config 2 --reg 0 --reps 30 >> $S 2>&1 || exit 1; echo "^ c2 $lib" >> $S
    FEDSIM_LIB=$L timeout -k 10 120 python -u scripts/lt_sweep.py --config 5 --reg 1 --reps 10 >> $S 2>&1 || exit 1; echo "^ c5 $lib" >> $S
    FEDSIM_LIB=$L timeout -k 10 120 python -u scripts/lt_sweep.py --config 1 --reg 1 --reps 10 >> $S 2>&1 || exit 1; echo "^ c1 $lib" >> $S
    FEDSIM_LIB=$L timeout -k 10 120 python -u scripts/lt_sweep.py --config 3 --reg 0 --prox --reps 5 >> $S 2>&1 || exit 1; echo "^ c3 $lib" >> $S
  done
done
grep -v amdgpu.ids $S
