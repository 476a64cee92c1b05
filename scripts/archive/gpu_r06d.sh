#!/bin/bash
# round 6: the double-buffered instance's early row issue depth (DB_E1 variants) at configs 2 and 5
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-r06d}
PKG=non-iid-distributed-learning-with-optimal-mixture-weights_amd
mkdir -p gpurun_out/$R
S=gpurun_out/$R/lt.txt
for k in 1 2; do
  for lib in libfedsim_dbe0 libfedsim_dbe2 libfedsim_dbe4 libfedsim; do
    for d in on; do
      FEDSIM_LIB=$PWD/$PKG/$lib.so timeout -k 10 120 python -u scripts/lt_sweep.py --config 2 --reg 0 --reps 30 --dbuf $d >> $S 2>&1 || exit 1; echo "^ c2 $lib dbuf $d" >> $S
      FEDSIM_LIB=$PWD/$PKG/$lib.so timeout -k 10 120 python -u scripts/lt_sweep.py --config 5 --reg 1 --reps 10 --dbuf $d >> $S 2>&1 || exit 1; echo "^ c5 $lib dbuf $d" >> $S
    done
  done
  timeout -k 10 120 python -u scripts/lt_sweep.py --config 2 --reg 0 --reps 30 --dbuf off >> $S 2>&1 || exit 1; echo "^ c2 split" >> $S
  timeout -k 10 120 python -u scripts/lt_sweep.py --config 5 --reg 1 --reps 10 --dbuf off >> $S 2>&1 || exit 1; echo "^ c5 split" >> $S
done
grep -v amdgpu.ids $S
