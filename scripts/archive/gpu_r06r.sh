#!/bin/bash
# round 6: narrow chained instances' index fetch handed through LDS by the last wave (SP_NARROW_LDSF) -- tests, config 1 A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-r06r}
PKG=non-iid-distributed-learning-with-optimal-mixture-weights_amd
mkdir -p gpurun_out/$R
timeout -k 10 600 python -u -m pytest tests/test_gpu_mb.py tests/test_gpu_split_early.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$R/tests.log 2>&1
rc=$?
tail -3 gpurun_out/$R/tests.log
[ $rc -eq 0 ] || exit $rc
S=gpurun_out/$R/lt.txt
for k in 1 2; do
  for lib in libfedsim libfedsim_noldsf; do
    L=$PWD/$PKG/$lib.so
    FEDSIM_LIB=$L timeout -k 10 120 python -u scripts/lt_sweep.py --config 1 --reg 1 --reps 10 >> $S 2>&1 || exit 1; echo "^ c1 mb $lib" >> $S
    FEDSIM_LIB=$L timeout -k 10 120 python -u scripts/lt_sweep.py --config 1 --reg 1 --reps 10 --mb off >> $S 2>&1 || exit 1; echo "^ c1 16x16x4 $lib" >> $S
  done
done
grep -v amdgpu.ids $S
