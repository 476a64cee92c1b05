#!/bin/bash
# Round 2, third GPU pass: schedule variants of the split-group kernel (FS_SP_SCHED), config tests.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r02c
mkdir -p $OUT
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
for sc in 0 1 2; do
  for c in 2 3 4; do
    FS_SP_SCHED=$sc timeout -k 10 180 python -u scripts/lt_sweep.py --config $c --G 0 > $OUT/s.tmp 2>&1; rc=$?
    grep -v amdgpu.ids $OUT/s.tmp | sed "s/^/sched=$sc /" | tee -a $OUT/sched.log; ok $rc || exit $rc
  done
  FS_SP_SCHED=$sc timeout -k 10 180 python -u scripts/lt_sweep.py --config 1 --G 4,8 --reps 3 > $OUT/s.tmp 2>&1; rc=$?
  grep -v amdgpu.ids $OUT/s.tmp | sed "s/^/sched=$sc /" | tee -a $OUT/sched.log; ok $rc || exit $rc
done
for sc in 1 2; do
  FEDSIM_LIB=$PWD/non-iid-distributed-learning-with-optimal-mixture-weights_amd/libfedsim_stamps.so FS_SP_SCHED=$sc \
    timeout -k 10 180 python -u scripts/stamps.py --config 2 > $OUT/s.tmp 2>&1; rc=$?
  grep -v amdgpu.ids $OUT/s.tmp | sed "s/^/sched=$sc /" | tee -a $OUT/stamps.log; ok $rc || exit $rc
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -v --timeout 300 --timeout-method thread \
  > $OUT/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" $OUT/tests.log | tail; ok $rc || exit $rc
exit 0
