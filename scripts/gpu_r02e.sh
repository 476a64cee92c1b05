#!/bin/bash
# Round 2, fifth GPU pass: the image-first schedule (FS_SP_SCHED=3): parity of every split
# width under it, then the sweep against schedule 1 and its stamps.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r02e
mkdir -p $OUT
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
FS_SP_SCHED=3 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "split or persistent or local_train or fullsize or timeout" \
  -v --timeout 120 --timeout-method thread > $OUT/parity3.log 2>&1; rc=$?; echo "parity sched3 rc=$rc"; tail -3 $OUT/parity3.log; ok $rc || exit $rc
for sc in 1 3; do
  for c in 2 4 5; do
    FS_SP_SCHED=$sc timeout -k 10 180 python -u scripts/lt_sweep.py --config $c --G 0 > $OUT/s.tmp 2>&1; rc=$?
    grep -v amdgpu.ids $OUT/s.tmp | sed "s/^/sched=$sc /" | tee -a $OUT/sched.log; ok $rc || exit $rc
  done
  FS_SP_SCHED=$sc timeout -k 10 180 python -u scripts/lt_sweep.py --config 3 --G 4 > $OUT/s.tmp 2>&1; rc=$?
  grep -v amdgpu.ids $OUT/s.tmp | sed "s/^/sched=$sc /" | tee -a $OUT/sched.log; ok $rc || exit $rc
  FS_SP_SCHED=$sc timeout -k 10 180 python -u scripts/lt_sweep.py --config 1 --G 8 --reps 3 > $OUT/s.tmp 2>&1; rc=$?
  grep -v amdgpu.ids $OUT/s.tmp | sed "s/^/sched=$sc /" | tee -a $OUT/sched.log; ok $rc || exit $rc
done
for c in 2 5; do
  FEDSIM_LIB=$PWD/non-iid-distributed-learning-with-optimal-mixture-weights_amd/libfedsim_stamps.so FS_SP_SCHED=3 \
    timeout -k 10 180 python -u scripts/stamps.py --config $c > $OUT/s.tmp 2>&1; rc=$?
  grep -v amdgpu.ids $OUT/s.tmp | sed "s/^/sched=3 /" | tee -a $OUT/stamps.log; ok $rc || exit $rc
done
exit 0
