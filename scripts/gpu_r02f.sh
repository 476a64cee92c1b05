#!/bin/bash
# Round 2, sixth GPU pass: 4-wave workgroups, two per CU (two client chains per CU).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r02f
mkdir -p $OUT
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "split or persistent or local_train or fullsize or timeout" \
  -v --timeout 120 --timeout-method thread > $OUT/parity.log 2>&1; rc=$?; echo "parity rc=$rc"; tail -3 $OUT/parity.log; ok $rc || exit $rc
run() { timeout -k 10 180 python -u scripts/lt_sweep.py "$@" > $OUT/s.tmp 2>&1; local rc=$?; grep -v amdgpu.ids $OUT/s.tmp | tee -a $OUT/sweep.log; return $rc; }
run --config 2 --G 2,4,8 || exit 1
FS_SP_SCHED=1 run --config 2 --G 4 || exit 1
run --config 4 --G 2,4,8 || exit 1
run --config 3 --G 4,8 || exit 1
run --config 5 --G 16 || exit 1
run --config 1 --G 4,8,16 --reps 3 || exit 1
FS_SPLIT_NW=8 run --config 1 --G 8 --reps 3 || exit 1
FEDSIM_LIB=$PWD/non-iid-distributed-learning-with-optimal-mixture-weights_amd/libfedsim_stamps.so \
  timeout -k 10 180 python -u scripts/stamps.py --config 2 --G 4 > $OUT/s.tmp 2>&1; rc=$?
grep -v amdgpu.ids $OUT/s.tmp | tee -a $OUT/stamps.log; ok $rc || exit $rc
exit 0
