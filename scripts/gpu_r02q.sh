#!/bin/bash
# group kernel schedules 2/3 (row loads interleaved into the backward): parity, sweep, stamps
set -o pipefail
mkdir -p gpurun_out/r02q
T="timeout -k 10"
for sc in 2 3; do
  FS_SP_SCHED=$sc $T 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "split or persistent or local_train or fullsize or golden" > gpurun_out/r02q/parity_$sc.log 2>&1
  rc=$?; echo "parity sched $sc rc=$rc"; tail -1 gpurun_out/r02q/parity_$sc.log; [ $rc -eq 0 ] || exit $rc
done
for c in "2 2" "4 2" "3 4" "5 16" "1 8"; do set -- $c
  for sc in 0 1 2 3; do
    [ $2 = 16 ] && [ $sc = 1 ] && continue; [ $2 = 16 ] && [ $sc = 3 ] && continue
    echo -n "sched $sc: "; FS_SP_SCHED=$sc $T 180 python -u scripts/lt_sweep.py --config $1 --G $2 --reps 3 || exit 1
  done
done > gpurun_out/r02q/sweep.log 2>&1
echo "sweep rc=$?"; grep -v amdgpu.ids gpurun_out/r02q/sweep.log
SL=$PWD/non-iid-distributed-learning-with-optimal-mixture-weights_amd/libfedsim_stamps.so
for c in "2 2 3" "2 2 2" "5 16 2"; do set -- $c
  echo "== stamps config $1 G $2 sched $3"
  FS_SP_SCHED=$3 FEDSIM_LIB=$SL $T 180 python -u scripts/stamps.py --config $1 --G $2 || exit 1
done > gpurun_out/r02q/stamps.log 2>&1
echo "stamps rc=$?"; grep -v amdgpu.ids gpurun_out/r02q/stamps.log
