#!/bin/bash
# group kernel schedules 4/5 + the schedule parity matrix
set -o pipefail
mkdir -p gpurun_out/r02w
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread \
  -k "split_schedules" > gpurun_out/r02w/sched_matrix.log 2>&1
echo "matrix rc=$?"; grep -E "passed|failed|FAILED" gpurun_out/r02w/sched_matrix.log | head -30
for sc in 4 5; do
  FS_SP_SCHED=$sc $T 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "(split or persistent or local_train or fullsize) and not split_schedules" > gpurun_out/r02w/parity_$sc.log 2>&1
  rc=$?; echo "parity sched $sc rc=$rc"; tail -1 gpurun_out/r02w/parity_$sc.log; [ $rc -eq 0 ] || exit $rc
done
for c in "2 2" "4 2" "3 4" "5 16" "1 8"; do set -- $c
  for sc in 2 4 5; do
    echo -n "sched $sc: "; FS_SP_SCHED=$sc $T 180 python -u scripts/lt_sweep.py --config $1 --G $2 --reps 3 || exit 1
  done
done > gpurun_out/r02w/sweep.log 2>&1
echo "sweep rc=$?"; grep -v amdgpu.ids gpurun_out/r02w/sweep.log
