#!/bin/bash
# schedule 3 (image-fed forward, registers stage the next step's rows): parity, sweep, stamps
set -o pipefail
mkdir -p gpurun_out/r02ac
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread -k "split_schedules" \
  > gpurun_out/r02ac/matrix.log 2>&1; echo "matrix rc=$?"; grep -E "passed|failed|FAILED" gpurun_out/r02ac/matrix.log | head
FS_SP_SCHED=3 $T 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread \
  -k "(split or persistent or local_train or fullsize or golden or config) and not split_schedules" > gpurun_out/r02ac/parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -1 gpurun_out/r02ac/parity.log; [ $rc -eq 0 ] || exit $rc
for c in "2 2" "4 2" "3 4" "5 16" "1 8"; do set -- $c
  for sc in 2 3; do
    echo -n "sched $sc: "; FS_SP_SCHED=$sc $T 180 python -u scripts/lt_sweep.py --config $1 --G $2 --reps 3 || exit 1
  done
done > gpurun_out/r02ac/sweep.log 2>&1
echo "sweep rc=$?"; grep -v amdgpu.ids gpurun_out/r02ac/sweep.log
FS_SP_SCHED=3 FEDSIM_LIB=$PWD/non-iid-distributed-learning-with-optimal-mixture-weights_amd/libfedsim_stamps.so \
  $T 180 python -u scripts/stamps.py --config 2 --G 2 2>&1 | grep -v amdgpu.ids
