#!/bin/bash
# group kernel: DPP softmax / wave sums, chained schedule 0 -- parity, stamps, sweep
set -o pipefail
mkdir -p gpurun_out/r02p
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread \
  -k "split or persistent or local_train or fullsize or golden or config or long" > gpurun_out/r02p/parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/r02p/parity.log; [ $rc -eq 0 ] || exit $rc
SL=$PWD/non-iid-distributed-learning-with-optimal-mixture-weights_amd/libfedsim_stamps.so
for c in "1 8 --chained" "2 2" "5 16"; do set -- $c
  echo "== stamps config $1 G $2 $3"
  FEDSIM_LIB=$SL $T 180 python -u scripts/stamps.py --config $1 --G $2 $3 || exit 1
done > gpurun_out/r02p/stamps.log 2>&1
echo "stamps rc=$?"; grep -v amdgpu.ids gpurun_out/r02p/stamps.log
for c in "1 8" "2 2" "4 2" "3 4" "5 16"; do set -- $c
  $T 180 python -u scripts/lt_sweep.py --config $1 --G $2 --reps 3 || exit 1
done > gpurun_out/r02p/sweep.log 2>&1
echo "sweep rc=$?"; grep -v amdgpu.ids gpurun_out/r02p/sweep.log
