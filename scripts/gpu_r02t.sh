#!/bin/bash
# prox anchor from memory: parity + FedProx sweeps
set -o pipefail
mkdir -p gpurun_out/r02t
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread \
  -k "split or persistent or local_train or fullsize or golden or config or long or prox" > gpurun_out/r02t/parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -1 gpurun_out/r02t/parity.log; [ $rc -eq 0 ] || exit $rc
for c in "3 1,4" "2 1,2" "5 1,16" "4 1,2"; do set -- $c
  $T 240 python -u scripts/lt_sweep.py --config $1 --G $2 --prox --reps 3 || exit 1
done > gpurun_out/r02t/sweep.log 2>&1
echo "sweep rc=$?"; grep -v amdgpu.ids gpurun_out/r02t/sweep.log
