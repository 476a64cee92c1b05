#!/bin/bash
# two-hop multi-CU p-solve exchange: parity + step time vs one hop
set -o pipefail
mkdir -p gpurun_out/r02h
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "mix" \
  > gpurun_out/r02h/parity.log 2>&1; echo "parity rc=$?"; tail -3 gpurun_out/r02h/parity.log
grep -q " passed" gpurun_out/r02h/parity.log && ! grep -q "FAILED\|Error" gpurun_out/r02h/parity.log || exit 1
for cfg in "1000 10 12800 2" "2000 2 4000 4" "300 4 4000 10" "100 10 12800 2"; do
  for h in 1 2; do
    echo "== $cfg hops $h"
    FS_MIX_SOLVER=mc FS_MIX_MC_HOPS=$h $T 120 python -u scripts/mix_time.py $cfg || exit 1
  done
done > gpurun_out/r02h/time.log 2>&1
echo "time rc=$?"; grep -v amdgpu.ids gpurun_out/r02h/time.log
