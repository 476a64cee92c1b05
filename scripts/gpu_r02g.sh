#!/bin/bash
# reg2 p-solver: parity (every solver variant) + step time vs the one-row-per-wave solver
set -o pipefail
mkdir -p gpurun_out/r02g
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "mix" \
  > gpurun_out/r02g/parity.log 2>&1; echo "parity rc=$?"; tail -3 gpurun_out/r02g/parity.log
grep -q " passed" gpurun_out/r02g/parity.log && ! grep -q "FAILED\|Error" gpurun_out/r02g/parity.log || exit 1
for cfg in "10 2 203 100" "100 10 12800 10" "256 4 4000 10" "60 8 4000 10"; do
  for v in reg reg2 reg2-select; do
    if [ $v = reg2-select ]; then export FS_MIX_SWAP=0; sv=reg2; else unset FS_MIX_SWAP; sv=$v; fi
    echo "== $cfg $v"
    FS_MIX_SOLVER=$sv $T 120 python -u scripts/mix_time.py $cfg || exit 1
  done
done > gpurun_out/r02g/time.log 2>&1
echo "time rc=$?"; cat gpurun_out/r02g/time.log
