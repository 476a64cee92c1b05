#!/bin/bash
# one-wave p-solver: parity + step time vs the register solver
set -o pipefail
mkdir -p gpurun_out/r02u
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread \
  -k "mix or fedamw or golden or config1" > gpurun_out/r02u/parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -3 gpurun_out/r02u/parity.log; [ $rc -eq 0 ] || exit $rc
for cfg in "10 2 6512 10" "16 4 4000 10" "5 3 4000 10"; do for v in wave reg; do
  echo "== $cfg $v"; FS_MIX_SOLVER=$v $T 120 python -u scripts/mix_time.py $cfg || exit 1
done; done > gpurun_out/r02u/time.log 2>&1
echo "time rc=$?"; grep -v amdgpu.ids gpurun_out/r02u/time.log | sed -e 's/mix_z.*mix_solve/mix_solve/'
