#!/bin/bash
# multi-CU p-solve: Z-slice issue point x exchange form -- parity + step time
set -o pipefail
mkdir -p gpurun_out/r02i
T="timeout -k 10"
for z in 1 2; do
  FS_MIX_MC_ZAT=$z $T 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
    -k "multi_cu" > gpurun_out/r02i/parity_z$z.log 2>&1 || { echo "parity z$z failed"; tail -5 gpurun_out/r02i/parity_z$z.log; exit 1; }
  tail -1 gpurun_out/r02i/parity_z$z.log
done
for cfg in "1000 10 12800 2" "300 4 4000 10" "100 10 12800 2"; do
  for h in 1 2; do for z in 0 1 2; do
    [ $h = 1 ] && [ $z = 1 ] && continue
    echo "== $cfg hops $h zat $z"
    FS_MIX_SOLVER=mc FS_MIX_MC_HOPS=$h FS_MIX_MC_ZAT=$z $T 120 python -u scripts/mix_time.py $cfg || exit 1
  done; done
done > gpurun_out/r02i/time.log 2>&1
echo "time rc=$?"; grep -v amdgpu.ids gpurun_out/r02i/time.log | grep -v "solver requested"
