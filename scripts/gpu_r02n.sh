#!/bin/bash
# config-2 p-solve: multi-CU slice width x exchange form x Z issue point
set -o pipefail
mkdir -p gpurun_out/r02n
T="timeout -k 10"
for S in 64 32 16 8; do for h in 1 2; do for z in 0 2; do
  echo "== S $S hops $h zat $z"
  FS_MIX_SOLVER=mc FS_MIX_MC_S=$S FS_MIX_MC_HOPS=$h FS_MIX_MC_ZAT=$z $T 120 python -u scripts/mix_time.py 100 10 12800 2 || exit 1
done; done; done > gpurun_out/r02n/time.log 2>&1
echo "time rc=$?"; grep -v amdgpu.ids gpurun_out/r02n/time.log | grep -v "solver requested" | sed -e 's/N=100 C=10 n_val=12800 epochs=2: //' -e 's/mix_z.*mix_solve/mix_solve/'
