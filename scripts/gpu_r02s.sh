#!/bin/bash
# FedProx group-kernel widths at configs 3 and 2 (planner: prox -> G = 1 when 2N >= CUs)
set -o pipefail
mkdir -p gpurun_out/r02s
T="timeout -k 10"
for c in "3 1,4,8" "2 1,2,4" "5 1,16"; do set -- $c
  $T 240 python -u scripts/lt_sweep.py --config $1 --G $2 --prox --reps 3 || exit 1
done > gpurun_out/r02s/sweep.log 2>&1
echo "sweep rc=$?"; grep -v amdgpu.ids gpurun_out/r02s/sweep.log
