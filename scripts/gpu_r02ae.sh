#!/bin/bash
# row-split p-solver: parity, then per-step timing against the register solver
set -o pipefail
mkdir -p gpurun_out/r02ae
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -m gpu -k "mix_solve" > gpurun_out/r02ae/tests.log 2>&1 || { tail -40 gpurun_out/r02ae/tests.log; exit 1; }
tail -3 gpurun_out/r02ae/tests.log
for shape in "100 10 12800 2" "10 2 1000 20" "200 4 6400 2" "60 8 6400 2"; do
  timeout -k 10 60 python scripts/mix_time.py $shape 2>&1 | tee -a gpurun_out/r02ae/time.log || exit 1
  for rw in 1 2 4; do
    FS_MIX_SOLVER=rows FS_MIX_ROWS_RW=$rw timeout -k 10 60 python scripts/mix_time.py $shape 2>&1 \
      | sed "s/^/rw=$rw /" | tee -a gpurun_out/r02ae/time.log || exit 1
  done
done
