#!/bin/bash
# row-split p-solver: rows per workgroup x ring-refill position, config 2 and config 5 shapes
set -o pipefail
mkdir -p gpurun_out/r02af
export PYTHONUNBUFFERED=1
FS_MIX_SOLVER=rows FS_MIX_ROWS_RW=8 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py -m gpu -k "mix_solve_rows" > gpurun_out/r02af/tests.log 2>&1 || { tail -30 gpurun_out/r02af/tests.log; exit 1; }
tail -2 gpurun_out/r02af/tests.log
for shape in "100 10 12800 2" "1000 10 3200 1"; do
  timeout -k 10 60 python scripts/mix_time.py $shape 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r02af/time.log || exit 1
  for early in 0 1; do for rw in 2 4 8; do
    FS_MIX_SOLVER=rows FS_MIX_ROWS_RW=$rw FS_MIX_ROWS_EARLY=$early timeout -k 10 60 python scripts/mix_time.py $shape 2>&1 \
      | grep -v amdgpu.ids | sed "s/^/rw=$rw early=$early /" | tee -a gpurun_out/r02af/time.log || exit 1
  done; done
done
