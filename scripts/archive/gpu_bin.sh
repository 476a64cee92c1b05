#!/bin/bash
# The one-wave binary p-solver on the GPU box: its tests, then time per step at config 1's
# shape (N = 10, C = 2, n_val = 3256, 2 epochs = 408 steps per launch) against wave / quad.
#   bash scripts/gpu_bin.sh <tag>
set -o pipefail
tag=${1:-bin}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
    -k "mix_solve or config1" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -3 $out/tests.log
for s in bin quad wave; do
  for e in 0 1; do
    FS_MIX_SOLVER=$s FS_MIX_EXACT=$e timeout -k 10 120 python -u scripts/mix_time.py 10 2 3256 2 >> $out/time.log 2>&1 || exit 1
  done
done
FS_MIX_SOLVER=bin timeout -k 10 120 python -u scripts/mix_time.py 16 2 32000 2 >> $out/time.log 2>&1 || exit 1
cat $out/time.log
