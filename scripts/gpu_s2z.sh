#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r02s2z}; mkdir -p $O
for ev in 0 1 0 1; do
  FS_BENCH_NO_EVENTS=$ev FS_BENCH_HOST_TIMES=1 timeout -k 10 300 python -u bench.py --steps 100 --no-fedamw-leg --no-cpu-baseline > $O/b_$ev.json 2> $O/b_$ev.err
  echo "noevents=$ev rc=$? $(grep 'host us' $O/b_$ev.err)"
done
