#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r02s2ab}; mkdir -p $O
for a in "20 3" "20 3" "20 10" "100 3" "20 3"; do set -- $a
  FS_BENCH_HOST_TIMES=1 timeout -k 10 300 python -u bench.py --steps $1 --warmup $2 --no-fedamw-leg --no-cpu-baseline > $O/b.json 2> $O/b.err
  echo "steps $1 warmup $2 rc=$? $(grep 'host us' $O/b.err)"
done
