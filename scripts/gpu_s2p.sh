#!/bin/bash
# host enqueue time per round (config 2 FedAvg) + a Python profile of the timed loop
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r02s2p}; mkdir -p $O
FS_BENCH_HOST_TIMES=1 timeout -k 10 200 python -u bench.py --steps 100 --warmup 3 --no-fedamw-leg --no-cpu-baseline > $O/b.json 2> $O/b.err; echo "bench rc=$?"
grep 'host us' $O/b.err
FS_BENCH_HOST_TIMES=1 timeout -k 10 300 python -u -m cProfile -s tottime bench.py --steps 100 --warmup 3 --no-fedamw-leg --no-cpu-baseline > $O/prof.txt 2> $O/prof.err; echo "cprofile rc=$?"
grep 'host us' $O/prof.err
