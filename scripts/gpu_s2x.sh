#!/bin/bash
# chunked shuffles: full GPU suite, bench A/B (chunk 8 vs per round), kernel trace of the default
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r02s2x}; mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step pytest timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
tail -1 $O/gpu_tests.log
for k in 8 1 16; do
  FS_SHUFFLE_CHUNK=$k FS_BENCH_HOST_TIMES=1 step "bench chunk $k" timeout -k 10 300 python -u bench.py --steps 50 --no-fedamw-leg --no-cpu-baseline > $O/bench_k$k.json 2> $O/bench_k$k.err
  grep 'host us' $O/bench_k$k.err
done
step trace timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o tr --output-format csv -- python3 -u bench.py --steps 20 --warmup 2 --no-fedamw-leg --no-cpu-baseline > $O/trace.log 2>&1
