#!/bin/bash
# what blocks the host per round: host-replayed shuffles; kernarg placement
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r02s2q}; mkdir -p $O
run() { local name=$1; shift; env "$@" FS_BENCH_HOST_TIMES=1 timeout -k 10 200 python -u bench.py --steps 100 --warmup 3 --no-fedamw-leg --no-cpu-baseline $EXTRA > $O/$name.json 2> $O/$name.err; echo "$name rc=$? $(grep 'host us' $O/$name.err)"; }
run base X=1
EXTRA=--host-shuffle run hostshuf X=1
EXTRA= run kern0 HIP_FORCE_DEV_KERNARG=0
EXTRA= run kern1 HIP_FORCE_DEV_KERNARG=1
EXTRA=--host-shuffle timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace -d $O/trace -o tr --output-format csv -- python3 -u bench.py --steps 10 --warmup 2 --no-fedamw-leg --no-cpu-baseline --host-shuffle > $O/trace.log 2>&1; echo "trace rc=$?"
