#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r02s2s}; mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step host_calls timeout -k 10 200 python -u scripts/host_calls.py > $O/host_calls.log 2>&1; grep -v amdgpu.ids $O/host_calls.log
FS_SEED_COPY=1 step host_calls_copy timeout -k 10 200 python -u scripts/host_calls.py > $O/host_calls_copy.log 2>&1; grep -v amdgpu.ids $O/host_calls_copy.log
step pytest timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
tail -1 $O/gpu_tests.log
step bench timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err
cut -c1-300 $O/bench_c2.json
