#!/bin/bash
# Round-end check: GPU suite, smoke, default bench line (config 2, + CPU baseline), rocprofv3
# kernel stats of the default bench, config 4 bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-s2final}; mkdir -p $O
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step pytest timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
tail -1 $O/gpu_tests.log
step smoke timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step bench_c2 timeout -k 10 300 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err
step prof_c2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 --output-format csv -- python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_c2.log 2>&1
step bench_c4 timeout -k 10 300 python -u bench.py --config 4 > $O/bench_c4.json 2> $O/bench_c4.err
