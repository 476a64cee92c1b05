#!/bin/bash
# full regression: every -m gpu test, smoke(), bench configs 2 and 5
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r02l
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
rc=$?; tail -2 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err; rc=$?; tail -1 $OUT/bench_c2.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --config 5 --steps 2 --warmup 1 > $OUT/bench_c5.json 2> $OUT/bench_c5.err; rc=$?
tail -1 $OUT/bench_c5.json; exit $rc
