#!/bin/bash
# final round-2 regression on the PMC-captured sources: tests, smoke, benches 2-5, kernel stats,
# config-1 experiment end to end
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r02z
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
rc=$?; tail -1 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
for c in 2 3 4 5; do
  A=""; [ $c = 5 ] && A="--steps 2 --warmup 1"; [ $c = 3 ] && A="--steps 5 --warmup 2"
  timeout -k 10 400 python -u bench.py --config $c $A > $OUT/bench_c$c.json 2> $OUT/bench_c$c.err; rc=$?
  echo "bench c$c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c2 -o c2 --output-format csv -- python3 -u bench.py --no-cpu-baseline > $OUT/prof_c2.log 2>&1
rc=$?; echo "prof c2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c3 -o c3 --output-format csv -- python3 -u bench.py --config 3 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/prof_c3.log 2>&1
rc=$?; echo "prof c3 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u run_experiment.py --dataset a9a --data-dir /nonexistent/ --result-dir gpurun_out/r02z/results > $OUT/exp_config1_a9a.log 2>&1
rc=$?; echo "exp rc=$rc"; tail -3 $OUT/exp_config1_a9a.log; exit $rc
