# GPU tests, then bench lines for each shuffle mode (+ optional extra bench args in $BENCH_ARGS)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline $BENCH_ARGS > gpurun_out/bench_dev.json 2> gpurun_out/bench_dev.err
rc=$?; echo "bench(device shuffle) rc=$rc"; cat gpurun_out/bench_dev.json; tail -3 gpurun_out/bench_dev.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline --host-shuffle $BENCH_ARGS > gpurun_out/bench_host.json 2> gpurun_out/bench_host.err
rc=$?; echo "bench(host shuffle) rc=$rc"; cat gpurun_out/bench_host.json; tail -3 gpurun_out/bench_host.err
exit $rc
