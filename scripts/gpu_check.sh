# Quick GPU iteration: gpu tests + one bench line (+ optional extra bench args in $BENCH_ARGS)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline $BENCH_ARGS > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
exit $rc
