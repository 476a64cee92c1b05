# p-solve / Z-GEMM: parity tests, then timings
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_experiment.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_mc_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/gpu_mc_tests.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
T="timeout -k 10 120 python -u scripts/mix_time.py"
$T 100 10 12800 1 && $T 1000 10 32000 1 && $T 10 2 6500 1 && $T 125 10 4000 1
