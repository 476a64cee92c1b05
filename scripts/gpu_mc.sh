# p-solve: parity tests, then per-step timing of the solvers at the config shapes
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "mix" --timeout 120 --timeout-method thread > gpurun_out/gpu_mc_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/gpu_mc_tests.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
T="timeout -k 10 120 python -u scripts/mix_time.py"
$T 100 10 12800 10 && \
$T 10 2 6500 10 && \
$T 64 7 6500 10 && \
$T 125 10 4000 10 && \
$T 1000 10 32000 1
