# p-solve: parity tests, then per-step timing of the multi-CU solver
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "mix" --timeout 120 --timeout-method thread > gpurun_out/gpu_mc_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/gpu_mc_tests.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
T="timeout -k 10 120 python -u scripts/mix_time.py"
$T 1000 10 32000 1 && \
$T 300 10 12800 1 && \
FS_MIX_SOLVER=mc $T 100 10 12800 2 && \
FS_MIX_SOLVER=mc $T 10 2 6500 2 && \
true
