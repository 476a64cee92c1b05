# mixture-solve parity tests + per-step timing (+ phase stamps with the diagnostic build)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "mix" --timeout 120 --timeout-method thread > gpurun_out/gpu_mix_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/gpu_mix_tests.log
[ $rc -eq 0 ] || exit $rc
STAMPLIB=$PWD/non-iid-distributed-learning-with-optimal-mixture-weights_amd/libfedsim_stamps.so
timeout -k 10 120 python -u scripts/mix_time.py 100 10 12800 10 && \
timeout -k 10 120 python -u scripts/mix_time.py 10 2 6500 10 && \
FEDSIM_LIB=$STAMPLIB timeout -k 10 120 python -u scripts/mix_time.py 100 10 12800 10 && \
FEDSIM_LIB=$STAMPLIB timeout -k 10 120 python -u scripts/mix_time.py 10 2 6500 10 && \
FEDSIM_LIB=$STAMPLIB timeout -k 10 120 python -u scripts/stamps.py 100 && \
timeout -k 10 120 python -u scripts/lt_time.py 100 1 2 4
