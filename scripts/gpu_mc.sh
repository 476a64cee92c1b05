# multi-CU p-solve: parity tests, then per-step timing vs the register solver
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "mix" --timeout 120 --timeout-method thread > gpurun_out/gpu_mc_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/gpu_mc_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/mix_time.py 100 10 12800 10 && \
FS_MIX_SOLVER=reg timeout -k 10 120 python -u scripts/mix_time.py 100 10 12800 10 && \
FS_MIX_MC_S=16 timeout -k 10 120 python -u scripts/mix_time.py 100 10 12800 10 && \
FS_MIX_MC_S=32 timeout -k 10 120 python -u scripts/mix_time.py 100 10 12800 10 && \
FS_MIX_SOLVER=mc FS_MIX_MC_S=8 timeout -k 10 120 python -u scripts/mix_time.py 10 2 6500 10 && \
timeout -k 10 120 python -u scripts/mix_time.py 10 2 6500 10 && \
timeout -k 10 120 python -u scripts/mix_time.py 1000 10 32000 1 && \
FS_MIX_MC_S=64 timeout -k 10 120 python -u scripts/mix_time.py 1000 10 32000 1
