# p-solve for N > 256 clients: multi-CU solver vs the single-workgroup global-memory solver
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python -u scripts/mix_time.py 1000 10 32000 1 && \
FS_MIX_SOLVER=global timeout -k 10 120 python -u scripts/mix_time.py 1000 10 3200 1 && \
timeout -k 10 120 python -u scripts/mix_time.py 300 10 12800 1 && \
FS_MIX_SOLVER=global timeout -k 10 120 python -u scripts/mix_time.py 300 10 12800 1 && \
FS_MIX_SOLVER=mc timeout -k 10 120 python -u scripts/mix_time.py 200 10 12800 1 && \
timeout -k 10 120 python -u scripts/mix_time.py 200 10 12800 1
