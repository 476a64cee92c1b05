#!/bin/bash
# Round-5 phase stamps (diagnostic build): p-solve (qmc at config 5's shape, quad at config 2's) with
# the shipped tuning, then the local-training forms at configs 2, 4 and 5.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-stamps_r05}
mkdir -p gpurun_out/$R
LIBS=$PWD/non-iid-distributed-learning-with-optimal-mixture-weights_amd/libfedsim_stamps.so
for a in "1000 10 32000 5" "100 10 12800 10"; do
  FEDSIM_LIB=$LIBS timeout -k 10 180 python -u scripts/mix_time.py $a >> gpurun_out/$R/mix.log 2>&1 \
    || { echo "mix $a rc=$?"; tail -20 gpurun_out/$R/mix.log; exit 1; }
done
grep -v amdgpu.ids gpurun_out/$R/mix.log
bash scripts/gpu_stamps.sh $R "--config 2" "--config 2 --pipe --G 2" "--config 4 --pipe --G 2" "--config 4 --pair --G 4" \
  "--config 5" "--config 5 --pipe --G 16"
