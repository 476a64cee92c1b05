#!/bin/bash
# p-solve phase stamps (diagnostic build libfedsim_stamps.so, s_memtime of wave 0 of workgroup 0)
# at config 5's qmc shape with and without helpers, and config 2's quad shape.
#   scripts/gpu_mixstamps.sh <tag>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-mixst}
mkdir -p gpurun_out/$TAG
OUT=gpurun_out/$TAG/mix_stamps.txt
: > $OUT
LIB=$PWD/non-iid-distributed-learning-with-optimal-mixture-weights_amd/libfedsim_stamps.so
run() {   # H LEAD N C NV EP
  FEDSIM_LIB=$LIB FS_MIX_PF_H=$1 FS_MIX_PF_LEAD=$2 timeout -k 10 120 python -u scripts/mix_time.py $3 $4 $5 $6 64 >> $OUT 2>&1 \
    || { echo "mix_time rc=$? (H=$1 lead=$2 N=$3)"; tail -20 $OUT; exit 1; }
  echo "  ^ H=$1 lead=$2" >> $OUT
}
run 0 0 1000 10 32000 5
run -1 0 1000 10 32000 5
run 0 0 100 10 12800 10
cat $OUT
