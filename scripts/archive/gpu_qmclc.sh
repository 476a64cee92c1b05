#!/bin/bash
# qmc lane width A/B at config 5's p-solve shape (N = 1000, C = 10, n_val = 32,000): 8 clients per
# lane (K = 8, default) vs 4 (K = 16), over helper counts/leads; then the stamps of both and of
# config 2's quad.   scripts/gpu_qmclc.sh <tag>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-qmclc}
mkdir -p gpurun_out/$TAG
OUT=gpurun_out/$TAG/qmc_lane_ab.txt
: > $OUT
LIB=$PWD/non-iid-distributed-learning-with-optimal-mixture-weights_amd/libfedsim_stamps.so
run() {   # LC H LEAD N C NV EP [lib]
  env ${8:+FEDSIM_LIB=$8} FS_MIX_QMC_LC=$1 FS_MIX_PF_H=$2 FS_MIX_PF_LEAD=$3 timeout -k 10 120 python -u scripts/mix_time.py $4 $5 $6 $7 64 \
    >> $OUT 2>&1 || { echo "mix_time rc=$? (LC=$1 H=$2 lead=$3 N=$4)"; tail -20 $OUT; exit 1; }
  echo "  ^ LC=$1 H=$2 lead=$3 ${8:+stamps}" >> $OUT
}
run 0 0 0 1000 10 32000 5
run 4 0 0 1000 10 32000 5
run 4 16 6 1000 10 32000 5
run 4 16 10 1000 10 32000 5
run 4 8 6 1000 10 32000 5
run 4 -1 0 1000 10 32000 5
run 0 0 0 1000 10 32000 5 $LIB
run 4 0 0 1000 10 32000 5 $LIB
run 0 0 0 100 10 12800 10
run 0 0 0 100 10 12800 10 $LIB
cat $OUT
