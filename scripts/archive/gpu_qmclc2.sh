#!/bin/bash
# qmc lane width A/B over client counts (8 vs 4 clients per lane; default helpers).
#   scripts/gpu_qmclc2.sh <tag>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-qmclc2}
mkdir -p gpurun_out/$TAG
OUT=gpurun_out/$TAG/qmc_lane_ab2.txt
: > $OUT
run() {   # LC N C NV EP
  FS_MIX_QMC_LC=$1 timeout -k 10 120 python -u scripts/mix_time.py $2 $3 $4 $5 64 >> $OUT 2>&1 \
    || { echo "mix_time rc=$? (LC=$1 N=$2)"; tail -20 $OUT; exit 1; }
  echo "  ^ LC=$1" >> $OUT
}
for n in "300 10 12800 5" "300 4 12800 5" "520 10 12800 5" "1000 10 32000 5" "1000 4 32000 5"; do
  run 8 $n
  run 4 $n
done
run 8 1000 10 32000 5
cat $OUT
