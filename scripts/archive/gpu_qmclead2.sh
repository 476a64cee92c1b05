#!/bin/bash
# qmc helper lead 6 vs 8 at N = 520 and 800 (C = 10), two reps.   scripts/gpu_qmclead2.sh <tag>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-qmclead2}
mkdir -p gpurun_out/$TAG
OUT=gpurun_out/$TAG/lead.txt
: > $OUT
run() {   # lead N NV
  FS_MIX_PF_LEAD=$1 timeout -k 10 120 python -u scripts/mix_time.py $2 10 $3 5 64 >> $OUT 2>&1 \
    || { echo "mix_time rc=$? (lead $1 N $2)"; tail -20 $OUT; exit 1; }
  echo "  ^ lead $1" >> $OUT
}
for rep in 1 2; do
  for l in 6 8; do run $l 520 12800; run $l 800 25600; done
done
grep -v "amdgpu.ids\|requested" $OUT
