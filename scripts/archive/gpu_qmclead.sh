#!/bin/bash
# qmc helper lead sweep with the first-poll delay, N = 1000 and N = 300.   scripts/gpu_qmclead.sh <tag>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-qmclead}
mkdir -p gpurun_out/$TAG
OUT=gpurun_out/$TAG/lead.txt
: > $OUT
run() {   # lead N NV
  FS_MIX_PF_LEAD=$1 timeout -k 10 120 python -u scripts/mix_time.py $2 10 $3 5 64 >> $OUT 2>&1 \
    || { echo "mix_time rc=$? (lead $1 N $2)"; tail -20 $OUT; exit 1; }
  echo "  ^ lead $1" >> $OUT
}
for rep in 1 2; do
  for l in 0 8 10 12 16; do run $l 1000 32000; done
done
for l in 0 8 10 12; do run $l 300 12800; done
grep -v "amdgpu.ids\|requested" $OUT
