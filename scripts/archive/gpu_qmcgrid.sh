#!/bin/bash
# qmc first-poll delay x helper lead grid at config 5's shape (N = 1000).   scripts/gpu_qmcgrid.sh <tag>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-qmcgrid}
mkdir -p gpurun_out/$TAG
OUT=gpurun_out/$TAG/grid.txt
: > $OUT
run() {   # lead delay
  FS_MIX_PF_LEAD=$1 FS_MIX_POLL_DELAY=$2 timeout -k 10 120 python -u scripts/mix_time.py 1000 10 32000 5 64 >> $OUT 2>&1 \
    || { echo "mix_time rc=$? (lead $1 delay $2)"; tail -20 $OUT; exit 1; }
  echo "  ^ lead $1 delay $2" >> $OUT
}
for rep in 1 2; do
  for l in ${LEADS:-7 8 9}; do
    for d in ${DELAYS:-10 14 18 22}; do run $l $d; done
  done
done
grep -v "amdgpu.ids\|requested" $OUT
