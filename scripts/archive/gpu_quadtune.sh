#!/bin/bash
# quad (loader form) helper count / lead sweep at config 2's p-solve shape.   scripts/gpu_quadtune.sh <tag>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-quadtune}
mkdir -p gpurun_out/$TAG
OUT=gpurun_out/$TAG/tune.txt
: > $OUT
run() {   # H LEAD
  FS_MIX_PF_H=$1 FS_MIX_PF_LEAD=$2 timeout -k 10 120 python -u scripts/mix_time.py 100 10 12800 10 64 >> $OUT 2>&1 \
    || { echo "mix_time rc=$? ($1 $2)"; tail -20 $OUT; exit 1; }
  echo "  ^ H=$1 lead=$2" >> $OUT
}
for rep in 1 2; do
  for hl in "0 0" "-1 0" "8 0" "16 0" "4 8" "4 24" "8 24"; do run $hl; done
done
grep -v "amdgpu.ids\|requested" $OUT
