#!/bin/bash
# qmc first-poll delay sweep (fs_tuning.mix_poll_delay via FS_MIX_POLL_DELAY; -1 = none) over
# client counts.   scripts/gpu_polldelay.sh <tag>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-polldelay}
mkdir -p gpurun_out/$TAG
OUT=gpurun_out/$TAG/sweep.txt
: > $OUT
run() {   # delay N C NV EP
  FS_MIX_POLL_DELAY=$1 timeout -k 10 120 python -u scripts/mix_time.py $2 $3 $4 $5 64 >> $OUT 2>&1 \
    || { echo "mix_time rc=$? (delay $1 N $2)"; tail -20 $OUT; exit 1; }
  echo "  ^ delay $1" >> $OUT
}
for d in -1 12 14 16 18 20 0; do run $d 1000 10 32000 5; done
for d in -1 4 8 12 16 0; do run $d 300 10 12800 5; done
for d in -1 8 12 16 0; do run $d 520 10 12800 5; done
for d in -1 8 16 0; do run $d 1000 4 32000 5; done
grep -v "amdgpu.ids\|requested" $OUT
