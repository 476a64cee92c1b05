#!/bin/bash
# qmc first-poll delay re-check at helper lead 8 over the shapes of the lead-6 sweep.   scripts/gpu_qmcdelay2.sh <tag>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-qmcdelay2}
mkdir -p gpurun_out/$TAG
OUT=gpurun_out/$TAG/delay.txt
: > $OUT
run() {   # delay N C NV epochs
  FS_MIX_POLL_DELAY=$1 timeout -k 10 120 python -u scripts/mix_time.py $2 $3 $4 $5 64 >> $OUT 2>&1 \
    || { echo "mix_time rc=$? (delay $1 N $2 C $3)"; tail -20 $OUT; exit 1; }
  echo "  ^ delay $1 (0 = by shape)" >> $OUT
}
for d in 0 8 10 12; do run $d 1000 10 32000 5; done
for d in 0 8 10 14; do run $d 800 10 25600 5; done
for d in 0 4 6 8 10; do run $d 300 10 12800 5; done
for d in 0 6 8 10; do run $d 520 10 12800 5; done
for d in 0 6 8 10; do run $d 1000 4 32000 5; done
grep -v "amdgpu.ids\|requested" $OUT
