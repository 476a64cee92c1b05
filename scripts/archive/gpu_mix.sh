#!/bin/bash
# p-solve timing sweep on one box (scripts/mix_time.py): config 5's qmc shape (N = 1000, C = 10,
# n_val = 32,000; D only sizes the Z GEMM, kept small) over prefetch helper counts and leads, and
# config 2's quad shape.   scripts/gpu_mix.sh <tag> [extra "H:LEAD" pairs...]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-mix}; shift
mkdir -p gpurun_out/$TAG
OUT=gpurun_out/$TAG/mix_sweep.txt
: > $OUT
run() {   # H LEAD N C NV EP
  FS_MIX_PF_H=$1 FS_MIX_PF_LEAD=$2 timeout -k 10 120 python -u scripts/mix_time.py $3 $4 $5 $6 64 >> $OUT 2>&1 \
    || { echo "mix_time rc=$? (H=$1 lead=$2 N=$3)"; tail -20 $OUT; exit 1; }
  echo "  ^ H=$1 lead=$2" >> $OUT
}
PAIRS=${*:-"0:0 -1:0 24:8 16:6"}
for hl in $PAIRS; do run ${hl%%:*} ${hl##*:} 1000 10 32000 5; done
for hl in 0:0; do run ${hl%%:*} ${hl##*:} 100 10 12800 10; done
cat $OUT
