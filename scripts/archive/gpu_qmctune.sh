#!/bin/bash
# qmc at config 5's shape with the first-poll delay: helper count / lead, delay 12-16, and a
# re-poll sleep variant (libfedsim_rps2.so).   scripts/gpu_qmctune.sh <tag>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-qmctune}
mkdir -p gpurun_out/$TAG
OUT=gpurun_out/$TAG/tune.txt
: > $OUT
PKG=$PWD/non-iid-distributed-learning-with-optimal-mixture-weights_amd
run() {   # label env...
  local label=$1; shift
  env "$@" timeout -k 10 120 python -u scripts/mix_time.py 1000 10 32000 5 64 >> $OUT 2>&1 \
    || { echo "mix_time rc=$? ($label)"; tail -20 $OUT; exit 1; }
  echo "  ^ $label" >> $OUT
}
for rep in 1 2; do
  run default FS_MIX_PF_H=0
  run "h8" FS_MIX_PF_H=8
  run "h16 lead4" FS_MIX_PF_H=16 FS_MIX_PF_LEAD=4
  run "h16 lead10" FS_MIX_PF_H=16 FS_MIX_PF_LEAD=10
  run "delay12" FS_MIX_POLL_DELAY=12
  run "delay15" FS_MIX_POLL_DELAY=15
  run "repoll sleep" FEDSIM_LIB=$PKG/libfedsim_rps2.so
done
grep -v "amdgpu.ids\|requested" $OUT
