#!/bin/bash
# fs_mix_z timing at config 5 (one GPU and one rank's share of 8) and config 2.   scripts/gpu_ztime.sh <tag>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-zt}
mkdir -p gpurun_out/$TAG
for a in "1000 10 16384 32000 5" "125 10 16384 32000 5" "100 10 2048 12800 10"; do
  timeout -k 10 120 python -u scripts/z_time.py $a >> gpurun_out/$TAG/z_time.txt 2>&1 || { echo "z_time rc=$? ($a)"; tail -20 gpurun_out/$TAG/z_time.txt; exit 1; }
done
cat gpurun_out/$TAG/z_time.txt
