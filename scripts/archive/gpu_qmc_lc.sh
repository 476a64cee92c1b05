#!/bin/bash
# qmc at config 5's shape: 4 vs 8 clients per lane (K = 16 vs 8) across first-poll delays
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-qmc_lc}
mkdir -p gpurun_out/$R
for lc in 4 8; do
  for d in -1 0 6 14 18 24; do
    echo "lc=$lc delay=$d" >> gpurun_out/$R/sweep.txt
    FS_MIX_QMC_LC=$lc FS_MIX_POLL_DELAY=$d timeout -k 10 120 python -u scripts/mix_time.py 1000 10 32000 5 2>&1 \
      | grep -v amdgpu.ids >> gpurun_out/$R/sweep.txt || { echo "rc=$?"; tail gpurun_out/$R/sweep.txt; exit 1; }
  done
done
cat gpurun_out/$R/sweep.txt
