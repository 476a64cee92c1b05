#!/bin/bash
# round-4 checks after the Z GEMM tile templating and the DPP g broadcast: mix / Z parity, the
# two-rank launcher, Z timing, p-solve timing
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-r04f}
mkdir -p gpurun_out/$R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -m gpu -x -q --timeout 240 \
  --timeout-method thread -k "mix or horizon or two_ranks or blocked or fedamw" > gpurun_out/$R/tests.log 2>&1 \
  || { echo "tests rc=$?"; tail -30 gpurun_out/$R/tests.log; exit 1; }
tail -2 gpurun_out/$R/tests.log
bash scripts/gpu_ztime.sh $R || exit 1
bash scripts/gpu_mix.sh $R "24:6" || exit 1
