#!/bin/bash
# split first-poll delay shipped: same-box A/B against the previous split build (libfedsim_prev.so),
# split/pair/teams tests, local-training PMC recapture, kernel trace, default bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=r04n
mkdir -p gpurun_out/$R
bash scripts/gpu_libab.sh libab8 "5 2" prev shipped || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_split_early.py tests/test_gpu_pair.py tests/test_gpu_teams.py tests/test_gpu_parity.py \
  -m gpu -x -q --timeout 200 --timeout-method thread -k "not mix and not horizon_fedamw" > gpurun_out/$R/tests.log 2>&1 \
  || { echo "tests rc=$?"; tail -30 gpurun_out/$R/tests.log; exit 1; }
tail -1 gpurun_out/$R/tests.log
bash scripts/gpu_pmc4.sh r04 || exit 1
