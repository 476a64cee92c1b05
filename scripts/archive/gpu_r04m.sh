#!/bin/bash
# after the qmc first-poll delay: p-solve / dist tests, FedAMW PMC recapture, default bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=r04m
mkdir -p gpurun_out/$R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_configs.py -m gpu -x -q \
  --timeout 240 --timeout-method thread -k "mix or horizon or fedamw or qmc or blocked or sharded or config5 or two_ranks" \
  > gpurun_out/$R/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/$R/tests.log; exit 1; }
tail -1 gpurun_out/$R/tests.log
bash scripts/gpu_pmc_mix.sh || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/$R/bench.json 2> gpurun_out/$R/bench.err || { echo "bench rc=$?"; tail -30 gpurun_out/$R/bench.err; exit 1; }
cut -c1-200 gpurun_out/$R/bench.json
