#!/bin/bash
# p-solve session: stamps + helper sweep on the batched re-poll, then the p-solve / FedAMW parity tests
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
bash scripts/gpu_mixstamps.sh r04s2 && bash scripts/gpu_mix.sh r04m3 || exit 1
mkdir -p gpurun_out/r04t
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_configs.py -x -v \
  --timeout 240 --timeout-method thread -k "mix or horizon or qmc or fedamw or blocked or sharded or config5" \
  > gpurun_out/r04t/psolve_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r04t/psolve_tests.log; exit 1; }
tail -3 gpurun_out/r04t/psolve_tests.log
