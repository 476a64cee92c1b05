#!/bin/bash
# PMC passes of the FedAMW workloads only (p-solve / Z GEMM sources changed):
#   scripts/gpu_pmc_mix.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
bash scripts/pmc_capture.sh c2_fedamw "--config 2 --algo fedamw --no-legs --no-fedamw-leg --steps 2 --warmup 1" "local_train|mix_solve|mix_z" || exit 1
bash scripts/pmc_capture.sh c5 "--config 5 --no-legs --steps 1 --warmup 1" "local_train|mix_solve|mix_z" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "quad or mix_solve_variants or dropin_fedamw or config2" > gpurun_out/pmc_mix_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/pmc_mix_tests.log; exit 1; }
tail -1 gpurun_out/pmc_mix_tests.log
