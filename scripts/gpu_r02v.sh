#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r02v
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread \
  -k "mix_solve_variants or auto_choice or golden" > gpurun_out/r02v/parity.log 2>&1
echo "rc=$?"; grep -E "passed|failed|FAILED" gpurun_out/r02v/parity.log | head -30
exit 0
