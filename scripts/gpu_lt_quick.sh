#!/bin/bash
# quick A/B: split-form launch times at configs 2, 5, 3 (two passes) + the split bitwise tests
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ltq
timeout -k 10 300 python -u -m pytest tests/test_gpu_split_early.py tests/test_gpu_pair.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ltq/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/ltq/tests.log; exit 1; }
tail -1 gpurun_out/ltq/tests.log
for pass in 1 2; do
  for c in 2 5; do timeout -k 10 120 python -u scripts/lt_sweep.py --config $c --reg 0 2>&1 | grep -v amdgpu.ids || exit 1; done
  timeout -k 10 120 python -u scripts/lt_sweep.py --config 3 --prox --reg 0 2>&1 | grep -v amdgpu.ids || exit 1
done
