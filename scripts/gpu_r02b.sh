#!/bin/bash
# Round 2, second GPU pass: BASELINE-config tests, long-horizon goldens, prep fixture, rest of
# the GPU suite; then in-kernel phase stamps of the split-group kernel.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r02b
mkdir -p $OUT
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_experiment.py tests/test_gpu_single.py \
  tests/test_gpu_dist.py "tests/test_gpu_parity.py::test_dropin_long_horizon_golden" -v --timeout 300 \
  --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" $OUT/tests.log | tail -40; ok $rc || exit $rc
for a in "--config 5" "--config 2" "--config 1" "--config 3" "--config 1 --G 16"; do
  FEDSIM_LIB=$PWD/non-iid-distributed-learning-with-optimal-mixture-weights_amd/libfedsim_stamps.so \
    timeout -k 10 180 python -u scripts/stamps.py $a > $OUT/stamps.log.tmp 2>&1; rc=$?
  grep -v amdgpu.ids $OUT/stamps.log.tmp | tee -a $OUT/stamps.log; ok $rc || exit $rc
done
exit 0
