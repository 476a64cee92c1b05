#!/bin/bash
# round 6 (session 2): the solver-horizon margins re-recorded on the final sources (mb instances)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06m2
rm -f gpurun_out/r06m2/horizon_margins.jsonl
FS_MARGINS_OUT=gpurun_out/r06m2/horizon_margins.jsonl timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k horizon > gpurun_out/r06m2/tests.log 2>&1
rc=$?
tail -3 gpurun_out/r06m2/tests.log
exit $rc
