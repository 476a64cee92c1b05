#!/bin/bash
# round 6 (session 2): the one-rank RCCL collectives test, then the PMC passes of configs 2, 4, 3
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06t
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -m gpu -x -v --timeout 240 --timeout-method thread \
  -k rccl > gpurun_out/r06t/rccl_test.log 2>&1
rc=$?
tail -3 gpurun_out/r06t/rccl_test.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r06_pmc1.sh
