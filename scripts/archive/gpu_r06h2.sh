#!/bin/bash
# round 6 (session 2): the forward-only mb instance at G = 2 (config 2) -- the GPU suite, then
# launch us by shape (the new instance) vs the 16x16x4 one (split_mb = -1) vs the full mb one
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06h2; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --deselect tests/test_gpu_mb.py::test_mb_selection > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  for mb in auto off on; do
    timeout -k 10 120 python -u scripts/lt_sweep.py --config 2 --G 2 --reg 0 --mb $mb >> $O/ab.txt 2>&1 || exit 1
    echo "^ c2 mb $mb" >> $O/ab.txt
  done
done
grep -v amdgpu.ids $O/ab.txt
