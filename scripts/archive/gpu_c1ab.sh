#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c1ab
for k in 1 2; do timeout -k 10 200 python -u scripts/lt_sweep.py --config 1 --G 8 2>&1 | grep -v amdgpu.ids; done
