#!/bin/bash
# round 6 record: full GPU suite (horizon margins recorded), smoke(), the default bench line
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-r06e}
mkdir -p gpurun_out/$R
rm -f gpurun_out/$R/horizon_margins.jsonl
FS_MARGINS_OUT=gpurun_out/$R/horizon_margins.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread \
  > gpurun_out/$R/gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/$R/gpu_tests.log
grep -E "^FAILED|^ERROR" gpurun_out/$R/gpu_tests.log | head -20
[ $rc -le 1 ] || { echo "tests rc=$rc"; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$R/smoke.log 2>&1 \
  || { echo "smoke rc=$?"; tail -30 gpurun_out/$R/smoke.log; exit 1; }
tail -2 gpurun_out/$R/smoke.log
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$R/bench_a.json 2> gpurun_out/$R/bench_a.err \
  || { echo "bench rc=$?"; tail -30 gpurun_out/$R/bench_a.err; exit 1; }
cut -c1-300 gpurun_out/$R/bench_a.json
grep -v amdgpu.ids gpurun_out/$R/bench_a.err | tail -5
