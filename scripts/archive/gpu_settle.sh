#!/bin/bash
# clock-settle A/B at the driver's --steps 20 --warmup 5: settle kind x length before the warm-up
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-settle2}
mkdir -p gpurun_out/$R
for k in 1 2; do
  for cfg in "gemm 0" "copy 100" "mixed 100" "mixed 200" "copy 300"; do
    set -- $cfg
    FS_BENCH_SETTLE_KIND=$1 FS_BENCH_SETTLE_MS=$2 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-legs --no-fedamw-leg \
      --steps 20 --warmup 5 > gpurun_out/$R/s$1_$2.$k.json 2>/dev/null || { echo "ab rc=$?"; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/$R/s$1_$2.$k.json')); print('settle=$1 $2', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['launch_ms'],4))"
  done
done
