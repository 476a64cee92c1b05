#!/bin/bash
# FedAMW: next round's shuffles enqueued after the training kernel, p-solve waits for them
set -o pipefail
mkdir -p gpurun_out/r02aa
T="timeout -k 10"
$T 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "fedamw or golden or long or config or dist or rng" \
  > gpurun_out/r02aa/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r02aa/tests.log; [ $rc -eq 0 ] || exit $rc
for mode in early late early late; do
  FS_FEDAMW_SHUFFLE=$mode $T 400 python -u bench.py --config 5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r02aa/c5_$mode.json 2>/dev/null || exit 1
  tail -1 gpurun_out/r02aa/c5_$mode.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 $mode', round(d['ms_per_step'],1), d['fedamw'])"
done
for mode in early late; do
  FS_FEDAMW_SHUFFLE=$mode $T 400 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r02aa/c2_$mode.json 2>/dev/null || exit 1
  tail -1 gpurun_out/r02aa/c2_$mode.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); f=d['fedamw']; print('c2 $mode', round(f['ms_per_round'],2), round(f['p_solve_us_per_step'],3))"
done
