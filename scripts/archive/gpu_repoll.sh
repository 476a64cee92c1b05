#!/bin/bash
# split hand-off: selective re-poll (libfedsim.so) vs reload-all (libfedsim_prev.so), same box;
# split/pair/early tests; stamps of config 5
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-repoll}
mkdir -p gpurun_out/$TAG
OUT=gpurun_out/$TAG/ab.txt
: > $OUT
PKG=$PWD/non-iid-distributed-learning-with-optimal-mixture-weights_amd
timeout -k 10 500 python -u -m pytest tests/test_gpu_split_early.py tests/test_gpu_pair.py -m gpu -x -q --timeout 150 \
  --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/$TAG/tests.log; exit 1; }
tail -1 gpurun_out/$TAG/tests.log
for c in 5 2; do
  for lib in libfedsim_prev.so libfedsim.so libfedsim_prev.so libfedsim.so; do
    FEDSIM_LIB=$PKG/$lib timeout -k 10 200 python -u bench.py --config $c --no-legs --no-fedamw-leg --no-cpu-baseline \
      --steps 6 --warmup 2 > gpurun_out/$TAG/b.json 2> gpurun_out/$TAG/b.err || { echo "bench rc=$? c$c $lib"; tail -20 gpurun_out/$TAG/b.err; exit 1; }
    python -c "import json; d = json.loads(open('gpurun_out/$TAG/b.json').read().strip().splitlines()[-1]); r = d['roofline']; print('config $c $lib', round(d['ms_per_step'], 4), 'ms/round, launch', round(r['launch_ms'], 4), 'frac', round(r['frac'], 4), r['form'], r['group_width'])" >> $OUT
  done
done
echo "== stamps config 5" >> $OUT
FEDSIM_LIB=$PKG/libfedsim_stamps.so timeout -k 10 150 python -u scripts/stamps.py --config 5 >> $OUT 2>&1 || { echo "stamps rc=$?"; exit 1; }
grep -v amdgpu.ids $OUT
