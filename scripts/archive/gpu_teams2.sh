#!/bin/bash
# team form (with the yielding spin): stamps split G = 2 vs teams G = 4 at config 2, then A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-teams2}
mkdir -p gpurun_out/$TAG
OUT=gpurun_out/$TAG/ab.txt
: > $OUT
PKG=$PWD/non-iid-distributed-learning-with-optimal-mixture-weights_amd
for a in "--G 2" "--G 4 --teams" "--G 4"; do
  echo "== stamps config 2 $a" >> $OUT
  FEDSIM_LIB=$PKG/libfedsim_stamps.so timeout -k 10 150 python -u scripts/stamps.py --config 2 $a >> $OUT 2>&1 \
    || { echo "stamps rc=$? ($a)"; tail -20 $OUT; exit 1; }
done
for c in 2 4; do
  for f in auto teams; do
    timeout -k 10 200 python -u bench.py --config $c --no-legs --no-fedamw-leg --no-cpu-baseline --steps 20 --warmup 3 \
      --train-form $f > gpurun_out/$TAG/b.json 2> gpurun_out/$TAG/b.err || { echo "bench rc=$? c$c $f"; tail -20 gpurun_out/$TAG/b.err; exit 1; }
    python -c "import json; d = json.loads(open('gpurun_out/$TAG/b.json').read().strip().splitlines()[-1]); r = d['roofline']; print('config $c $f', round(d['value']), 'cr/s', round(d['ms_per_step'], 4), 'ms/round, launch', round(r['launch_ms'], 4), 'frac', round(r['frac'], 4), r['form'], r['group_width'])" >> $OUT
  done
done
grep -v amdgpu.ids $OUT
