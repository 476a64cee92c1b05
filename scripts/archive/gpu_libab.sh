#!/bin/bash
# bench A/B of library variants on one box (FEDSIM_LIB), alternating.
#   scripts/gpu_libab.sh <tag> "<configs>" <variant> [variant ...]   (variant "shipped" = libfedsim.so)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=$1; CONFIGS=$2; shift 2
mkdir -p gpurun_out/$TAG
OUT=gpurun_out/$TAG/ab.txt
: > $OUT
PKG=$PWD/non-iid-distributed-learning-with-optimal-mixture-weights_amd
for c in $CONFIGS; do
  for rep in 1 2; do
    for v in "$@"; do
      lib=libfedsim.so; [ "$v" = shipped ] || lib=libfedsim_$v.so
      FEDSIM_LIB=$PKG/$lib timeout -k 10 200 python -u bench.py --config $c --no-legs --no-fedamw-leg --no-cpu-baseline \
        --steps 8 --warmup 2 > gpurun_out/$TAG/b.json 2> gpurun_out/$TAG/b.err || { echo "bench rc=$? c$c $v"; tail -20 gpurun_out/$TAG/b.err; exit 1; }
      python -c "import json; d = json.loads(open('gpurun_out/$TAG/b.json').read().strip().splitlines()[-1]); r = d['roofline']; print('config $c $v', round(d['ms_per_step'], 4), 'ms/round, launch', round(r['launch_ms'], 4), 'frac', round(r['frac'], 4), r['form'], r['group_width'])" >> $OUT
    done
  done
done
cat $OUT
