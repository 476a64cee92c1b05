#!/bin/bash
# rehearsal of bench.py's multi-rank path on one GPU (2 ranks, gloo): config 2 weak, config 5 strong
set -o pipefail
mkdir -p gpurun_out/r02ad
export FS_BENCH_BACKEND=gloo
for c in "2 --no-fedamw-leg --steps 3 --warmup 1" "5 --steps 1 --warmup 1"; do set -- $c
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --config $1 ${@:2} --no-cpu-baseline > gpurun_out/r02ad/c$1.json 2> gpurun_out/r02ad/c$1.err
  rc=$?; echo "config $1 rc=$rc"; tail -1 gpurun_out/r02ad/c$1.json | cut -c1-400; [ $rc -eq 0 ] || { tail -20 gpurun_out/r02ad/c$1.err; exit $rc; }
done
