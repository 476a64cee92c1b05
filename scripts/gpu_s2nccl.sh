#!/bin/bash
# RCCL path rehearsal: 2 ranks sharing the box's one GPU over the nccl (RCCL) backend.  RCCL
# may refuse two ranks on one device; this only checks that the path initialises and runs.
set -o pipefail
mkdir -p gpurun_out/r02s2nccl
NCCL_DEBUG=WARN timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29531 bench.py --gpus 2 --config 2 --no-fedamw-leg --steps 3 --warmup 1 --no-cpu-baseline \
  > gpurun_out/r02s2nccl/c2.json 2> gpurun_out/r02s2nccl/c2.err
rc=$?; echo "nccl 2 ranks rc=$rc"; tail -1 gpurun_out/r02s2nccl/c2.json | cut -c1-300; grep -i -E 'error|duplicate|warn' gpurun_out/r02s2nccl/c2.err | head -8
exit 0
