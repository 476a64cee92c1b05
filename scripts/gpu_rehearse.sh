#!/bin/bash
# bench.py --gpus 2 rehearsed on a one-GPU box: the parent spawns two ranks sharing the GPU over
# gloo (FS_BENCH_BACKEND=gloo); the line must report n_gpus 2 from the process group.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r03}
mkdir -p gpurun_out/$TAG
for cfg in 2 5; do
  FS_BENCH_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --config $cfg --steps 3 --warmup 1 --no-legs \
    --no-fedamw-leg > gpurun_out/$TAG/rehearse_c$cfg.json 2> gpurun_out/$TAG/rehearse_c$cfg.err \
    || { echo "rehearse c$cfg rc=$?"; tail -20 gpurun_out/$TAG/rehearse_c$cfg.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/$TAG/rehearse_c$cfg.json')); print('config $cfg', d['n_gpus'], d['dist'], round(d['value']))"
done
