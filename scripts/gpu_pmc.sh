#!/bin/bash
# Round profile: PMC passes (scripts/pmc_capture.sh) for every bench workload, then the kernel
# trace of the default bench command.   scripts/gpu_pmc.sh <round-tag>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-r05}
set -e
bash scripts/pmc_capture.sh c2 "--config 2 --no-legs --no-fedamw-leg --steps 3 --warmup 1" "local_train"
bash scripts/pmc_capture.sh c4 "--config 4 --no-legs --steps 3 --warmup 1" "local_train"
bash scripts/pmc_capture.sh c3 "--config 3 --no-legs --steps 2 --warmup 1" "local_train"
bash scripts/pmc_capture.sh c3_nofuse "--config 3 --no-legs --steps 2 --warmup 1 --no-eval-fuse" "local_train"
bash scripts/pmc_capture.sh c2_fedamw "--config 2 --algo fedamw --no-legs --no-fedamw-leg --steps 2 --warmup 1" "local_train|mix_solve|mix_z"
bash scripts/pmc_capture.sh c5 "--config 5 --no-legs --steps 1 --warmup 1" "local_train|mix_solve|mix_z"
mkdir -p gpurun_out/trace_$R
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_$R -o $R --output-format csv -- python3 -u bench.py \
  > gpurun_out/trace_$R/bench.json 2> gpurun_out/trace_$R/bench.err
echo "trace rc=$?"
