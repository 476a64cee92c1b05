#!/bin/bash
# round 6 profile, part 2: PMC passes of config 2's FedAMW leg and config 5, the kernel trace of the
# default bench command, then the default bench line twice
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${1:-r06}
set -e
bash scripts/pmc_capture.sh c2_fedamw "--config 2 --algo fedamw --no-legs --no-fedamw-leg --steps 2 --warmup 1" "local_train|mix_solve|mix_z"
bash scripts/pmc_capture.sh c5 "--config 5 --no-legs --steps 1 --warmup 1" "local_train|mix_solve|mix_z"
mkdir -p gpurun_out/trace_$R
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_$R -o $R --output-format csv -- python3 -u bench.py \
  > gpurun_out/trace_$R/bench.json 2> gpurun_out/trace_$R/bench.err
echo "trace rc=$?"
