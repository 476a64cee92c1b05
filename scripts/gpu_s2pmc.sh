#!/bin/bash
# PMC traffic of the measured kernels at every BASELINE config (per-kernel source revisions)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash scripts/pmc_capture.sh c2 "--config 2 --steps 3 --warmup 1 --no-fedamw-leg" "local_train" || exit 1
bash scripts/pmc_capture.sh c2_fedamw "--config 2 --algo fedamw --steps 1 --warmup 1" "mix_solve" || exit 1
bash scripts/pmc_capture.sh c4 "--config 4 --steps 3 --warmup 1" "local_train" || exit 1
bash scripts/pmc_capture.sh c3 "--config 3 --steps 2 --warmup 1" "local_train" || exit 1
bash scripts/pmc_capture.sh c5 "--config 5 --steps 1 --warmup 1" "local_train" || exit 1
