#!/bin/bash
# PMC traffic of the current p-solvers: config 2's FedAMW leg (quad) and config 5 (qmc)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash scripts/pmc_capture.sh c2_fedamw "--config 2 --algo fedamw --steps 1 --warmup 1" "mix_solve" || exit 1
bash scripts/pmc_capture.sh c5_fedamw "--config 5 --steps 1 --warmup 1" "mix_solve" || exit 1
