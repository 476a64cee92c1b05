#!/bin/bash
# PMC traffic at config 5 (group kernel) and of config 2's FedAMW p-solve
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash scripts/pmc_capture.sh c5 "--config 5 --steps 1 --warmup 1" "local_train" || exit 1
bash scripts/pmc_capture.sh c2_fedamw "--config 2 --algo fedamw --steps 1 --warmup 1" "mix_solve" || exit 1
