#!/bin/bash
# PMC traffic of the training launch (with its deferred-evaluation blocks) at configs 2 and 4
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash scripts/pmc_capture.sh c2 "--config 2 --steps 3 --warmup 1 --no-fedamw-leg" "local_train" || exit 1
bash scripts/pmc_capture.sh c4 "--config 4 --steps 3 --warmup 1" "local_train" || exit 1
