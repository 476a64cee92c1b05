#!/bin/bash
# qmc helper lead 8: p-solve tests, FedAMW PMC recapture, then the record (full suite, smoke, bench x2)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
bash scripts/gpu_pmc_mix.sh || exit 1
bash scripts/gpu_r04final.sh r04final6
