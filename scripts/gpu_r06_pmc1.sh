#!/bin/bash
# round 6 profile, part 1: PMC passes of configs 2, 4, 3 (and 3 without the fused evaluation)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -e
bash scripts/pmc_capture.sh c2 "--config 2 --no-legs --no-fedamw-leg --steps 3 --warmup 1" "local_train"
bash scripts/pmc_capture.sh c4 "--config 4 --no-legs --steps 3 --warmup 1" "local_train"
bash scripts/pmc_capture.sh c3 "--config 3 --no-legs --steps 2 --warmup 1" "local_train"
bash scripts/pmc_capture.sh c3_nofuse "--config 3 --no-legs --steps 2 --warmup 1 --no-eval-fuse" "local_train"
