#!/bin/bash
# round 6 (session 2): every PMC pass (scripts/gpu_r06_pmc1.sh, gpu_r06_pmc2.sh: configs 2, 4, 3,
# 3 without the fused evaluation, 2's FedAMW leg, 5) and the default bench's kernel trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash scripts/gpu_r06_pmc1.sh && bash scripts/gpu_r06_pmc2.sh ${1:-r06}
