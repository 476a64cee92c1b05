#!/bin/bash
# one box session: Z-GEMM timing, p-solve stamps and helper sweep, then the stream form's tests / A/B / stamps
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash scripts/gpu_ztime.sh r04z2 && bash scripts/gpu_mixstamps.sh r04s1 && bash scripts/gpu_mix.sh r04m2 && bash scripts/gpu_stream.sh r04st
