#!/bin/bash
# Device assembly of ONE split-form kernel instance (seconds, not the whole file's minutes):
#   scripts/split_asm.sh "2, 2, false, 4, 1, 8, 2, 3" out.s [extra hipcc flags]
# (template arguments RT, G, PROX, EARLY, TEAMS, WAVES, TPWK, MBK of local_train_split_kernel)
set -e
args=$1; out=$2; shift 2
d=$(cd "$(dirname "$0")/.." && pwd)/non-iid-distributed-learning-with-optimal-mixture-weights_amd/csrc
t=$(mktemp /tmp/split_one_XXXX.hip)
cat > "$t" <<SRC
#define FS_SPLIT_KERNEL_ONLY
#include "$d/local_train_split.hip"
template __global__ void fs::local_train_split_kernel<$args>(fs::LTParams, fs::SplitWS);
SRC
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -munsafe-fp-atomics --offload-device-only -S -I"$d" -I"$d/../../include" "$@" "$t" -o "$out"
rm -f "$t"
