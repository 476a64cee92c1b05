#!/bin/bash
# Per-kernel register / LDS usage of one HIP source (compiler view): scripts/resusage.sh <file.hip> [extra flags]
f=$1; shift
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -Rpass-analysis=kernel-resource-usage "$@" -c "$f" -o /tmp/resusage.o 2>&1 \
 | sed -n 's/.*remark: *//p' | sed 's/ \[-Rpass-analysis=kernel-resource-usage\]//' \
 | awk '/^Function Name/{if(n)print line; line=$3; n=1; next} /^(VGPRs|AGPRs|Occupancy|SGPRs Spill|VGPRs Spill|LDS Size)/{line=line" | "$0} END{print line}' \
 | c++filt | sed 's/(fs::LTParams, fs::SplitWS)//'
