#!/bin/bash
# Usage: tools/resusage.sh <file.hip> [extra hipcc flags] -- per-kernel VGPR / spill / occupancy of gm:: kernels
f=$1; shift
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC "$@" -c "$f" -o /tmp/resusage.o -Rpass-analysis=kernel-resource-usage 2>&1 \
 | grep "remark:" | sed -E 's/.*remark: +//; s/ \[-Rpass.*//' \
 | awk '/^Function Name/{name=$3} /^VGPRs:/{v=$2} /^VGPRs Spill/{sp=$3} /^ScratchSize/{s=$3} /^LDS Size/{l=$4} /^Occupancy/{o=$3}
        /^LDS Size/{ if (name ~ /^_ZN2gm/) printf "%-80s vgpr=%-4s spill=%-4s scratch=%-5s lds=%-6s occ=%s\n", substr(name,1,80), v, sp, s, l, o}'
