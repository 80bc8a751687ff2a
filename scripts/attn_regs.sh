#!/bin/bash
# Print VGPR count / spills of the attention kernels for a flag set: scripts/attn_regs.sh "-DFOO"
SRC=$(cd $(dirname $0)/.. && pwd)/video-styler_amd/csrc/attention.hip
D=$(mktemp -d); cd $D
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -std=c++17 $1 --save-temps -c $SRC -o a.o 2>/dev/null
grep -E '^\s+\.(name|vgpr_count|vgpr_spill_count):' *gfx950.s | grep -A2 'attn_fwd' | paste - - - | awk '{print $2, $4, $6}'
rm -rf $D
