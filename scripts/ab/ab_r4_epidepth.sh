#!/bin/bash
# A/B: residual rows prefetched in the 4-wave GEMM epilogue (W4_EPI_DEPTH_BF16 2 = shipped, 3, 4;
# the variant libraries are built with EXTRA=-DW4_EPI_DEPTH_BF16=N into abl_d3/ abl_d4/): alternating
# processes, w4 only, the residual-epilogue block shapes.
set -o pipefail
cd "$(dirname "$0")/../.."
export AB_VARIANTS=w4 AB_SHAPES=o-proj,ffn-down,cross-o
for r in 1 2 3; do
  for lib in video-styler_amd/vstyler/lib/libvstyler.so abl_d3/libvstyler.so abl_d4/libvstyler.so; do
    echo "== round $r lib $lib"
    VSTYLER_LIB=$PWD/$lib timeout -k 10 240 python -u tests/probes/gemm_ab.py 59280 || exit $?
  done
done
