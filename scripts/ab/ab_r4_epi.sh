#!/bin/bash
# A/B of the 4-wave GEMM tile epilogue (pair arithmetic, r4) against the previous build
# (abl_old/libvstyler.so, built from the parent commit's gemm.hip): alternating processes, w4 only.
set -o pipefail
cd "$(dirname "$0")/../.."
export AB_VARIANTS=w4 AB_SHAPES=${AB_SHAPES:-qkv,o-proj,ffn-up,ffn-down,cross-o}
for r in 1 2 3; do
  for lib in abl_old/libvstyler.so video-styler_amd/vstyler/lib/libvstyler.so; do
    echo "== round $r lib $lib"
    VSTYLER_LIB=$PWD/$lib timeout -k 10 240 python -u tests/probes/gemm_ab.py 59280 || exit $?
  done
done
