#!/bin/bash
# A/B: cache policy of the 4-wave GEMM epilogue (variant libraries built with EXTRA=-DW4_OUT_CPOL /
# -DW4_RES_CPOL into abl_<name>/: s2 = nt output stores, b2 = nt stores + nt residual loads,
# s18 = sc1|nt stores): alternating processes, w4 only.
set -o pipefail
cd "$(dirname "$0")/../.."
export AB_VARIANTS=w4 AB_SHAPES=${AB_SHAPES:-qkv,o-proj,ffn-up,ffn-down,cross-o}
for r in 1 2 3; do
  for lib in video-styler_amd/vstyler/lib/libvstyler.so abl_s2/libvstyler.so abl_b2/libvstyler.so abl_s18/libvstyler.so; do
    echo "== round $r lib $lib"
    VSTYLER_LIB=$PWD/$lib timeout -k 10 240 python -u tests/probes/gemm_ab.py 59280 || exit $?
  done
done
