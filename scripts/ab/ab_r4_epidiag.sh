#!/bin/bash
# Diagnostic: what the 4-wave GEMM's tile epilogue costs in memory traffic.  Variant libraries built
# with EXTRA=-DW4_DIAG=N into abl_xN/ (1: every output store dropped by the buffer range check,
# 2: residual loads answered by it, 3: both; instruction streams unchanged): alternating processes.
set -o pipefail
cd "$(dirname "$0")/../.."
export AB_VARIANTS=w4 AB_SHAPES=qkv,o-proj,ffn-down,cross-o
for r in 1 2; do
  for lib in video-styler_amd/vstyler/lib/libvstyler.so abl_x1/libvstyler.so abl_x2/libvstyler.so abl_x3/libvstyler.so; do
    echo "== round $r lib $lib"
    VSTYLER_LIB=$PWD/$lib timeout -k 10 240 python -u tests/probes/gemm_ab.py 59280 || exit $?
  done
done
