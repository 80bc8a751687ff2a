#!/bin/bash
# r6 step 10: GEMM raster-group height (M-tiles per group, VS_GEMM_GM) 2 / 4 (product) / 8 / 16
set -o pipefail
mkdir -p gpurun_out
L=video-styler_amd/vstyler/lib
for r in 1 2; do
for v in product gm2 gm8 gm16; do
  if [ $v = product ]; then lib=$L/libvstyler.so; else lib=$L/diag_$v/libvstyler.so; fi
  VSTYLER_LIB=$lib timeout -k 10 300 python -u tests/probes/gemm_diag.py 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" | tee -a gpurun_out/r6_gemm_gm_s10.log || exit 1
done
done
