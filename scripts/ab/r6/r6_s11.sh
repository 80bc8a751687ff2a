#!/bin/bash
# r6 step 11: raster-group height for the K = 5120 shapes (o-proj / q|k|v / FFN-up) at 59 280 and at
# the SP = 8 rank's 7410 rows (K >= 8192 shapes are fixed at 2 in every build)
set -o pipefail
mkdir -p gpurun_out
L=video-styler_amd/vstyler/lib
for M in 59280 7410; do
for r in 1 2; do
for v in product gm2 gm8; do
  if [ $v = product ]; then lib=$L/libvstyler.so; else lib=$L/diag_$v/libvstyler.so; fi
  GD_M=$M VSTYLER_LIB=$lib timeout -k 10 300 python -u tests/probes/gemm_diag.py 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" | tee -a gpurun_out/r6_gemm_gm_s11.log || exit 1
done
done
done
