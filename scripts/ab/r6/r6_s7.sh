#!/bin/bash
# r6 step 7: what bounds the 4-wave GEMM -- diagnostic builds without the operand DMA, without the
# fragment reads, without both (garbage results; time only), against the product library
set -o pipefail
mkdir -p gpurun_out
L=video-styler_amd/vstyler/lib
for r in 1 2; do
for v in product nodma noread nodmaread; do
  if [ $v = product ]; then lib=$L/libvstyler.so; else lib=$L/diag_$v/libvstyler.so; fi
  VSTYLER_LIB=$lib timeout -k 10 300 python -u tests/probes/gemm_diag.py 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" | tee -a gpurun_out/r6_gemm_diag_s7.log || exit 1
done
done
