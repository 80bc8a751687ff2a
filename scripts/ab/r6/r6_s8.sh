#!/bin/bash
# r6 step 8: cross-attention with desynchronised item switches (every other slot starts late)
set -o pipefail
mkdir -p gpurun_out
L=video-styler_amd/vstyler/lib
for r in 1 2 3; do
for v in product ds1 ds3; do
  if [ $v = product ]; then lib=$L/libvstyler.so; else lib=$L/diag_$v/libvstyler.so; fi
  VSTYLER_LIB=$lib timeout -k 10 300 python -u tests/probes/attn_bench.py 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" | tee -a gpurun_out/r6_attn_desync_s8.log || exit 1
done
done
