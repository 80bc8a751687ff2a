#!/bin/bash
# r5 GPU session 41: row kernels with 320 / 640 / 128 threads per row (LN, RMSNorm+RoPE) vs 256
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
L=$R/video-styler_amd/vstyler/lib
for i in 1 2 3; do
  for lib in prod rt320 rt640 rt128; do
    if [ $lib = prod ]; then unset VSTYLER_LIB; else export VSTYLER_LIB=$L/diag_$lib/libvstyler.so; fi
    echo "== $lib" >> gpurun_out/r5_ln_rows_ab_s41.log
    timeout -k 10 120 python -u tests/probes/ln_bench.py >> gpurun_out/r5_ln_rows_ab_s41.log 2>&1 || { tail -20 gpurun_out/r5_ln_rows_ab_s41.log; exit 1; }
  done
done
grep -v "Warning\|amdgpu.ids" gpurun_out/r5_ln_rows_ab_s41.log
