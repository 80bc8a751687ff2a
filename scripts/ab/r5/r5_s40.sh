#!/bin/bash
# r5 GPU session 40: LayerNorm(+modulate) with NR rows per workgroup (shared block reductions):
# layernorm tests on the product build (2 rows), then ln_bench 2 / 1 / 4 rows interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
L=$R/video-styler_amd/vstyler/lib
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp8_gpu.py -k "layernorm or ln_ or modulate" -q -rfE --timeout 120 --timeout-method thread > gpurun_out/r5_ln_tests_s40.log 2>&1
rc=$?; grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r5_ln_tests_s40.log | tail -6
if [ $rc -ne 0 ]; then tail -30 gpurun_out/r5_ln_tests_s40.log; exit 1; fi
for i in 1 2 3; do
  for lib in prod ln1 ln4; do
    if [ $lib = prod ]; then unset VSTYLER_LIB; else export VSTYLER_LIB=$L/diag_$lib/libvstyler.so; fi
    echo "== $lib" >> gpurun_out/r5_ln_rows_ab_s40.log
    timeout -k 10 120 python -u tests/probes/ln_bench.py >> gpurun_out/r5_ln_rows_ab_s40.log 2>&1 || { tail -20 gpurun_out/r5_ln_rows_ab_s40.log; exit 1; }
  done
done
grep -v "Warning\|amdgpu.ids" gpurun_out/r5_ln_rows_ab_s40.log
