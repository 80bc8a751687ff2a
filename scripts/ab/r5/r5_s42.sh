#!/bin/bash
# r5 GPU session 42: 128-thread row kernels as the product (LN+modulate, RMSNorm+RoPE, residual LN):
# row-kernel / fp8 / model tests, then the 14B bench against the 256-thread build, interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
L=$R/video-styler_amd/vstyler/lib
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp8_gpu.py tests/test_model_gpu.py -q -rfE --timeout 200 --timeout-method thread > gpurun_out/r5_row_tests_s42.log 2>&1
rc=$?; grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r5_row_tests_s42.log | tail -6
if [ $rc -ne 0 ]; then tail -30 gpurun_out/r5_row_tests_s42.log; exit 1; fi
for i in 1 2; do
  for lib in new old; do
    if [ $lib = new ]; then unset VSTYLER_LIB; else export VSTYLER_LIB=$L/diag_rt256/libvstyler.so; fi
    timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-e2e > gpurun_out/r5_bench_${lib}_s42_$i.json 2> gpurun_out/r5_bench_${lib}_s42_$i.err || { tail -20 gpurun_out/r5_bench_${lib}_s42_$i.err; exit 1; }
    echo "$lib $i $(cut -c1-150 gpurun_out/r5_bench_${lib}_s42_$i.json)"
  done
done
unset VSTYLER_LIB
timeout -k 10 120 python -u tests/probes/ln_bench.py 2>&1 | grep -v "Warning\|amdgpu.ids"
