#!/bin/bash
# r5 GPU session 20: wide-row fp8 quantisation (block per row) and the one-round LayerNorm statistics --
# tests, row-kernel microbenchmarks new vs previous library, the 14B bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
OLD=$R/video-styler_amd/vstyler/lib/old/libvstyler.so
timeout -k 10 600 python -u -m pytest tests/test_fp8_gpu.py tests/test_kernels_gpu.py tests/test_production_model_gpu.py tests/test_model_gpu.py -k "quant or ln_fusion or layernorm or model or production" -q -rfE --timeout 200 --timeout-method thread > gpurun_out/r5_quant_tests_s20.log 2>&1
rc=$?; grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r5_quant_tests_s20.log | tail -6
if [ $rc -ne 0 ]; then tail -30 gpurun_out/r5_quant_tests_s20.log; exit 1; fi
for i in 1 2; do
  for lib in new old; do
    if [ $lib = old ]; then export VSTYLER_LIB=$OLD; else unset VSTYLER_LIB; fi
    echo "== $lib" >> gpurun_out/r5_quant_ab_s20.log
    timeout -k 10 120 python -u tests/probes/quant_bench.py >> gpurun_out/r5_quant_ab_s20.log 2>&1 || { tail -20 gpurun_out/r5_quant_ab_s20.log; exit 1; }
    timeout -k 10 120 python -u tests/probes/ln_bench.py >> gpurun_out/r5_quant_ab_s20.log 2>&1 || { tail -20 gpurun_out/r5_quant_ab_s20.log; exit 1; }
  done
done
grep -v "Warning\|amdgpu.ids" gpurun_out/r5_quant_ab_s20.log
unset VSTYLER_LIB
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-e2e > gpurun_out/r5_bench_s20.json 2> gpurun_out/r5_bench_s20.err || { tail -20 gpurun_out/r5_bench_s20.err; exit 1; }
cut -c1-200 gpurun_out/r5_bench_s20.json
