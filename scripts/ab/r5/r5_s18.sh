#!/bin/bash
# r5 GPU session 18: fp8 row quantisation with the row kept in registers (one read of x) -- fp8 tests,
# microbenchmark new vs previous library, config-5 bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
OLD=$R/video-styler_amd/vstyler/lib/old/libvstyler.so
timeout -k 10 600 python -u -m pytest tests/test_fp8_gpu.py tests/test_production_c4c5_gpu.py -k "fp8 or c5 or quant" -q -rfE --timeout 300 --timeout-method thread > gpurun_out/r5_fp8_tests_s18.log 2>&1
rc=$?; grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r5_fp8_tests_s18.log | tail -6
if [ $rc -ne 0 ]; then tail -30 gpurun_out/r5_fp8_tests_s18.log; exit 1; fi
for i in 1 2; do
  for lib in new old; do
    if [ $lib = old ]; then export VSTYLER_LIB=$OLD; else unset VSTYLER_LIB; fi
    echo "== $lib" >> gpurun_out/r5_quant_ab_s18.log
    timeout -k 10 120 python -u tests/probes/quant_bench.py >> gpurun_out/r5_quant_ab_s18.log 2>&1 || { tail -20 gpurun_out/r5_quant_ab_s18.log; exit 1; }
  done
done
unset VSTYLER_LIB
grep -v "Warning\|amdgpu.ids" gpurun_out/r5_quant_ab_s18.log
timeout -k 10 500 python -u bench.py --config fp8 --steps 4 --no-cpu-baseline --no-e2e > gpurun_out/r5_bench_fp8_s18.json 2> gpurun_out/r5_bench_fp8_s18.err || { tail -20 gpurun_out/r5_bench_fp8_s18.err; exit 1; }
cut -c1-200 gpurun_out/r5_bench_fp8_s18.json
