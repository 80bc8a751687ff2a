#!/bin/bash
# r5 GPU session 13: LayerNorm / RMSNorm+RoPE kernels one wave per row -- elementwise + model tests,
# the row-kernel microbenchmark new vs previous library (interleaved), the 14B bench under rocprof.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
OLD=$R/video-styler_amd/vstyler/lib/old/libvstyler.so
fault() { grep -qiE "memory access fault|illegal address|HSA_STATUS_ERROR|hipErrorLaunchFailure|core dumped" "$1"; }
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_production_model_gpu.py tests/test_model_gpu.py -q -rfE --timeout 300 --timeout-method thread > gpurun_out/r5_rows_tests_s13.log 2>&1
rc=$?; grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r5_rows_tests_s13.log | tail -8
if [ $rc -ne 0 ] || fault gpurun_out/r5_rows_tests_s13.log; then tail -30 gpurun_out/r5_rows_tests_s13.log; exit 1; fi
for i in 1 2; do
  for lib in new old; do
    if [ $lib = old ]; then export VSTYLER_LIB=$OLD; else unset VSTYLER_LIB; fi
    echo "== $lib" >> gpurun_out/r5_ln_ab_s13.log
    timeout -k 10 120 python -u tests/probes/ln_bench.py >> gpurun_out/r5_ln_ab_s13.log 2>&1 || { tail -20 gpurun_out/r5_ln_ab_s13.log; exit 1; }
  done
done
unset VSTYLER_LIB
grep -v Warning gpurun_out/r5_ln_ab_s13.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r5s13 -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $R/gpurun_out/prof_r5s13.log 2>&1 || { tail -20 $R/gpurun_out/prof_r5s13.log; exit 1; }
grep '"metric"' $R/gpurun_out/prof_r5s13.log | cut -c1-200
cd $R
VSTYLER_LIB=$R/video-styler_amd/vstyler/lib/diag_w4st/libvstyler.so W4S_SKV=512 timeout -k 10 200 python -u tests/probes/w4_stamps.py > gpurun_out/r5_w4_switch_cross_s13.log 2>&1 || { tail -20 gpurun_out/r5_w4_switch_cross_s13.log; exit 1; }
grep -v Warning gpurun_out/r5_w4_switch_cross_s13.log
