#!/bin/bash
# r5 GPU session 21: attn_fwd_w4 with the next item's Q loaded after the O store (88 -> 9 VGPR spills)
# -- attention tests, switch stamps, self/cross microbenchmark and key-count sweep new vs previous
# library (interleaved), the 14B bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
OLD=$R/video-styler_amd/vstyler/lib/old/libvstyler.so
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_attention_production_gpu.py -k "attention or attn" -q -rfE --timeout 300 --timeout-method thread > gpurun_out/r5_attn_tests_s21.log 2>&1
rc=$?; grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r5_attn_tests_s21.log | tail -6
if [ $rc -ne 0 ]; then tail -30 gpurun_out/r5_attn_tests_s21.log; exit 1; fi
VSTYLER_LIB=$R/video-styler_amd/vstyler/lib/diag_w4st/libvstyler.so W4S_SKV=512 timeout -k 10 200 python -u tests/probes/w4_stamps.py > gpurun_out/r5_w4_switch_s21.log 2>&1 || { tail -20 gpurun_out/r5_w4_switch_s21.log; exit 1; }
grep -v "Warning\|amdgpu.ids" gpurun_out/r5_w4_switch_s21.log
for i in 1 2 3; do
  for lib in new old; do
    if [ $lib = old ]; then export VSTYLER_LIB=$OLD; else unset VSTYLER_LIB; fi
    echo "== $lib" >> gpurun_out/r5_attn_ab_s21.log
    timeout -k 10 120 python -u tests/probes/attn_bench.py >> gpurun_out/r5_attn_ab_s21.log 2>&1 || { tail -20 gpurun_out/r5_attn_ab_s21.log; exit 1; }
  done
done
unset VSTYLER_LIB
grep -v "Warning\|amdgpu.ids" gpurun_out/r5_attn_ab_s21.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-e2e > gpurun_out/r5_bench_s21.json 2> gpurun_out/r5_bench_s21.err || { tail -20 gpurun_out/r5_bench_s21.err; exit 1; }
cut -c1-200 gpurun_out/r5_bench_s21.json
