#!/bin/bash
# r5 GPU session 25: attn_fwd_w4 K-fragment LDS bases (kept) and the row sums as v_dot2c_f32_bf16 of
# the packed P with (1, 1) (diag_dot: one VALU per P pair instead of two adds) -- attention tests on
# both, self/cross microbenchmark new / dot / old interleaved, the 14B bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
L=$R/video-styler_amd/vstyler/lib
for lib in new dot; do
  if [ $lib = new ]; then unset VSTYLER_LIB; else export VSTYLER_LIB=$L/diag_$lib/libvstyler.so; fi
  timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_attention_production_gpu.py -k "attention or attn" -q -rfE --timeout 300 --timeout-method thread > gpurun_out/r5_attn_tests_${lib}_s25.log 2>&1
  rc=$?; echo "tests $lib:"; grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r5_attn_tests_${lib}_s25.log | tail -6
  if [ $rc -ne 0 ]; then tail -30 gpurun_out/r5_attn_tests_${lib}_s25.log; exit 1; fi
done
for i in 1 2 3; do
  for lib in new dot old; do
    case $lib in new) unset VSTYLER_LIB;; old) export VSTYLER_LIB=$L/old/libvstyler.so;; *) export VSTYLER_LIB=$L/diag_$lib/libvstyler.so;; esac
    echo "== $lib" >> gpurun_out/r5_attn_ab_s25.log
    timeout -k 10 120 python -u tests/probes/attn_bench.py >> gpurun_out/r5_attn_ab_s25.log 2>&1 || { tail -20 gpurun_out/r5_attn_ab_s25.log; exit 1; }
  done
done
unset VSTYLER_LIB
grep -v "Warning\|amdgpu.ids" gpurun_out/r5_attn_ab_s25.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-e2e > gpurun_out/r5_bench_s25.json 2> gpurun_out/r5_bench_s25.err || { tail -20 gpurun_out/r5_bench_s25.err; exit 1; }
cut -c1-200 gpurun_out/r5_bench_s25.json
