#!/bin/bash
# r5 GPU session 23: attn_fwd_w4 softmax VALU cuts -- packed row-sum adds (PKSUM) and per-tile opaque
# LDS bases (immediate ds offsets: 32 -> 12 v_add_u32 per tile) -- attention tests, then
# self/cross microbenchmark new / nopk / nobase / old interleaved, the 14B bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
L=$R/video-styler_amd/vstyler/lib
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_attention_production_gpu.py -k "attention or attn" -q -rfE --timeout 300 --timeout-method thread > gpurun_out/r5_attn_tests_s23.log 2>&1
rc=$?; grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r5_attn_tests_s23.log | tail -6
if [ $rc -ne 0 ]; then tail -30 gpurun_out/r5_attn_tests_s23.log; exit 1; fi
for i in 1 2 3; do
  for lib in new nopk nobase old; do
    case $lib in new) unset VSTYLER_LIB;; old) export VSTYLER_LIB=$L/old/libvstyler.so;; *) export VSTYLER_LIB=$L/diag_$lib/libvstyler.so;; esac
    echo "== $lib" >> gpurun_out/r5_attn_ab_s23.log
    timeout -k 10 120 python -u tests/probes/attn_bench.py >> gpurun_out/r5_attn_ab_s23.log 2>&1 || { tail -20 gpurun_out/r5_attn_ab_s23.log; exit 1; }
  done
done
unset VSTYLER_LIB
grep -v "Warning\|amdgpu.ids" gpurun_out/r5_attn_ab_s23.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-e2e > gpurun_out/r5_bench_s23.json 2> gpurun_out/r5_bench_s23.err || { tail -20 gpurun_out/r5_bench_s23.err; exit 1; }
cut -c1-200 gpurun_out/r5_bench_s23.json
