#!/bin/bash
# r5 GPU session 10: attn_fwd_w4 item switch -- all sixteen Q loads issued before the conversion and
# the next item's Q prefetched in the first tile.  Attention tests, switch stamps, key-count sweep
# and the 14B step, the new library against the previous one (lib/old), interleaved.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
OLD=$R/video-styler_amd/vstyler/lib/old/libvstyler.so
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_attention_production_gpu.py -k "attention or attn" -q -rfE --timeout 300 --timeout-method thread > gpurun_out/r5_attn_tests_s10.log 2>&1
rc=$?; tail -3 gpurun_out/r5_attn_tests_s10.log
if [ $rc -ne 0 ]; then tail -30 gpurun_out/r5_attn_tests_s10.log; exit 1; fi
VSTYLER_LIB=$R/video-styler_amd/vstyler/lib/diag_w4st/libvstyler.so W4S_SKV=512 timeout -k 10 200 python -u tests/probes/w4_stamps.py > gpurun_out/r5_w4_switch_cross_s10.log 2>&1 || { tail -20 gpurun_out/r5_w4_switch_cross_s10.log; exit 1; }
grep -v Warning gpurun_out/r5_w4_switch_cross_s10.log
VSTYLER_LIB=$R/video-styler_amd/vstyler/lib/diag_w4st/libvstyler.so timeout -k 10 200 python -u tests/probes/w4_stamps.py > gpurun_out/r5_w4_switch_self_s10.log 2>&1 || { tail -20 gpurun_out/r5_w4_switch_self_s10.log; exit 1; }
grep -v Warning gpurun_out/r5_w4_switch_self_s10.log
for lib in new old; do
  if [ $lib = old ]; then export VSTYLER_LIB=$OLD; else unset VSTYLER_LIB; fi
  echo "== $lib" >> gpurun_out/r5_attn_skv_s10.log
  SKV=512,1024,4096 timeout -k 10 300 python -u tests/probes/attn_skv_sweep.py >> gpurun_out/r5_attn_skv_s10.log 2>&1 || { tail -20 gpurun_out/r5_attn_skv_s10.log; exit 1; }
done
unset VSTYLER_LIB
grep -v Warning gpurun_out/r5_attn_skv_s10.log
for i in 1 2; do
  for lib in new old; do
    if [ $lib = old ]; then export VSTYLER_LIB=$OLD; else unset VSTYLER_LIB; fi
    echo "== $lib" >> gpurun_out/r5_bench_ab_s10.log
    timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-e2e >> gpurun_out/r5_bench_ab_s10.log 2>&1 || { tail -20 gpurun_out/r5_bench_ab_s10.log; exit 1; }
  done
done
unset VSTYLER_LIB
grep -E "^==|\"value\"" gpurun_out/r5_bench_ab_s10.log | sed 's/"unit.*"roofline"/ .../' | cut -c1-220
