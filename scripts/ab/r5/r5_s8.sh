#!/bin/bash
# r5 GPU session 8: VAE conv (LDS swizzle conflict-free for the fragment reads, tap-cached gather
# addresses) -- VAE tests, then interleaved encode/decode timings of the new and the previous library;
# the attention key-count sweep (item-switch vs per-tile cost, both kernels).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_vae_gpu.py tests/test_production_c4c5_gpu.py -k "vae" -q -rfE --timeout 300 --timeout-method thread > gpurun_out/r5_vae_tests_s8.log 2>&1
rc=$?; tail -3 gpurun_out/r5_vae_tests_s8.log
if [ $rc -ne 0 ]; then tail -30 gpurun_out/r5_vae_tests_s8.log; exit 1; fi
for i in 1 2; do
  for lib in new old; do
    if [ $lib = old ]; then export VSTYLER_LIB=$R/video-styler_amd/vstyler/lib/old/libvstyler.so; else unset VSTYLER_LIB; fi
    echo "== $lib" >> gpurun_out/r5_vae_ab_s8.log
    VAE_REPS=1 timeout -k 10 200 python -u tests/probes/vae_bench.py >> gpurun_out/r5_vae_ab_s8.log 2>&1 || { tail -20 gpurun_out/r5_vae_ab_s8.log; exit 1; }
  done
done
unset VSTYLER_LIB
grep -E "^==|^(encode|decode)" gpurun_out/r5_vae_ab_s8.log
timeout -k 10 300 python -u tests/probes/attn_skv_sweep.py > gpurun_out/r5_attn_skv_s8.log 2>&1 || { tail -20 gpurun_out/r5_attn_skv_s8.log; exit 1; }
grep -v Warning gpurun_out/r5_attn_skv_s8.log
