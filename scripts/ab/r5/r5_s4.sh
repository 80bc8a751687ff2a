#!/bin/bash
# r5 GPU session 4: -m gpu suite (C4 sampled rows, one fixed tile per block, small-grid rule), the
# held-CU probe (queue vs static lists), the context-GEMM A/B vs the A/B build's library route, and
# the 14B bench.  A crash, fault or time limit ends the session.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
fault() { grep -qiE "memory access fault|illegal address|HSA_STATUS_ERROR|hipErrorLaunchFailure|core dumped" "$1"; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rfE --timeout 300 --timeout-method thread > gpurun_out/r5_pytest_gpu_s4.log 2>&1
rc=$?; grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r5_pytest_gpu_s4.log | tail -12
grep -E "C4 14B|VAE tiled" gpurun_out/r5_pytest_gpu_s4.log | head -4
if [ $rc -gt 1 ] || fault gpurun_out/r5_pytest_gpu_s4.log; then tail -30 gpurun_out/r5_pytest_gpu_s4.log; exit 1; fi
timeout -k 10 400 python -u tests/probes/cu_hold.py > gpurun_out/r5_cu_hold.log 2>&1 || { tail -20 gpurun_out/r5_cu_hold.log; exit 1; }
cat gpurun_out/r5_cu_hold.log
AB_MODEL=ctx AB_VARIANTS=auto,t128,lt VSTYLER_LIB=$R/video-styler_amd/vstyler/lib/ab/libvstyler.so \
  timeout -k 10 200 python -u tests/probes/gemm_ab.py 1024 > gpurun_out/r5_gemm_ab_ctx.log 2>&1 || { tail -20 gpurun_out/r5_gemm_ab_ctx.log; exit 1; }
grep -v Warning gpurun_out/r5_gemm_ab_ctx.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r5_bench_s4.json 2> gpurun_out/r5_bench_s4.err || { tail -20 gpurun_out/r5_bench_s4.err; exit 1; }
cat gpurun_out/r5_bench_s4.json
