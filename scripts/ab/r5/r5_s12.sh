#!/bin/bash
# r5 GPU session 12: split-tail K pieces launched before the persistent GEMM blocks (queue schedule)
# -- GEMM tests (bf16 + fp8 + queue), the held-CU probe, the 14B bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
fault() { grep -qiE "memory access fault|illegal address|HSA_STATUS_ERROR|hipErrorLaunchFailure|core dumped" "$1"; }
timeout -k 10 600 python -u -m pytest tests/test_gemm_queue_gpu.py tests/test_kernels_gpu.py tests/test_fp8_gpu.py tests/test_gemm8p_gpu.py -k "gemm" -q -rfE --timeout 300 --timeout-method thread > gpurun_out/r5_gemm_tests_s12.log 2>&1
rc=$?; grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r5_gemm_tests_s12.log | tail -8
if [ $rc -ne 0 ] || fault gpurun_out/r5_gemm_tests_s12.log; then tail -30 gpurun_out/r5_gemm_tests_s12.log; exit 1; fi
timeout -k 10 400 python -u tests/probes/cu_hold.py > gpurun_out/r5_cu_hold_s12.log 2>&1 || { tail -20 gpurun_out/r5_cu_hold_s12.log; exit 1; }
grep -v Warning gpurun_out/r5_cu_hold_s12.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r5_bench_s12.json 2> gpurun_out/r5_bench_s12.err || { tail -20 gpurun_out/r5_bench_s12.err; exit 1; }
cut -c1-300 gpurun_out/r5_bench_s12.json
