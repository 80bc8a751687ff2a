#!/bin/bash
# r6 step 3: the held-CU reserve plan (1-3 round GEMMs keep 1/16 of each round as pieces)
set -o pipefail
mkdir -p gpurun_out
fault() { grep -qiE "memory access fault|illegal address|HSA_STATUS_ERROR|hipErrorLaunchFailure|core dumped" "$1"; }
timeout -k 10 600 python -u -m pytest tests/test_gemm_queue_gpu.py tests/test_kernels_gpu.py tests/test_fp8_gpu.py tests/test_gemm8p_gpu.py -k "gemm" -q -rfE --timeout 300 --timeout-method thread > gpurun_out/r6_gemm_tests_s3.log 2>&1
rc=$?; grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r6_gemm_tests_s3.log | tail -8
if [ $rc -ne 0 ] || fault gpurun_out/r6_gemm_tests_s3.log; then tail -30 gpurun_out/r6_gemm_tests_s3.log; exit 1; fi
CH_ONLY=7410 timeout -k 10 500 python -u tests/probes/cu_hold.py > gpurun_out/r6_cu_hold_s3.log 2>&1 || { tail -20 gpurun_out/r6_cu_hold_s3.log; exit 1; }
grep -v Warning gpurun_out/r6_cu_hold_s3.log
