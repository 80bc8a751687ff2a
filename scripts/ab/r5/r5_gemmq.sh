#!/bin/bash
# r5 GPU session 1: the 4-wave GEMMs with the XCD tile queues -- multi-tile bit-exact tests (queue and
# static lists), the existing GEMM / fp8 suites, then same-box A/Bs per 14B block GEMM (queue vs
# static vs hipBLASLt) and one default bench line.  Each GPU step has its own time limit; a crash,
# fault or time limit ends the session.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
fault() { grep -qiE "memory access fault|illegal address|HSA_STATUS_ERROR|hipErrorLaunchFailure|core dumped" "$1"; }
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_queue_gpu.py \
  > gpurun_out/r5_gemmq_tests.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r5_gemmq_tests.log | tail -2
if [ $rc -ne 0 ] || fault gpurun_out/r5_gemmq_tests.log; then tail -40 gpurun_out/r5_gemmq_tests.log; exit 1; fi
timeout -k 10 500 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gemm8p_gpu.py \
  tests/test_fp8_gpu.py tests/test_kernels_gpu.py -k "gemm" > gpurun_out/r5_gemm_suite.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r5_gemm_suite.log | tail -2
if [ $rc -gt 1 ] || fault gpurun_out/r5_gemm_suite.log; then tail -40 gpurun_out/r5_gemm_suite.log; exit 1; fi
timeout -k 10 300 python -u tests/probes/gemm_ab.py 59280 7410 > gpurun_out/r5_gemm_ab.log 2>&1 || { tail -20 gpurun_out/r5_gemm_ab.log; exit 1; }
cat gpurun_out/r5_gemm_ab.log
timeout -k 10 200 python -u tests/probes/gemm_fp8_ab.py 59280 > gpurun_out/r5_gemm_fp8_ab.log 2>&1 || { tail -20 gpurun_out/r5_gemm_fp8_ab.log; exit 1; }
cat gpurun_out/r5_gemm_fp8_ab.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/r5_bench_q.json 2> gpurun_out/r5_bench_q.err || { tail -20 gpurun_out/r5_bench_q.err; exit 1; }
cat gpurun_out/r5_bench_q.json
