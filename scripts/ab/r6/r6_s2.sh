#!/bin/bash
# r6 step 2: split-tail pieces from the queue's piece pool -- GEMM tests, the held-CU probe (GEMMs), the 14B bench
set -o pipefail
mkdir -p gpurun_out
fault() { grep -qiE "memory access fault|illegal address|HSA_STATUS_ERROR|hipErrorLaunchFailure|core dumped" "$1"; }
timeout -k 10 600 python -u -m pytest tests/test_gemm_queue_gpu.py tests/test_kernels_gpu.py tests/test_fp8_gpu.py tests/test_gemm8p_gpu.py -k "gemm" -q -rfE --timeout 300 --timeout-method thread > gpurun_out/r6_gemm_tests_s2.log 2>&1
rc=$?; grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r6_gemm_tests_s2.log | tail -8
if [ $rc -ne 0 ] || fault gpurun_out/r6_gemm_tests_s2.log; then tail -30 gpurun_out/r6_gemm_tests_s2.log; exit 1; fi
CH_ONLY=ffn timeout -k 10 500 python -u tests/probes/cu_hold.py > gpurun_out/r6_cu_hold_s2.log 2>&1 || { tail -20 gpurun_out/r6_cu_hold_s2.log; exit 1; }
grep -v Warning gpurun_out/r6_cu_hold_s2.log
for i in 1 2; do
for pq in 1 0; do
VSTYLER_OPTS=piece_queue=$pq timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-e2e --steps 5 --warmup 2 > gpurun_out/r6_bench_pq${pq}_$i.json 2> gpurun_out/r6_bench_pq${pq}_$i.err || { tail -20 gpurun_out/r6_bench_pq${pq}_$i.err; exit 1; }
echo "piece_queue=$pq round $i: $(cut -c1-200 gpurun_out/r6_bench_pq${pq}_$i.json)"
done
done
