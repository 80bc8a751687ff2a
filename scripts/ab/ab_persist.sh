#!/bin/bash
# scratch: persistent 8-phase GEMM -- parity tests, then A/B against the one-tile-per-block grid
# (VS_GEMM_PERSIST=0) and hipBLASLt, then the SP graph probe over the native communicator (last)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gemm8p_gpu.py tests/test_kernels_gpu.py -k gemm > gpurun_out/persist_tests.log 2>&1 || { tail -30 gpurun_out/persist_tests.log; exit 1; }
tail -3 gpurun_out/persist_tests.log
for r in 1 2; do
  for p in 0 1; do
    echo "== VS_GEMM_PERSIST=$p round $r" | tee -a gpurun_out/persist_ab.log
    VS_GEMM_PERSIST=$p timeout -k 10 150 python -u tests/probes/gemm_ab.py 59280 7410 3705 2>&1 | tee -a gpurun_out/persist_ab.log || exit 1
  done
done
PYTHONFAULTHANDLER=1 VSTYLER_SP_GRAPH=1 timeout -k 10 120 python -u -X faulthandler tests/probes/sp_graph_probe.py native 3 > gpurun_out/sp_graph_native.log 2>&1
echo "sp native probe rc=$?"
