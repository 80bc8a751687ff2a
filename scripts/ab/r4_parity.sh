#!/bin/bash
# r4 GPU parity session: the production-shape parity tests (C5 fp8 both routes, C4 block pair at
# 223 200 GEMM rows, VAE 480x832 3x3 tiles), then -- last, after a clean run only -- the SP graph
# capture test at RCCL world 1.  A test failure (pytest rc 1) still lets the next step run; a time
# limit, crash or GPU fault ends the session.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 750 python -u -m pytest -v -s --timeout 600 --timeout-method thread -m "gpu or gpu_long" tests/test_production_c4c5_gpu.py \
  > gpurun_out/prod_c4c5.log 2>&1
rc=$?
grep -E "^(PASSED|FAILED)|passed|failed" gpurun_out/prod_c4c5.log | tail -6
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "production tests ended with rc $rc: stopping"; exit 1; fi
if grep -qiE "memory access fault|illegal address|HSA_STATUS_ERROR|hipErrorLaunchFailure|core dumped" gpurun_out/prod_c4c5.log; then
  echo "GPU fault reported: stopping"; exit 1; fi
timeout -k 10 330 python -u -m pytest -v -s --timeout 300 --timeout-method thread \
  tests/test_sp.py::test_ulysses_rccl_world1_graph_capture > gpurun_out/sp_capture.log 2>&1
echo "sp capture rc $?"
