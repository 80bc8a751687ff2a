#!/bin/bash
# scratch A/B driver (not part of the product)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
VS_GEMM_IMPL=r timeout -k 10 300 python -u -m pytest tests/test_gemm8p_gpu.py -x -q --timeout 120 --timeout-method thread -k "not fp8" 2>&1 | tail -3
AB_VARIANTS=r,s,lt timeout -k 10 400 python -u tests/probes/gemm8p_ab.py 59280 7410 2>&1 | grep -v amdgpu.ids | tee gpurun_out/gemm_w4r_ab.log
