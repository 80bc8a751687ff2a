#!/bin/bash
# scratch A/B driver for one gpurun call (not part of the product)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
VS_GEMM_IMPL=s timeout -k 10 300 python -u -m pytest tests/test_gemm8p_gpu.py -x -q --timeout 120 --timeout-method thread -k "not fp8" 2>&1 | tail -3
AB_VARIANTS=s,1b,8p,lt timeout -k 10 400 python -u tests/probes/gemm8p_ab.py 59280 7410 2>&1 | tee gpurun_out/gemm_stag_ab.log
VS_FP8_BACKEND=vs timeout -k 10 300 python -u -m pytest tests/test_gemm8p_gpu.py -x -q --timeout 120 --timeout-method thread -k "fp8" 2>&1 | tail -3
AB_VARIANTS=vs,vstyler,lt timeout -k 10 300 python -u tests/probes/gemm_fp8_8p_ab.py 59280 2>&1 | tee gpurun_out/gemm_fp8_stag_ab.log
