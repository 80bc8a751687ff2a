#!/bin/bash
# scratch A/B driver for one gpurun call (not part of the product)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
AB_VARIANTS=s,lt timeout -k 10 400 python -u tests/probes/gemm8p_ab.py 3705 14820 2>&1 | grep -v amdgpu.ids | tee gpurun_out/gemm_stag_ab2.log
