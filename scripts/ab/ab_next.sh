#!/bin/bash
# scratch A/B driver for one gpurun call (not part of the product)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
for w in 1 0 1 0; do
  echo "== VS_GEMM_WIDE=$w" | tee -a gpurun_out/gemm_wide_ab2.log
  VS_GEMM_WIDE=$w AB_VARIANTS=vstyler,lt timeout -k 10 300 python -u tests/probes/gemm_ab.py 59280 7410 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/gemm_wide_ab2.log || exit 1
done
