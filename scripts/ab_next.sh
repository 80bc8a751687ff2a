#!/bin/bash
# scratch A/B driver for one gpurun call (not part of the product)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
for c in torch native; do
  MASTER_PORT=$((29611 + RANDOM % 1000)) timeout -k 10 150 python -u tests/probes/sp_graph_probe.py $c 3 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/sp_graph_probe.log
  rc=$?; echo "rc=$rc" | tee -a gpurun_out/sp_graph_probe.log
  [ $rc -eq 0 ] || exit 1          # a timed-out / failed GPU step ends the call
done
bash scripts/ab_attn.sh dma dmaa dmab || exit 1
for w in 1 0 1 0; do
  echo "== VS_GEMM_WIDE=$w" | tee -a gpurun_out/gemm_wide_ab.log
  VS_GEMM_WIDE=$w AB_VARIANTS=vstyler timeout -k 10 300 python -u tests/probes/gemm_ab.py 59280 7410 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/gemm_wide_ab.log || exit 1
done
