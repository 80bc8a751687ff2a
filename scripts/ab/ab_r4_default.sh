#!/bin/bash
# same-box A/B of the r4 default routing against the r3 routing, bf16 headline step and config 5 (fp8):
#   bf16: default (residual GEMMs on the 4-wave kernel) vs VS_GEMM_OWN=0 (r3: hipBLASLt + fused residual-LN)
#   fp8:  default (4-wave fp8 kernel except q|k|v) vs VS_FP8_BACKEND=lt (r3: hipBLASLt fp8 everywhere)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
LOG=gpurun_out/bench_r4_default_ab.log
run() {
  echo "== $1" | tee -a $LOG
  env $2 timeout -k 10 300 python -u bench.py $3 --no-cpu-baseline --no-e2e 2>/dev/null | tee -a $LOG || exit 1
}
run bf16-r4 VS_GEMM_OWN=2 "--steps 5 --warmup 1"
run bf16-r3 VS_GEMM_OWN=0 "--steps 5 --warmup 1"
run fp8-r4 VS_FP8_BACKEND=auto "--config fp8 --steps 4 --warmup 1"
run fp8-r3 VS_FP8_BACKEND=lt "--config fp8 --steps 4 --warmup 1"
run bf16-r4 VS_GEMM_OWN=2 "--steps 5 --warmup 1"
run bf16-r3 VS_GEMM_OWN=0 "--steps 5 --warmup 1"
