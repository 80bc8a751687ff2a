#!/bin/bash
# same-box A/B, bf16 headline step: nt output stores of the 4-wave GEMM epilogue (default build) vs
# plain stores (abl_nt0/, built with EXTRA=-DW4_OUT_CPOL=0), default routing (VS_GEMM_OWN=2), and the
# GELU FFN-up on the 4-wave kernel too (VS_GEMM_OWN=3, nt), interleaved
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
LOG=gpurun_out/bench_r4_nt_ab.log
run() {
  echo "== $1" | tee -a $LOG
  env $2 timeout -k 10 300 python -u bench.py $3 --no-cpu-baseline --no-e2e 2>/dev/null | tee -a $LOG || exit 1
}
for r in 1 2; do
  run own2-nt VS_GEMM_OWN=2 "--steps 5 --warmup 1"
  run own2-plain "VS_GEMM_OWN=2 VSTYLER_LIB=$PWD/abl_nt0/libvstyler.so" "--steps 5 --warmup 1"
  run own3-nt VS_GEMM_OWN=3 "--steps 5 --warmup 1"
done
