#!/bin/bash
# same-box step A/B: default vs + FFN-up on the 4-wave kernel (VS_GEMM_OWN=3) vs the same with raster
# groups of 2 M-tiles (VS_GEMM_GM=2: FFN-up 1456 vs 1418 TF/s alone, gemm_gm_w4_ab.log), interleaved
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
LOG=gpurun_out/bench_r4_gm2_ab.log
run() {
  echo "== $1" | tee -a $LOG
  env $2 timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e 2>/dev/null | tee -a $LOG || exit 1
}
for i in 1 2; do
  run default VS_GEMM_OWN=2
  run own3 VS_GEMM_OWN=3
  run own3gm2 "VS_GEMM_OWN=3 VS_GEMM_GM=2"
  run gm2 "VS_GEMM_OWN=2 VS_GEMM_GM=2"
done
