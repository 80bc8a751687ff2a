#!/bin/bash
# same-box bench A/B of the SP = 1 GEMM routing levels (VS_GEMM_OWN; see own_wins in gemm.hip),
# interleaved; lvl 0 = r3 routing on the 4-wave kernel, 1 = + o-proj, 2 = + FFN-down, 3 = + FFN-up
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
LOG=gpurun_out/bench_route2_ab.log
run() {
  echo "== $1" | tee -a $LOG
  env $2 timeout -k 10 240 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e 2>/dev/null | tee -a $LOG || exit 1
}
run own1 VS_GEMM_OWN=1
run own3 VS_GEMM_OWN=3
run own2 VS_GEMM_OWN=2
run own0 VS_GEMM_OWN=0
run own3 VS_GEMM_OWN=3
run own1 VS_GEMM_OWN=1
