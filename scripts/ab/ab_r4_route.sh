#!/bin/bash
# same-box bench A/B of the SP = 1 GEMM routing, interleaved:
#   r3   VS_GEMM_KERNEL=8p          (r3 routing: hipBLASLt for the block GEMMs, 8-phase kernel elsewhere)
#   r4   default                    (persistent 4-wave kernel, + the gate-residual o-proj on it)
#   own2 VS_GEMM_OWN=2               (+ the gate-residual FFN-down)
#   all  VS_GEMM_BACKEND=vstyler    (every GEMM on the 4-wave kernel)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
LOG=gpurun_out/bench_route_ab.log
run() {
  echo "== $1" | tee -a $LOG
  env $2 timeout -k 10 240 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e 2>/dev/null | tee -a $LOG || exit 1
}
run r3 VS_GEMM_KERNEL=8p
run r4 VS_GEMM_OWN=1
run own2 VS_GEMM_OWN=2
run all VS_GEMM_BACKEND=vstyler
run r4 VS_GEMM_OWN=1
run r3 VS_GEMM_KERNEL=8p
