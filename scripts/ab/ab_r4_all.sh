#!/bin/bash
# same-box step A/B: r4 default routing vs every GEMM on the hand-written kernels
# (VS_GEMM_BACKEND=vstyler) vs + the GELU FFN-up (VS_GEMM_OWN=3), interleaved, + a rocprof
# kernel-stats run of the all-hand-written step
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
R=$(pwd)
mkdir -p gpurun_out
LOG=gpurun_out/bench_r4_all_ab.log
run() {
  echo "== $1" | tee -a $LOG
  env $2 timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e 2>/dev/null | tee -a $LOG || exit 1
}
run default VS_GEMM_OWN=2
run all VS_GEMM_BACKEND=vstyler
run own3 VS_GEMM_OWN=3
run default VS_GEMM_OWN=2
run all VS_GEMM_BACKEND=vstyler
run own3 VS_GEMM_OWN=3
cd /tmp && export TMPDIR=/tmp
VS_GEMM_BACKEND=vstyler timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_all -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > $R/gpurun_out/prof_all.log 2>&1 || { tail -20 $R/gpurun_out/prof_all.log; exit 1; }
