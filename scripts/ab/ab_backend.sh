#!/bin/bash
# scratch: same-box bench A/B of the GEMM backend (default routing vs hand-written kernels only)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
for i in 1 2; do
  for be in auto vstyler; do
    echo "== VS_GEMM_BACKEND=$be" | tee -a gpurun_out/bench_backend_ab.log
    if [ $be = auto ]; then E=""; else E="VS_GEMM_BACKEND=$be"; fi
    env $E timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e 2>/dev/null | tee -a gpurun_out/bench_backend_ab.log || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
VS_GEMM_BACKEND=vstyler timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_own -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > $GRAFT_REPO_ROOT/gpurun_out/prof_own.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_own.log; exit 1; }
