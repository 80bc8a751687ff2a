#!/bin/bash
# same-box bench A/B: default routing (hipBLASLt for the SP=1 block GEMMs) vs every GEMM on the
# hand-written 4-wave kernel (VS_GEMM_BACKEND=vstyler VS_GEMM_KERNEL=4w), interleaved; then a
# rocprof kernel-stats run of the 4-wave variant (step breakdown)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
R=$(pwd)
mkdir -p gpurun_out
LOG=gpurun_out/bench_w4_ab.log
for i in 1 2; do
  for v in auto w4; do
    echo "== $v" | tee -a $LOG
    if [ $v = auto ]; then E="VS_GEMM_KERNEL=8p"; else E="VS_GEMM_BACKEND=vstyler VS_GEMM_KERNEL=4w"; fi
    env $E timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e 2>/dev/null | tee -a $LOG || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
VS_GEMM_BACKEND=vstyler VS_GEMM_KERNEL=4w timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_w4 -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > $R/gpurun_out/prof_w4.log 2>&1 || { tail -20 $R/gpurun_out/prof_w4.log; exit 1; }
find $R/gpurun_out/prof_w4 -name "*stats*"
