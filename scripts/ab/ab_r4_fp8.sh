#!/bin/bash
# same-box config-5 (fp8) step A/B: auto (4-wave fp8 kernel, hipBLASLt for q|k|v) vs every fp8 GEMM on
# the MFMA kernel (vstyler) vs every fp8 GEMM on hipBLASLt (lt, the r3 default), interleaved
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
LOG=gpurun_out/bench_r4_fp8_ab.log
run() {
  echo "== $1" | tee -a $LOG
  VS_FP8_BACKEND=$1 timeout -k 10 300 python -u bench.py --config fp8 --steps 4 --warmup 1 --no-cpu-baseline --no-e2e 2>/dev/null | tee -a $LOG || exit 1
}
for i in 1 2; do run auto; run vstyler; run lt; done
