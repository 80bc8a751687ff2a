#!/bin/bash
# r5 GPU session 2 (queue build with the asm head atomic): per-GEMM A/B (queue / static / hipBLASLt),
# L2->fabric read bytes of the FFN-up and q|k|v GEMMs on each, then the headline step with the
# default routing vs every block GEMM on the hand-written kernels (VS_GEMM_BACKEND=vstyler),
# interleaved.  Each GPU step has its own time limit; a crash or time limit ends the session.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u tests/probes/gemm_ab.py 59280 > gpurun_out/r5_gemm_ab2.log 2>&1 || { tail -20 gpurun_out/r5_gemm_ab2.log; exit 1; }
grep -v Warning gpurun_out/r5_gemm_ab2.log
cd /tmp && export TMPDIR=/tmp
for N in 13824 15360; do
  for V in w4 w4s lt; do
    OUT=$R/gpurun_out/pmc_fetch_${V}_$N
    mkdir -p $OUT
    if [ $V = lt ]; then B=lt; else B=vstyler; fi
    if [ $V = w4s ]; then Q=0; else Q=1; fi
    KP_N=$N VS_GEMM_QUEUE=$Q VS_GEMM_BACKEND=$B timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT -o p1 -- python3 $R/tests/probes/kernel_pmc.py gemm > $OUT/p1.log 2>&1 || { tail -5 $OUT/p1.log; exit 1; }
  done
done
cd $R
for N in 13824 15360; do
  for V in w4 w4s; do python3 scripts/pmc_summary.py fetch_${V}_$N gemm_bf16_tn_4w | grep -E "median|HBM read"; done
  python3 scripts/pmc_summary.py fetch_lt_$N Cijk | grep -E "median|HBM read"
done
LOG=gpurun_out/r5_bench_own_ab.log
run() {
  echo "== $1" >> $LOG
  env $2 timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e >> $LOG 2>/dev/null || { echo "bench $1 failed"; exit 1; }
}
for r in 1 2; do
  run default "VS_GEMM_QUEUE=1"
  run all-own "VS_GEMM_BACKEND=vstyler"
done
grep -E "^==|value" $LOG | sed 's/"config.*//'
