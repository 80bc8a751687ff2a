#!/bin/bash
# L2->fabric read bytes (FETCH_SIZE) of the FFN-up GEMM at 59 280 and 7410 rows on the 4-wave kernel
# and hipBLASLt: does the 4-wave kernel's extra traffic grow with the tiles per workgroup (drift)?
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for M in 59280 7410; do
  for V in w4 lt; do
    OUT=$R/gpurun_out/pmc_fetch_${V}_$M
    mkdir -p $OUT
    if [ $V = w4 ]; then B=vstyler; else B=lt; fi
    KP_M=$M VS_GEMM_BACKEND=$B timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT -o p1 -- python3 $R/tests/probes/kernel_pmc.py gemm > $OUT/p1.log 2>&1 || { tail -5 $OUT/p1.log; exit 1; }
  done
done
cd $R
for M in 59280 7410; do
  python3 scripts/pmc_summary.py fetch_w4_$M gemm_bf16_tn_4w | grep -E "median|HBM read"
  python3 scripts/pmc_summary.py fetch_lt_$M Cijk | grep -E "median|HBM read"
done
