#!/bin/bash
# PMC passes P3/P4 (HBM bytes, L2 hit) for the 14B FFN-up GEMM: hand-written kernel vs hipBLASLt.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
P3="FETCH_SIZE"
P4="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
for BE in vstyler lt; do
  OUT=$R/gpurun_out/pmc_gemm_$BE
  mkdir -p $OUT
  i=2
  for P in "$P3" "$P4"; do
    i=$((i+1))
    VS_GEMM_BACKEND=$BE VSTYLER_GEMM_TILE=256 timeout -k 10 240 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT -o p$i -- python3 $R/tests/probes/kernel_pmc.py gemm > $OUT/p$i.log 2>&1 || { tail -5 $OUT/p$i.log; exit 1; }
  done
done
cd $R
python3 scripts/pmc_summary.py gemm_vstyler gemm_bf16_tn_8p
python3 scripts/pmc_summary.py gemm_lt Cijk
