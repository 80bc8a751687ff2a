#!/bin/bash
# PMC passes (P1 stall mix, P2 MFMA/LDS, P3 HBM fetch) of the 59 280 x 13 824 x 5120 GEMM on the
# persistent 4-wave kernel and on hipBLASLt, one rocprofv3 run per pass, then both summaries
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
P3="FETCH_SIZE"
for V in w4 lt; do
  OUT=$R/gpurun_out/pmc_gemm_$V
  mkdir -p $OUT
  if [ $V = w4 ]; then B=vstyler; else B=lt; fi
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    VS_GEMM_BACKEND=$B timeout -k 10 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT -o p$i -- python3 $R/tests/probes/kernel_pmc.py gemm > $OUT/p$i.log 2>&1 || { tail -5 $OUT/p$i.log; exit 1; }
  done
done
cd $R
python3 scripts/pmc_summary.py gemm_w4 gemm_bf16_tn_4w
python3 scripts/pmc_summary.py gemm_lt Cijk
