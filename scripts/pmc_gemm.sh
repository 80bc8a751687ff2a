#!/bin/bash
# PMC passes P1/P2 of scripts/pmc.sh for the 14B FFN-up GEMM on the hand-written kernel and on hipBLASLt.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_LDS_UNALIGNED_STALL SQ_INSTS_MFMA SQ_INSTS_VALU"
for BE in vstyler lt; do
  OUT=$R/gpurun_out/pmc_gemm_$BE
  mkdir -p $OUT
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    VS_GEMM_BACKEND=$BE VSTYLER_GEMM_TILE=256 timeout -k 10 240 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT -o p$i -- python3 $R/tests/probes/kernel_pmc.py gemm > $OUT/p$i.log 2>&1 || { tail -5 $OUT/p$i.log; exit 1; }
  done
done
cd $R
python3 scripts/pmc_summary.py gemm_vstyler gemm_bf16_tn_8p
python3 scripts/pmc_summary.py gemm_lt Cijk
