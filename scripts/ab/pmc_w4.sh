#!/bin/bash
# PMC passes of scripts/pmc.sh (P1-P4) for the 14B FFN-up GEMM (59 280 x 13 824 x 5120) on the
# hand-written 4-wave kernel (VS_GEMM_KERNEL=4w), then its summary
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
OUT=$R/gpurun_out/pmc_gemm_w4
mkdir -p $OUT
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_LDS_UNALIGNED_STALL SQ_INSTS_MFMA SQ_INSTS_VALU"
P3="FETCH_SIZE"
P4="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  VS_GEMM_BACKEND=vstyler VSTYLER_GEMM_TILE=256 VS_GEMM_KERNEL=4w timeout -k 10 240 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT -o p$i -- python3 $R/tests/probes/kernel_pmc.py gemm > $OUT/p$i.log 2>&1 || { tail -5 $OUT/p$i.log; exit 1; }
done
cd $R
python3 scripts/pmc_summary.py gemm_w4 gemm_bf16_tn_4w
