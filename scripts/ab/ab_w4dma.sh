#!/bin/bash
# same-box A/B of the 4-wave GEMM's DMA issue: the built library (one-instruction DMAs, M0 stepped
# by SALU) vs the previous source built into lib/diag_prev (v_add + hazard nop per DMA), interleaved
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
LOG=gpurun_out/gemm_w4dma_ab.log
for i in 1 2; do
  echo "== new" | tee -a $LOG
  AB_VARIANTS=w4,lt timeout -k 10 200 python -u tests/probes/gemm_ab.py 59280 7410 2>&1 | grep TF | tee -a $LOG || exit 1
  echo "== prev" | tee -a $LOG
  VSTYLER_LIB=video-styler_amd/vstyler/lib/diag_prev/libvstyler.so AB_VARIANTS=w4 timeout -k 10 200 python -u tests/probes/gemm_ab.py 59280 7410 2>&1 | grep TF | tee -a $LOG || exit 1
done
