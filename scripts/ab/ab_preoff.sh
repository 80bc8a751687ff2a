#!/bin/bash
# scratch: the 8-phase GEMM with its eight DMA row offsets computed once (VS_GEMM_PREOFF=1 build)
# vs the per-stage offsets, interleaved rounds; hipBLASLt timed beside as the box control
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
L=video-styler_amd/vstyler/lib
for r in 1 2; do
  for v in base preoff; do
    if [ $v = base ]; then LIB=$L/libvstyler.so; else LIB=$L/diag_$v/libvstyler.so; fi
    echo "== $v round $r" | tee -a gpurun_out/preoff_ab.log
    VSTYLER_LIB=$LIB timeout -k 10 150 python -u tests/probes/gemm_ab.py 59280 7410 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/preoff_ab.log || exit 1
  done
done
