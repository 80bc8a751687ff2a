#!/bin/bash
# scratch: fp8 8-phase GEMM with hoisted DMA offsets -- fp8 tests, A/B vs the previous build
# (diag_fp8base), then the per-rank SP = 8 step with the hoisted bf16 offsets
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gemm8p_gpu.py tests/test_fp8_gpu.py > gpurun_out/fp8_tests.log 2>&1 || { tail -30 gpurun_out/fp8_tests.log; exit 1; }
tail -1 gpurun_out/fp8_tests.log
L=video-styler_amd/vstyler/lib
for r in 1 2; do
  for v in base new; do
    if [ $v = new ]; then LIB=$L/libvstyler.so; else LIB=$L/diag_fp8base/libvstyler.so; fi
    echo "== $v round $r" | tee -a gpurun_out/fp8_preoff_ab.log
    VSTYLER_LIB=$LIB timeout -k 10 150 python -u tests/probes/gemm_fp8_ab.py 59280 7410 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/fp8_preoff_ab.log || exit 1
  done
done
SPC_REPS=3 timeout -k 10 400 python -u tests/probes/sp_rank_compute.py 8 4 2>&1 | grep -v amdgpu.ids | tee gpurun_out/sp_rank_480p_preoff.log
