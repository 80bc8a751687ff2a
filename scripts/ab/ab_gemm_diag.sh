#!/bin/bash
# scratch: timing of GEMM diagnostic builds (VSTYLER_LIB per build) on the 59280-row 14B shapes
#   bash scripts/ab/ab_gemm_diag.sh <variant for AB_VARIANTS> <diag name>...
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
V=$1; shift
for v in base "$@"; do
  if [ $v = base ]; then L=$PWD/video-styler_amd/vstyler/lib/libvstyler.so; else L=$PWD/video-styler_amd/vstyler/lib/diag_$v/libvstyler.so; fi
  echo "== $v" | tee -a gpurun_out/gemm_diag.log
  VSTYLER_LIB=$L AB_VARIANTS=$V timeout -k 10 200 python -u tests/probes/gemm_ab.py 59280 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/gemm_diag.log || exit 1
done
