#!/bin/bash
# r5 GPU session 38: halo conv v2 compute-side diagnostics (wrong results; timing only): no DMA (h1),
# no DMA + no barrier (h4), no DMA + no epilogue (h5), no DMA + no MFMA (h6), against the product build
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
L=$R/video-styler_amd/vstyler/lib
for lib in prod h1 h4 h5 h6 prod; do
  if [ $lib = prod ]; then unset VSTYLER_LIB; else export VSTYLER_LIB=$L/diag_$lib/libvstyler.so; fi
  echo "== $lib" >> gpurun_out/r5_halo_diag_s38.log
  VCP_HALO_ONLY=1 timeout -k 10 120 python -u tests/probes/vae_conv_probe.py >> gpurun_out/r5_halo_diag_s38.log 2>&1 || { tail -20 gpurun_out/r5_halo_diag_s38.log; exit 1; }
done
grep -v "Warning\|amdgpu.ids\|halo 0" gpurun_out/r5_halo_diag_s38.log
