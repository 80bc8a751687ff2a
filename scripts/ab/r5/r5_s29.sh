#!/bin/bash
# r5 GPU session 29: where the halo conv's time goes -- diagnostic builds without the DMA (1), without
# the MFMAs (2), without the per-stage DMA wait (3), against the product build (conv probe, halo only)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
L=$R/video-styler_amd/vstyler/lib
for lib in prod halo1 halo2 halo3 prod; do
  if [ $lib = prod ]; then unset VSTYLER_LIB; else export VSTYLER_LIB=$L/diag_$lib/libvstyler.so; fi
  echo "== $lib" >> gpurun_out/r5_halo_diag_s29.log
  VCP_HALO_ONLY=1 timeout -k 10 120 python -u tests/probes/vae_conv_probe.py >> gpurun_out/r5_halo_diag_s29.log 2>&1 || { tail -20 gpurun_out/r5_halo_diag_s29.log; exit 1; }
done
grep -v "Warning\|amdgpu.ids\|halo 0" gpurun_out/r5_halo_diag_s29.log
