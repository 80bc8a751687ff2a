#!/bin/bash
# r5 GPU session 28c: halo conv, XCD-aware frame-fastest block order -- VAE tests, conv probe (halo vs per-tap)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_vae_gpu.py -q -rfE --timeout 120 --timeout-method thread > gpurun_out/r5_vae_tests_s28c.log 2>&1
rc=$?; grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r5_vae_tests_s28c.log | tail -8
if [ $rc -ne 0 ]; then tail -40 gpurun_out/r5_vae_tests_s28c.log; exit 1; fi
VCP_HALO_ONLY=1 timeout -k 10 200 python -u tests/probes/vae_conv_probe.py > gpurun_out/r5_vae_conv_probe_s28c.log 2>&1 || { tail -20 gpurun_out/r5_vae_conv_probe_s28c.log; exit 1; }
grep -v "Warning\|amdgpu.ids" gpurun_out/r5_vae_conv_probe_s28c.log
