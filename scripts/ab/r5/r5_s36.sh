#!/bin/bash
# r5 GPU session 36: halo conv with the nearest-x2 upsample gather -- VAE tests, conv probe (halo vs per-tap)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_vae_gpu.py -q -rfE --timeout 120 --timeout-method thread > gpurun_out/r5_vae_tests_s36.log 2>&1
rc=$?; grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r5_vae_tests_s36.log | tail -8
if [ $rc -ne 0 ]; then tail -40 gpurun_out/r5_vae_tests_s36.log; exit 1; fi
VCP_HALO_ONLY=1 timeout -k 10 200 python -u tests/probes/vae_conv_probe.py > gpurun_out/r5_vae_conv_probe_s36.log 2>&1 || { tail -20 gpurun_out/r5_vae_conv_probe_s36.log; exit 1; }
grep -v "Warning\|amdgpu.ids" gpurun_out/r5_vae_conv_probe_s36.log
timeout -k 10 300 python -u tests/probes/vae_bench.py > gpurun_out/r5_vae_bench_s36.log 2>&1 || { tail -20 gpurun_out/r5_vae_bench_s36.log; exit 1; }
grep -v "Warning\|amdgpu.ids" gpurun_out/r5_vae_bench_s36.log
