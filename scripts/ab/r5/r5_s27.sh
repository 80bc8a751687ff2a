#!/bin/bash
# r5 GPU session 27: the patch-resident VAE conv (vae_conv_halo_kernel) -- VAE GPU tests, conv probe
# halo vs per-tap, the 832x480x73 tiled encode / decode.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_vae_gpu.py -q -rfE --timeout 120 --timeout-method thread > gpurun_out/r5_vae_tests_s27.log 2>&1
rc=$?; grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r5_vae_tests_s27.log | tail -8
if [ $rc -ne 0 ]; then tail -40 gpurun_out/r5_vae_tests_s27.log; exit 1; fi
timeout -k 10 200 python -u tests/probes/vae_conv_probe.py > gpurun_out/r5_vae_conv_probe_s27.log 2>&1 || { tail -20 gpurun_out/r5_vae_conv_probe_s27.log; exit 1; }
grep -v "Warning\|amdgpu.ids" gpurun_out/r5_vae_conv_probe_s27.log
timeout -k 10 300 python -u tests/probes/vae_bench.py > gpurun_out/r5_vae_bench_s27.log 2>&1 || { tail -20 gpurun_out/r5_vae_bench_s27.log; exit 1; }
grep -v "Warning\|amdgpu.ids" gpurun_out/r5_vae_bench_s27.log
