#!/bin/bash
# r5 GPU session 44: VAE rmsnorm with 16 lanes per pixel (whole-row coalesced loads / stores) --
# VAE tests, rmsnorm probe, the 832x480x73 encode / decode
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_vae_gpu.py tests/test_vace_e2e_gpu.py -q -rfE --timeout 200 --timeout-method thread > gpurun_out/r5_vae_tests_s44.log 2>&1
rc=$?; grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r5_vae_tests_s44.log | tail -6
if [ $rc -ne 0 ]; then tail -40 gpurun_out/r5_vae_tests_s44.log; exit 1; fi
timeout -k 10 120 python -u tests/probes/vae_rmsnorm_bench.py > gpurun_out/r5_vae_rmsnorm_s44.log 2>&1 || { tail -20 gpurun_out/r5_vae_rmsnorm_s44.log; exit 1; }
grep -v "Warning\|amdgpu.ids" gpurun_out/r5_vae_rmsnorm_s44.log
timeout -k 10 300 python -u tests/probes/vae_bench.py > gpurun_out/r5_vae_bench_s44.log 2>&1 || { tail -20 gpurun_out/r5_vae_bench_s44.log; exit 1; }
grep -v "Warning\|amdgpu.ids" gpurun_out/r5_vae_bench_s44.log
