#!/bin/bash
# the VAE flash attention: its parity tests, the VAE suite, and the flash vs GEMM-route A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_vae_attention_gpu.py tests/test_vae_gpu.py tests/test_abi.py -q -x -rfE --timeout 200 --timeout-method thread > gpurun_out/pytest_vaeattn.log 2>&1 || { tail -40 gpurun_out/pytest_vaeattn.log; exit 1; }
tail -3 gpurun_out/pytest_vaeattn.log
timeout -k 10 300 python -u tests/probes/vae_attn_ab.py > gpurun_out/vae_attn_ab.log 2>&1 || { tail -30 gpurun_out/vae_attn_ab.log; exit 1; }
cat gpurun_out/vae_attn_ab.log
VAE_REPS=1 timeout -k 10 300 python -u tests/probes/vae_bench.py > gpurun_out/vae_bench_flash.log 2>&1 || { tail -30 gpurun_out/vae_bench_flash.log; exit 1; }
cat gpurun_out/vae_bench_flash.log
