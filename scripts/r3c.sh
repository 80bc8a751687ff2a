set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gemm8p_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gemm8p_r3c.log 2>&1 || { tail -40 gpurun_out/pytest_gemm8p_r3c.log; exit 1; }
tail -3 gpurun_out/pytest_gemm8p_r3c.log
timeout -k 10 300 python -u tests/probes/gemm8p_ab.py 59280 7410 > gpurun_out/gemm8p_ab_r3c.log 2>&1; grep -v amdgpu.ids gpurun_out/gemm8p_ab_r3c.log
timeout -k 10 300 python -u tests/probes/gemm_fp8_8p_ab.py 59280 > gpurun_out/gemm_fp8_ab_r3c.log 2>&1; grep -v amdgpu.ids gpurun_out/gemm_fp8_ab_r3c.log
timeout -k 10 300 python -u tests/probes/c3_debug.py > gpurun_out/c3_debug_r3c.log 2>&1; grep -v amdgpu.ids gpurun_out/c3_debug_r3c.log
