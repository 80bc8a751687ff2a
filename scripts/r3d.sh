set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gemm8p_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gemm8p_r3d.log 2>&1 || { tail -40 gpurun_out/pytest_gemm8p_r3d.log; exit 1; }
tail -3 gpurun_out/pytest_gemm8p_r3d.log
timeout -k 10 300 python -u tests/probes/gemm8p_ab.py 59280 7410 > gpurun_out/gemm8p_ab_r3d.log 2>&1; cat gpurun_out/gemm8p_ab_r3d.log | grep -v amdgpu.ids
