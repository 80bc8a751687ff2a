set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gemm8p_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gemm8p_r3b.log 2>&1 || { tail -40 gpurun_out/pytest_gemm8p_r3b.log; exit 1; }
tail -3 gpurun_out/pytest_gemm8p_r3b.log
timeout -k 10 300 python -u tests/probes/gemm8p_ab.py 59280 7410 > gpurun_out/gemm8p_ab_r3b.log 2>&1; cat gpurun_out/gemm8p_ab_r3b.log
timeout -k 10 400 python -u -m pytest tests/test_attention_production_gpu.py tests/test_production_model_gpu.py -v -s --timeout 200 --timeout-method thread > gpurun_out/pytest_prod_r3b.log 2>&1; grep -E "PASS|FAIL|Error|worst|floor" gpurun_out/pytest_prod_r3b.log | tail -30
