set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_attention_production_gpu.py -v -s --timeout 200 --timeout-method thread -k fused_qkv > gpurun_out/pytest_attnviews_r3g.log 2>&1; grep -E "PASS|FAIL|worst|Error" gpurun_out/pytest_attnviews_r3g.log | head -20
timeout -k 10 300 python -u -m pytest tests/test_gemm8p_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gemm8p_r3g.log 2>&1 || { tail -40 gpurun_out/pytest_gemm8p_r3g.log; exit 1; }
tail -2 gpurun_out/pytest_gemm8p_r3g.log
timeout -k 10 300 python -u tests/probes/gemm8p_ab.py 59280 7410 > gpurun_out/gemm8p_ab_r3g.log 2>&1; grep -v amdgpu.ids gpurun_out/gemm8p_ab_r3g.log
