set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attn or attention" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_attn_r3n.log 2>&1 || { tail -40 gpurun_out/pytest_attn_r3n.log; exit 1; }
tail -3 gpurun_out/pytest_attn_r3n.log
timeout -k 10 300 python -u -m pytest tests/test_attention_production_gpu.py -x -q -s --timeout 200 --timeout-method thread > gpurun_out/pytest_attnprod_r3n.log 2>&1 || { tail -40 gpurun_out/pytest_attnprod_r3n.log; exit 1; }
grep -E "worst|passed|failed" gpurun_out/pytest_attnprod_r3n.log
ATTN_AB=8,4 timeout -k 10 300 python -u tests/probes/attn_bench.py 2>&1 | tee gpurun_out/attn_ab_r3n.log
