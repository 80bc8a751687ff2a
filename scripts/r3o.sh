set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_attention_production_gpu.py -x -q -s --timeout 200 --timeout-method thread > gpurun_out/pytest_attnprod_r3o.log 2>&1 || { tail -40 gpurun_out/pytest_attnprod_r3o.log; exit 1; }
grep -E "worst|passed|failed" gpurun_out/pytest_attnprod_r3o.log
ATTN_AB=8,4 timeout -k 10 300 python -u tests/probes/attn_bench.py 2>&1 | tee gpurun_out/attn_ab_r3o.log
echo "== PIPE=0 (compiler-scheduled body)"
VS_ATTN_W4_PIPE=0 ATTN_AB=4 timeout -k 10 300 python -u tests/probes/attn_bench.py 2>&1 | tee -a gpurun_out/attn_ab_r3o.log
