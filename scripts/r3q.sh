set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_attention_production_gpu.py -x -q -s --timeout 200 --timeout-method thread > gpurun_out/pytest_attnprod_r3q.log 2>&1 || { tail -40 gpurun_out/pytest_attnprod_r3q.log; exit 1; }
grep -E "worst|passed|failed" gpurun_out/pytest_attnprod_r3q.log
ATTN_AB=8,4 timeout -k 10 300 python -u tests/probes/attn_bench.py 2>&1 | tee gpurun_out/attn_ab_r3q.log
PMC_TAG=attn_w4q bash scripts/pmc.sh attn && python3 scripts/pmc_summary.py attn_w4q attn_fwd_w4 > gpurun_out/pmc_attn_w4q/summary.txt 2>&1; cat gpurun_out/pmc_attn_w4q/summary.txt
