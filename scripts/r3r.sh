set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_attention_production_gpu.py -x -q -s --timeout 200 --timeout-method thread > gpurun_out/pytest_attnprod_r3r.log 2>&1 || { tail -40 gpurun_out/pytest_attnprod_r3r.log; exit 1; }
grep -E "worst|passed|failed" gpurun_out/pytest_attnprod_r3r.log
for i in 1 2; do
ATTN_AB=8,4 timeout -k 10 300 python -u tests/probes/attn_bench.py 2>&1 | tee -a gpurun_out/attn_ab_r3r.log
echo "== r3q lib"
VSTYLER_LIB=$PWD/build/diag/w4q/libvstyler.so ATTN_AB=4 timeout -k 10 300 python -u tests/probes/attn_bench.py 2>&1 | tee -a gpurun_out/attn_ab_r3r.log
done
echo "== stamps"
VSTYLER_LIB=$PWD/build/diag/w4st/libvstyler.so timeout -k 10 300 python -u tests/probes/w4_stamps.py 2>&1 | tee gpurun_out/w4_stamps_r3r.log
