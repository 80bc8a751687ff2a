set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k attention --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1; rc=$?; tail -3 gpurun_out/attn_tests.log; [ $rc -eq 0 ] || exit 1
for i in 1 2; do
 echo "== v1"; VS_ATTN_IMPL=1 timeout -k 10 300 python tests/probes/attn_bench.py || exit 1
 echo "== v2"; VS_ATTN_IMPL=2 timeout -k 10 300 python tests/probes/attn_bench.py || exit 1
done
