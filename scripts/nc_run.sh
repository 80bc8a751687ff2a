set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -k attention --timeout 120 --timeout-method thread > gpurun_out/pytest_nc.log 2>&1 || { tail -40 gpurun_out/pytest_nc.log; exit 1; }
tail -3 gpurun_out/pytest_nc.log
for i in 1 2; do
  echo "== NC=0"; VS_ATTN_NC=0 timeout -k 10 300 python tests/probes/attn_bench.py || exit 1
  echo "== NC (default)"; timeout -k 10 300 python tests/probes/attn_bench.py || exit 1
done
