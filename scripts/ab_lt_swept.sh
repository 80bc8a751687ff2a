#!/bin/bash
# hipBLASLt route A/B: the link-time library (torch's bundled build, VS_LT_LIB=linked) vs the default
# (the private ROCm-7.2 copy + swept candidates) on the 14B block GEMMs at 59280 and 3705 rows, after
# a debug pass and the GPU tests, then the bench.  Each GPU step has its own time limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TAG=${1:-lt}
VS_LT_DEBUG=1 timeout -k 10 300 python tests/probes/lt_debug.py > gpurun_out/lt_debug_$TAG.log 2>&1 || { tail -30 gpurun_out/lt_debug_$TAG.log; exit 1; }
grep -E "pick|dlopen|dlsym|kernel library|resolved" gpurun_out/lt_debug_$TAG.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_$TAG.log
for i in 1 2; do
  echo "== VS_LT_LIB=linked"; VS_LT_LIB=linked timeout -k 10 300 python tests/probes/gemm_backend_ab.py 59280 3705 || exit 1
  echo "== default"; timeout -k 10 300 python tests/probes/gemm_backend_ab.py 59280 3705 || exit 1
done > gpurun_out/lt_lib_ab_$TAG.log 2>&1
grep -v amdgpu.ids gpurun_out/lt_lib_ab_$TAG.log
timeout -k 10 900 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
