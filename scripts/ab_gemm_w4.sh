set -o pipefail
cd $GRAFT_REPO_ROOT
VS_GEMM_IMPL=4 VSTYLER_GEMM_TILE=256 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp8_gpu.py -x -q -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/gemm_w4_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gemm_w4_tests.log; [ $rc -eq 0 ] || exit 1
echo "== impl 8 (default)"; timeout -k 10 300 python tests/probes/gemm_bench.py || exit 1
echo "== impl 4"; VS_GEMM_IMPL=4 timeout -k 10 300 python tests/probes/gemm_bench.py || exit 1
