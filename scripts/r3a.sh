set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r3a.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r3a.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_r3a.log
timeout -k 10 300 python -u tests/probes/gemm_backend_ab.py 59280 > gpurun_out/gemm_ab_r3a.log 2>&1; cat gpurun_out/gemm_ab_r3a.log
