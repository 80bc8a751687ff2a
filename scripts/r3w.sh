set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r3w.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_r3w.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_gpu_r3w.log | tail -2
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_r3w.json 2> gpurun_out/bench_r3w.err || { tail -20 gpurun_out/bench_r3w.err; exit 1; }
cat gpurun_out/bench_r3w.json
