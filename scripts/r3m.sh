set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r3m.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_r3m.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_r3m.log
grep -E "noise floor|worst" gpurun_out/pytest_gpu_r3m.log | head -20
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --no-e2e --no-cpu-baseline > gpurun_out/bench_r3m.json 2> gpurun_out/bench_r3m.err || { tail -20 gpurun_out/bench_r3m.err; exit 1; }
cat gpurun_out/bench_r3m.json
