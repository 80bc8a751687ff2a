#!/bin/bash
# GPU tests, the 14B bench, and the C2 / SP A/B of the hipBLASLt build, on one box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TAG=${1:-r2n}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 900 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cut -c1-300 gpurun_out/bench_$TAG.json
bash scripts/ab_lt_lib_workloads.sh > gpurun_out/lt_lib_workloads_ab_$TAG.log 2>&1 || { tail -20 gpurun_out/lt_lib_workloads_ab_$TAG.log; exit 1; }
cat gpurun_out/lt_lib_workloads_ab_$TAG.log
