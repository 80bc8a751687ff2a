#!/bin/bash
# GPU-box session: tests -> bench -> rocprofv3 kernel stats.  Each GPU step has its own time limit;
# the first failure ends the session (no retries).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r1}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -m pytest tests -m gpu -q -rA > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_$TAG.log
grep -E "noise floor" gpurun_out/pytest_gpu_$TAG.log | head
timeout -k 10 900 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/prof_$TAG.log; exit 1; }
find $R/gpurun_out/prof_$TAG -name "*stats*" | head
