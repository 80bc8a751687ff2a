#!/bin/bash
# GPU-box session: tests -> bench -> rocprofv3 kernel stats.  Each GPU step has its own time limit;
# a crash or time limit ends the session (no retries).  Usage: bash scripts/gpu_round.sh <tag> [pytest -k expr]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r3}
mkdir -p $R/gpurun_out
cd $R
K=${2:+-k "$2"}
# a test failure is reported and the bench still runs; a timeout / crash of the runner ends the session
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread $K \
  > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
if [ $rc -ne 0 ]; then grep -E "^FAILED|^ERROR" gpurun_out/pytest_gpu_$TAG.log | head -20; fi
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; fi
# a GPU fault in any test ends the session too (nothing more runs on the GPU after one)
if grep -qiE "memory access fault|illegal address|HSA_STATUS_ERROR|hipErrorLaunchFailure|core dumped" gpurun_out/pytest_gpu_$TAG.log; then
  echo "GPU fault reported by the tests: stopping"; exit 1; fi
grep -E "passed|failed" gpurun_out/pytest_gpu_$TAG.log | tail -2
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > $R/gpurun_out/prof_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/prof_$TAG.log; exit 1; }
find $R/gpurun_out/prof_$TAG -name "*stats*"
