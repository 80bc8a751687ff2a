#!/bin/bash
# the whole -m gpu suite + smoke (round-end tier), one process each, own time limits
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r6}
timeout -k 10 1050 python -u -m pytest tests -m gpu -q -rfE --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
grep -E "^FAILED|^ERROR" gpurun_out/pytest_gpu_$TAG.log | head -20
grep -E "passed|failed" gpurun_out/pytest_gpu_$TAG.log | tail -2
if [ $rc -ne 0 ]; then tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
grep smoke gpurun_out/smoke_$TAG.log
