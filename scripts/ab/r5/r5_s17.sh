#!/bin/bash
# r5 GPU session 17: config 5 (fp8, UniPC, SLG; eager launches) under rocprofv3 kernel trace -- is the
# GPU busy for the whole timed span?
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_fp8_r5s17 -o run --output-format csv -- python3 $R/bench.py --config fp8 --steps 4 --warmup 1 --no-cpu-baseline --no-e2e > $R/gpurun_out/prof_fp8_r5s17.log 2>&1 || { tail -20 $R/gpurun_out/prof_fp8_r5s17.log; exit 1; }
grep '"metric"' $R/gpurun_out/prof_fp8_r5s17.log | cut -c1-250
