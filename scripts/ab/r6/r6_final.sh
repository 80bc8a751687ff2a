#!/bin/bash
# r6 final session: whole -m gpu suite + smoke, the bench line, a rocprofv3 kernel-trace --stats run
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TAG=${1:-r6f}
mkdir -p gpurun_out
bash scripts/ab/r6/r6_tests.sh $TAG || exit 1
timeout -k 10 700 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cut -c1-300 gpurun_out/bench_$TAG.json
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > $R/gpurun_out/prof_$TAG.log 2>&1) || { tail -20 gpurun_out/prof_$TAG.log; exit 1; }
grep '"value"' gpurun_out/prof_$TAG.log | cut -c1-200
