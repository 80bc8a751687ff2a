#!/bin/bash
# r6 measurement session: the bench line (cpu baseline + measured e2e pipe() call), a rocprofv3
# kernel-trace --stats run of the bench, PMC passes of the self- and cross-attention
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TAG=${1:-r6b}
mkdir -p gpurun_out
timeout -k 10 700 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cut -c1-400 gpurun_out/bench_$TAG.json
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > $R/gpurun_out/prof_$TAG.log 2>&1) || { tail -20 gpurun_out/prof_$TAG.log; exit 1; }
grep '"value"' gpurun_out/prof_$TAG.log | cut -c1-200
PMC_TAG=attn_w4_$TAG timeout -k 10 900 bash scripts/pmc.sh attn > gpurun_out/pmc_attn_$TAG.log 2>&1 || { tail -20 gpurun_out/pmc_attn_$TAG.log; exit 1; }
python3 scripts/pmc_summary.py attn_w4_$TAG attn_fwd_w4 > gpurun_out/pmc_attn_w4_$TAG/summary.txt; cat gpurun_out/pmc_attn_w4_$TAG/summary.txt
PMC_TAG=cross_$TAG timeout -k 10 900 bash scripts/pmc.sh cross > gpurun_out/pmc_cross_$TAG.log 2>&1 || { tail -20 gpurun_out/pmc_cross_$TAG.log; exit 1; }
python3 scripts/pmc_summary.py cross_$TAG attn_fwd_w4 > gpurun_out/pmc_cross_$TAG/summary.txt; cat gpurun_out/pmc_cross_$TAG/summary.txt
