#!/bin/bash
# The private ROCm-7.2 hipBLASLt on the other workloads: C2 (1.3B), config 5 (fp8), the SP=8/4 per-rank
# compute probe.  Each step has its own time limit; the first failure ends the run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TAG=${1:-r2m}
timeout -k 10 600 python bench.py --model 1.3B --no-cpu-baseline --no-e2e > gpurun_out/bench_c2_$TAG.json 2> gpurun_out/bench_c2_$TAG.err || { tail -20 gpurun_out/bench_c2_$TAG.err; exit 1; }
cat gpurun_out/bench_c2_$TAG.json | cut -c1-400
timeout -k 10 600 python bench.py --config fp8 --no-cpu-baseline --no-e2e > gpurun_out/bench_fp8_$TAG.json 2> gpurun_out/bench_fp8_$TAG.err || { tail -20 gpurun_out/bench_fp8_$TAG.err; exit 1; }
cat gpurun_out/bench_fp8_$TAG.json | cut -c1-400
timeout -k 10 600 python tests/probes/sp_rank_compute.py 8 4 > gpurun_out/sp_rank_$TAG.log 2>&1 || { tail -20 gpurun_out/sp_rank_$TAG.log; exit 1; }
grep -v amdgpu.ids gpurun_out/sp_rank_$TAG.log
