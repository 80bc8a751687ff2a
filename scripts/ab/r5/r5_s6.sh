#!/bin/bash
# r5 GPU session 6: config 5 (fp8, all GEMMs on the hand-written fp8 kernel), the C4 shape on one GPU,
# and a rocprofv3 kernel-stats run of the default 14B bench.  A crash, fault or time limit ends it.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --config fp8 --steps 4 --no-cpu-baseline > gpurun_out/r5_bench_fp8_s6.json 2> gpurun_out/r5_bench_fp8_s6.err || { tail -20 gpurun_out/r5_bench_fp8_s6.err; exit 1; }
cat gpurun_out/r5_bench_fp8_s6.json
timeout -k 10 400 python -u bench.py --frames 121 --height 720 --width 1280 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/r5_bench_c4_s6.json 2> gpurun_out/r5_bench_c4_s6.err || { tail -20 gpurun_out/r5_bench_c4_s6.err; exit 1; }
cat gpurun_out/r5_bench_c4_s6.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r5s6 -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $R/gpurun_out/prof_r5s6.log 2>&1 || { tail -20 $R/gpurun_out/prof_r5s6.log; exit 1; }
grep '"metric"' $R/gpurun_out/prof_r5s6.log
