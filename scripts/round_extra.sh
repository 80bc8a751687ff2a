#!/bin/bash
# The other BASELINE configurations on one GPU (after scripts/gpu_round.sh): config 5 (fp8, 4-step
# UniPC), C2 (1.3B) and the C4 shape (1280x720x121).  Each under its own limit; a failure ends it.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
TAG=${1:-r3}
timeout -k 10 400 python -u bench.py --config fp8 --steps 4 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/bench_fp8_$TAG.json 2> gpurun_out/bench_fp8_$TAG.err || { tail -5 gpurun_out/bench_fp8_$TAG.err; exit 1; }
cat gpurun_out/bench_fp8_$TAG.json
timeout -k 10 300 python -u bench.py --model 1.3B --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/bench_1p3b_$TAG.json 2> gpurun_out/bench_1p3b_$TAG.err || { tail -5 gpurun_out/bench_1p3b_$TAG.err; exit 1; }
cat gpurun_out/bench_1p3b_$TAG.json
timeout -k 10 500 python -u bench.py --frames 121 --height 720 --width 1280 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --progress > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.err || { tail -5 gpurun_out/bench_c4_$TAG.err; exit 1; }
cat gpurun_out/bench_c4_$TAG.json
