#!/bin/bash
# r6: the other configurations on the final tree -- config 5 (fp8, 4-step UniPC), the 1.3B model, C4's
# 1280x720x121 on one GPU
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r6}
timeout -k 10 500 python -u bench.py --config fp8 --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/bench_fp8_${TAG}.json 2> gpurun_out/bench_fp8_${TAG}.err || { tail -20 gpurun_out/bench_fp8_${TAG}.err; exit 1; }
cut -c1-220 gpurun_out/bench_fp8_${TAG}.json
timeout -k 10 400 python -u bench.py --model 1.3B --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/bench_1p3b_${TAG}.json 2> gpurun_out/bench_1p3b_${TAG}.err || { tail -20 gpurun_out/bench_1p3b_${TAG}.err; exit 1; }
cut -c1-220 gpurun_out/bench_1p3b_${TAG}.json
timeout -k 10 500 python -u bench.py --frames 121 --height 720 --width 1280 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/bench_c4_${TAG}.json 2> gpurun_out/bench_c4_${TAG}.err || { tail -20 gpurun_out/bench_c4_${TAG}.err; exit 1; }
cut -c1-220 gpurun_out/bench_c4_${TAG}.json
