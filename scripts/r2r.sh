#!/bin/bash
# GPU tests, the SP=4/8 per-rank compute probe and the bench (no CPU baseline), one box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TAG=${1:-r2r}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 300 python tests/probes/sp_rank_compute.py 4 8 > gpurun_out/sp_rank_$TAG.log 2>&1 || { tail -20 gpurun_out/sp_rank_$TAG.log; exit 1; }
grep -v amdgpu.ids gpurun_out/sp_rank_$TAG.log
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); print(d['value'], d['ms_per_step'], d['roofline']['achieved'], d['e2e']['sec_per_video'])"
