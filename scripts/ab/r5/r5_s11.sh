#!/bin/bash
# r5 GPU session 11: cross-attention on attn_fwd_w4 (items of >= 4 key tiles), attention queues bound
# by the attention wrapper -- full -m gpu suite, attention microbenchmark, 14B bench + kernel stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
fault() { grep -qiE "memory access fault|illegal address|HSA_STATUS_ERROR|hipErrorLaunchFailure|core dumped" "$1"; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rfE --timeout 300 --timeout-method thread > gpurun_out/r5_pytest_gpu_s11.log 2>&1
rc=$?; grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r5_pytest_gpu_s11.log | tail -12
if [ $rc -gt 1 ] || fault gpurun_out/r5_pytest_gpu_s11.log; then tail -30 gpurun_out/r5_pytest_gpu_s11.log; exit 1; fi
timeout -k 10 300 python -u tests/probes/attn_bench.py > gpurun_out/r5_attn_bench_s11.log 2>&1 || { tail -20 gpurun_out/r5_attn_bench_s11.log; exit 1; }
grep -v Warning gpurun_out/r5_attn_bench_s11.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r5s11 -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $R/gpurun_out/prof_r5s11.log 2>&1 || { tail -20 $R/gpurun_out/prof_r5s11.log; exit 1; }
grep '"metric"' $R/gpurun_out/prof_r5s11.log | cut -c1-200
