#!/bin/bash
# scratch: GPU tests with the hoisted-offset GEMM + SP=1 own routing, then same-box bench A/B
# (VS_GEMM_OWN_SP1=1 default vs 0 = the r3s10 routing), then rocprof of the default bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r3s11.log 2>&1 || { grep -E "^FAILED|^ERROR|Error" gpurun_out/pytest_gpu_r3s11.log | head; tail -20 gpurun_out/pytest_gpu_r3s11.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r3s11.log
for i in 1 2; do
  for v in 1 0; do
    echo "== VS_GEMM_OWN_SP1=$v" | tee -a gpurun_out/bench_own_sp1_ab.log
    VS_GEMM_OWN_SP1=$v timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e 2>/dev/null | tee -a gpurun_out/bench_own_sp1_ab.log || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r3s11 -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > $R/gpurun_out/prof_r3s11.log 2>&1 || { tail -20 $R/gpurun_out/prof_r3s11.log; exit 1; }
echo prof done
