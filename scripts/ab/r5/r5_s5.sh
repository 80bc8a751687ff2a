#!/bin/bash
# r5 GPU session 5: -m gpu suite with the attention item queues and the queue-fed first tiles, the
# held-CU probe again, and two interleaved 14B bench pairs (queues vs static lists, VSTYLER_OPTS).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
fault() { grep -qiE "memory access fault|illegal address|HSA_STATUS_ERROR|hipErrorLaunchFailure|core dumped" "$1"; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rfE --timeout 300 --timeout-method thread > gpurun_out/r5_pytest_gpu_s5.log 2>&1
rc=$?; grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r5_pytest_gpu_s5.log | tail -12
if [ $rc -ne 0 ] || fault gpurun_out/r5_pytest_gpu_s5.log; then tail -30 gpurun_out/r5_pytest_gpu_s5.log; exit 1; fi
timeout -k 10 400 python -u tests/probes/cu_hold.py > gpurun_out/r5_cu_hold_s5.log 2>&1 || { tail -20 gpurun_out/r5_cu_hold_s5.log; exit 1; }
grep -v Warning gpurun_out/r5_cu_hold_s5.log
LOG=gpurun_out/r5_bench_queue_ab_s5.log
run() {
  echo "== $1" >> $LOG
  env $2 timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e >> $LOG 2>/dev/null || { echo "bench $1 failed"; exit 1; }
}
for r in 1 2; do
  run queue "VSTYLER_OPTS=queue=1"
  run static "VSTYLER_OPTS=queue=0"
done
grep -E "^==|value" $LOG | sed 's/"config.*//'
