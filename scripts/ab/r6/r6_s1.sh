#!/bin/bash
# r6 step 1: new SP world-2/4/8 tests, T5 at XXL dims, launcher refusal on a 1-GPU box, bench + measured e2e
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 800 --timeout-method thread -m gpu \
  tests/test_sp.py tests/test_t5_gpu.py > gpurun_out/r6_s1_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -50 gpurun_out/r6_s1_pytest.log; exit 1; }
tail -5 gpurun_out/r6_s1_pytest.log
timeout -k 10 120 python bench.py --gpus 2 > gpurun_out/r6_s1_gpus2.log 2>&1; rc=$?
echo "bench --gpus 2 rc=$rc"; cat gpurun_out/r6_s1_gpus2.log | tail -3
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/r6_s1_bench.json 2> gpurun_out/r6_s1_bench.err || { echo "bench failed"; tail -30 gpurun_out/r6_s1_bench.err; exit 1; }
cat gpurun_out/r6_s1_bench.json
