#!/bin/bash
# r5 GPU session 19: config-5 LayerNorms straight into fp8_linear's quantised input -- fp8 tests (quant
# widths, LN-fp8 == two passes, model bit-identity, C5), the 14B forward A/B, the config-5 bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fp8_gpu.py tests/test_production_c4c5_gpu.py tests/test_kernels_gpu.py -k "fp8 or c5 or quant or layernorm" -q -rfE --timeout 300 --timeout-method thread > gpurun_out/r5_fp8_tests_s19.log 2>&1
rc=$?; grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r5_fp8_tests_s19.log | tail -6
if [ $rc -ne 0 ]; then tail -30 gpurun_out/r5_fp8_tests_s19.log; exit 1; fi
timeout -k 10 400 python -u tests/probes/fp8_ln_fusion_ab.py > gpurun_out/r5_fp8_ln_ab_s19.log 2>&1 || { tail -20 gpurun_out/r5_fp8_ln_ab_s19.log; exit 1; }
grep -v "Warning\|amdgpu.ids" gpurun_out/r5_fp8_ln_ab_s19.log
timeout -k 10 500 python -u bench.py --config fp8 --steps 4 --no-cpu-baseline --no-e2e > gpurun_out/r5_bench_fp8_s19.json 2> gpurun_out/r5_bench_fp8_s19.err || { tail -20 gpurun_out/r5_bench_fp8_s19.err; exit 1; }
cut -c1-200 gpurun_out/r5_bench_fp8_s19.json
