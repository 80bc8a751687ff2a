#!/bin/bash
# r5 GPU session 3: the product build without the vendor-library route -- full -m gpu suite, smoke,
# the 1.3B-shape GEMM A/B against the A/B build's library route, the 14B and 1.3B benches and a
# rocprofv3 kernel-stats run of the 14B step.  A crash, fault or time limit ends the session.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
fault() { grep -qiE "memory access fault|illegal address|HSA_STATUS_ERROR|hipErrorLaunchFailure|core dumped" "$1"; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rfE --timeout 300 --timeout-method thread > gpurun_out/r5_pytest_gpu_s3.log 2>&1
rc=$?; grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r5_pytest_gpu_s3.log | tail -12
if [ $rc -gt 1 ] || fault gpurun_out/r5_pytest_gpu_s3.log; then tail -30 gpurun_out/r5_pytest_gpu_s3.log; exit 1; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5_smoke_s3.log 2>&1 || { tail -20 gpurun_out/r5_smoke_s3.log; exit 1; }
tail -1 gpurun_out/r5_smoke_s3.log
AB_MODEL=1.3B AB_VARIANTS=auto,t128,w4,lt VSTYLER_LIB=$R/video-styler_amd/vstyler/lib/ab/libvstyler.so \
  timeout -k 10 300 python -u tests/probes/gemm_ab.py 59280 > gpurun_out/r5_gemm_ab_1p3b.log 2>&1 || { tail -20 gpurun_out/r5_gemm_ab_1p3b.log; exit 1; }
grep -v Warning gpurun_out/r5_gemm_ab_1p3b.log
timeout -k 10 400 python -u bench.py > gpurun_out/r5_bench_s3.json 2> gpurun_out/r5_bench_s3.err || { tail -20 gpurun_out/r5_bench_s3.err; exit 1; }
cat gpurun_out/r5_bench_s3.json
timeout -k 10 300 python -u bench.py --model 1.3B --steps 5 --no-cpu-baseline --no-e2e > gpurun_out/r5_bench_1p3b_s3.json 2> gpurun_out/r5_bench_1p3b_s3.err || { tail -20 gpurun_out/r5_bench_1p3b_s3.err; exit 1; }
cat gpurun_out/r5_bench_1p3b_s3.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r5s3 -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > $R/gpurun_out/prof_r5s3.log 2>&1 || { tail -20 $R/gpurun_out/prof_r5s3.log; exit 1; }
find $R/gpurun_out/prof_r5s3 -name "*stats*"
