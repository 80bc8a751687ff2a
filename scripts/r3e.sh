set -o pipefail
cd $GRAFT_REPO_ROOT
P=tests/probes/c3_variants.py
L=gpurun_out/c3_variants_r3e.log
timeout -k 10 200 python -u $P > $L 2>&1
VS_GEMM_BACKEND=vstyler timeout -k 10 200 python -u $P >> $L 2>&1
VS_LT_SWEPT=0 timeout -k 10 200 python -u $P >> $L 2>&1
VS_LT_TUNE=0 timeout -k 10 200 python -u $P >> $L 2>&1
VS_LT_GELU=0 VSTYLER_FUSE_FFN_LN=0 timeout -k 10 200 python -u $P >> $L 2>&1
grep -v amdgpu.ids $L
timeout -k 10 300 python -u -m pytest tests/test_gemm8p_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gemm8p_r3e.log 2>&1 || { tail -40 gpurun_out/pytest_gemm8p_r3e.log; exit 1; }
tail -3 gpurun_out/pytest_gemm8p_r3e.log
timeout -k 10 300 python -u tests/probes/gemm8p_ab.py 59280 7410 > gpurun_out/gemm8p_ab_r3e.log 2>&1; grep -v amdgpu.ids gpurun_out/gemm8p_ab_r3e.log
timeout -k 10 300 python -u tests/probes/gemm_fp8_8p_ab.py 59280 > gpurun_out/gemm_fp8_ab_r3e.log 2>&1; grep -v amdgpu.ids gpurun_out/gemm_fp8_ab_r3e.log
