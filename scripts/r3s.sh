set -o pipefail
cd $GRAFT_REPO_ROOT
echo "== stamps (product build)"
VSTYLER_LIB=$PWD/build/diag/w4st/libvstyler.so timeout -k 10 300 python -u tests/probes/w4_stamps.py 2>&1 | tee gpurun_out/w4_stamps_r3s.log
echo "== stamps NODMA"
VSTYLER_LIB=$PWD/build/diag/w4nd/libvstyler.so timeout -k 10 300 python -u tests/probes/w4_stamps.py 2>&1 | tee -a gpurun_out/w4_stamps_r3s.log
echo "== time NODMA"
VSTYLER_LIB=$PWD/build/diag/w4nd/libvstyler.so ATTN_AB=4 timeout -k 10 300 python -u tests/probes/attn_bench.py 2>&1 | tee -a gpurun_out/w4_stamps_r3s.log
