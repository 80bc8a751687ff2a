set -o pipefail
cd $GRAFT_REPO_ROOT
for v in w4ne w4nd w4st; do
echo "== stamps $v"
VSTYLER_LIB=$PWD/build/diag/$v/libvstyler.so timeout -k 10 300 python -u tests/probes/w4_stamps.py 2>&1 | tee -a gpurun_out/w4_stamps_r3u.log
VSTYLER_LIB=$PWD/build/diag/$v/libvstyler.so ATTN_AB=4 timeout -k 10 300 python -u tests/probes/attn_bench.py 2>&1 | grep self | tee -a gpurun_out/w4_stamps_r3u.log
done
