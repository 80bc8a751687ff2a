set -o pipefail
cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
echo "== default"
ATTN_AB=4 timeout -k 10 300 python -u tests/probes/attn_bench.py 2>&1 | grep self | tee -a gpurun_out/w4_c2_ab_r3v.log
echo "== C_SMP2"
VSTYLER_LIB=$PWD/build/diag/c2p/libvstyler.so ATTN_AB=4 timeout -k 10 300 python -u tests/probes/attn_bench.py 2>&1 | grep self | tee -a gpurun_out/w4_c2_ab_r3v.log
done
