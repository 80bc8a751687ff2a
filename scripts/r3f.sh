set -o pipefail
cd $GRAFT_REPO_ROOT
P=tests/probes/c3_variants.py
L=gpurun_out/c3_variants_r3f.log
: > $L
for V in "" "VS_GEMM_BACKEND=vstyler" "VSTYLER_FUSE_RES_LN=0 VSTYLER_FUSE_FFN_LN=0" "VS_ATTN_NC=0" "VS_ATTN_NO_SPLIT=1" "VS_ATTN_NO_PERSIST=1" "C3_VACE=0"; do
  env $V timeout -k 10 200 python -u $P 2>&1 | grep -v "amdgpu.ids\|Latency" >> $L || { echo "variant $V failed rc=$?" >> $L; break; }
done
cat $L
