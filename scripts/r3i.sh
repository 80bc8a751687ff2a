set -o pipefail
cd $GRAFT_REPO_ROOT
P=tests/probes/c3_poison.py
L=gpurun_out/c3_poison_r3i.log
: > $L
for V in "VSTYLER_WS_POISON=0" "VSTYLER_WS_POISON=1" "VSTYLER_WS_POISON=0 C3_ORDER=product" "VSTYLER_WS_POISON=1 VS_ATTN_NC=0"; do
  env $V timeout -k 10 200 python -u $P 2>&1 | grep -v "amdgpu.ids\|Latency" >> $L || { echo "variant $V failed" >> $L; break; }
done
cat $L
