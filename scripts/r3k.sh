set -o pipefail
cd $GRAFT_REPO_ROOT
P=tests/probes/c3_variants.py
L=gpurun_out/c3_tune_r3k.log
: > $L
for i in 1 2 3; do
  VS_LT_DEBUG=1 timeout -k 10 200 python -u $P 2>&1 | grep -E "B2 vs oracle|pick" >> $L || { echo "run $i failed" >> $L; break; }
done
for i in 1 2; do
  VS_LT_TUNE=0 timeout -k 10 200 python -u $P 2>&1 | grep -E "B2 vs oracle" >> $L || { echo "tune0 run $i failed" >> $L; break; }
done
cat $L
