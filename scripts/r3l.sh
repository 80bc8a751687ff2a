set -o pipefail
cd $GRAFT_REPO_ROOT
L=gpurun_out/gemm_diag_r3l.log
: > $L
for D in "" NODMA NOMFMA NOBAR; do
  if [ -n "$D" ]; then export VSTYLER_LIB=$GRAFT_REPO_ROOT/video-styler_amd/vstyler/lib/diag/libvstyler_$D.so; else unset VSTYLER_LIB; fi
  echo "== ${D:-default}" >> $L
  AB_VARIANTS=1b timeout -k 10 200 python -u tests/probes/gemm8p_ab.py 59280 2>&1 | grep -v amdgpu.ids >> $L || { echo "diag $D failed" >> $L; break; }
done
cat $L
