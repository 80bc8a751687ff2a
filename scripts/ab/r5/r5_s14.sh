#!/bin/bash
# r5 GPU session 14: attn_fwd_w4 with the last 1 / 2 softmax steps of phase C moved into the tail
# of phase D (A/B builds lib/diag_cm1, diag_cm2) against the product build, interleaved rounds.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in base cm1 cm2; do
    if [ $v = base ]; then unset VSTYLER_LIB; else export VSTYLER_LIB=$R/video-styler_amd/vstyler/lib/diag_$v/libvstyler.so; fi
    echo "== $v" >> gpurun_out/r5_cmove_ab_s14.log
    timeout -k 10 120 python -u tests/probes/attn_bench.py >> gpurun_out/r5_cmove_ab_s14.log 2>&1 || { tail -20 gpurun_out/r5_cmove_ab_s14.log; exit 1; }
  done
done
unset VSTYLER_LIB
grep -v Warning gpurun_out/r5_cmove_ab_s14.log | grep -v amdgpu.ids
