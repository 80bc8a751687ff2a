#!/bin/bash
# scratch: interleaved same-box A/B of attention builds: scripts/ab/ab_attn.sh <tag> <diag name>...
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
TAG=$1; shift
for i in 1 2 3; do
  for v in base "$@"; do
    if [ $v = base ]; then L=$PWD/video-styler_amd/vstyler/lib/libvstyler.so; else L=$PWD/video-styler_amd/vstyler/lib/diag_$v/libvstyler.so; fi
    echo "== $v" | tee -a gpurun_out/attn_ab_$TAG.log
    VSTYLER_LIB=$L ATTN_AB=4 timeout -k 10 200 python -u tests/probes/attn_bench.py 2>&1 | grep self | tee -a gpurun_out/attn_ab_$TAG.log || exit 1
  done
done
