#!/bin/bash
# A/B an attention build flag on the GPU box: default lib vs one built with EXTRA flags ($1).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
make -C video-styler_amd/csrc -j16 OUT_DIR=$R/build/alt OBJ_DIR=$R/build/alt_obj EXTRA="$1" > /dev/null || exit 1
for i in 1 2; do
  echo "== A (default)"; timeout -k 10 300 python tests/probes/attn_bench.py || exit 1
  echo "== B ($1)"; VSTYLER_LIB=$R/build/alt/libvstyler.so timeout -k 10 300 python tests/probes/attn_bench.py || exit 1
done
