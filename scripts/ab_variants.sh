#!/bin/bash
# On the GPU box: time tests/probes/${PROBE:-attn_bench.py} for the default lib and each build/var_*/ lib, twice.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
PROBE=${PROBE:-attn_bench.py}
for i in $(seq 1 ${REPS:-2}); do
  echo "== base"; timeout -k 10 300 python tests/probes/$PROBE || exit 1
  for d in build/var_*/; do
    [ -f $d/libvstyler.so ] || continue
    echo "== $(basename $d)"; VSTYLER_LIB=$R/$d/libvstyler.so timeout -k 10 300 python tests/probes/$PROBE || exit 1
  done
done
