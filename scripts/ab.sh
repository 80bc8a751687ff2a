#!/bin/bash
# A/B/C build flags on the GPU box: ./scripts/ab.sh <probe.py> "<flags B>" ["<flags C>" ...]
# Builds one library per flag set, then runs the probe against each, twice, interleaved.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
probe=$1; shift
i=0
for f in "$@"; do
  make -C video-styler_amd/csrc -j16 OUT_DIR=$R/build/alt$i OBJ_DIR=$R/build/alt_obj$i EXTRA="$f" > /dev/null || exit 1
  i=$((i+1))
done
for rep in 1 2; do
  echo "== A (default)"; timeout -k 10 300 python $probe || exit 1
  i=0
  for f in "$@"; do
    echo "== variant $i ($f)"; VSTYLER_LIB=$R/build/alt$i/libvstyler.so timeout -k 10 300 python $probe || exit 1
    i=$((i+1))
  done
done
