#!/bin/bash
# On the GPU box: run tests/probes/$PROBE (args $@) for the default lib and every
# tests/probes/var/*/libvstyler.so, interleaved, two rounds; stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
PROBE=${PROBE:-cross_ab.py}
for i in 1 2; do
  timeout -k 10 300 python tests/probes/$PROBE "$@" 2>&1 | grep -v amdgpu.ids || exit 1
  for d in tests/probes/var/*/; do
    [ -f $d/libvstyler.so ] || continue
    VSTYLER_LIB=$R/$d/libvstyler.so timeout -k 10 300 python tests/probes/$PROBE "$@" 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
