#!/bin/bash
# max-ILP scheduling for every source (build/var_ilpall) vs the default (attention only): the row
# kernels (rownorm_ab.py, bit-identity checked) and the VAE (vae_bench.py), interleaved.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for i in 1 2; do
  echo "== base"; timeout -k 10 300 python tests/probes/rownorm_ab.py base$i || exit 1
  echo "== ilpall"; VSTYLER_LIB=$R/build/var_ilpall/libvstyler.so timeout -k 10 300 python tests/probes/rownorm_ab.py ilp$i base$i || exit 1
done
for i in 1 2; do
  echo "== base"; timeout -k 10 300 python tests/probes/vae_bench.py || exit 1
  echo "== ilpall"; VSTYLER_LIB=$R/build/var_ilpall/libvstyler.so timeout -k 10 300 python tests/probes/vae_bench.py || exit 1
done
