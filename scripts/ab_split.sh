set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
for i in 1 2; do
  echo "== split"; timeout -k 10 300 python tests/probes/attn_bench.py || exit 1
  echo "== nosplit"; VS_ATTN_NO_SPLIT=1 timeout -k 10 300 python tests/probes/attn_bench.py || exit 1
  echo "== head"; VSTYLER_LIB=$R/build/var_head/libvstyler.so timeout -k 10 300 python tests/probes/attn_bench.py || exit 1
done
