#!/bin/bash
# Same-box A/B of the hipBLASLt build on the 14B bench (VS_LT_LIB=linked vs default), interleaved.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for i in 1 2; do
  for lib in linked default; do
    if [ $lib = linked ]; then export VS_LT_LIB=linked; else unset VS_LT_LIB; fi
    echo "== $lib"
    timeout -k 10 400 python bench.py --no-cpu-baseline --no-e2e 2> /dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('14B', d['value'], 'steps/s', d['ms_per_step'], 'ms, attention', d['roofline']['achieved'])" || exit 1
  done
done
