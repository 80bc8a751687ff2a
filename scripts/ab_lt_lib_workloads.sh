#!/bin/bash
# Same-box A/B of the hipBLASLt build (VS_LT_LIB=linked: torch's bundled one; default: the private
# ROCm-7.2 copy) on C2 (1.3B bench) and the SP=8 / SP=4 per-rank compute probe.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for i in 1 2; do
  for lib in linked default; do
    if [ $lib = linked ]; then export VS_LT_LIB=linked; else unset VS_LT_LIB; fi
    echo "== $lib"
    timeout -k 10 300 python bench.py --model 1.3B --no-cpu-baseline --no-e2e 2> /dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('C2', d['value'], 'steps/s', d['ms_per_step'], 'ms, attention', d['roofline']['achieved'])" || exit 1
    timeout -k 10 300 python tests/probes/sp_rank_compute.py 8 4 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
