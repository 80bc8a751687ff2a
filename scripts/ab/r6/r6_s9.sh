#!/bin/bash
# r6 step 9: the CFG shared prefix (first DiT / VACE block's phases 1-3 once for both samples):
# the whole -m gpu suite, then the 14B bench with the option on / off, interleaved
set -o pipefail
mkdir -p gpurun_out
bash scripts/ab/r6/r6_tests.sh r6c || exit 1
for i in 1 2; do
for pf in 1 0; do
VSTYLER_OPTS=cfg_prefix=$pf timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-e2e --steps 5 --warmup 2 > gpurun_out/r6_bench_pf${pf}_$i.json 2> gpurun_out/r6_bench_pf${pf}_$i.err || { tail -20 gpurun_out/r6_bench_pf${pf}_$i.err; exit 1; }
echo "cfg_prefix=$pf round $i: $(cut -c1-200 gpurun_out/r6_bench_pf${pf}_$i.json)"
done
done
