#!/bin/bash
# the 14B step with gemm.o built with max-ilp vs the product library, interleaved bench runs
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/gemmflags_step_ab.log
: > $out
for r in 1 2; do
  for v in base maxilp; do
    VSTYLER_LIB=$PWD/abl/g_$v/libvstyler.so timeout -k 10 400 python -u bench.py --steps 5 --no-e2e --no-cpu-baseline > gpurun_out/gf_$v$r.json 2> gpurun_out/gf_$v$r.err || { echo "FAILED $v"; tail -20 gpurun_out/gf_$v$r.err; exit 1; }
    echo "round $r $v $(cut -c1-200 gpurun_out/gf_$v$r.json)" >> $out
  done
done
cat $out
