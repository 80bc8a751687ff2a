#!/bin/bash
# gemm.o code-generation flags A/B: the product library vs gemm.o rebuilt with a scheduler strategy
# (abl/g_*/libvstyler.so; each passes scripts/check_isa.py), tests/probes/gemm_ab.py (4-wave kernel,
# XCD queues) at 59 280 rows per variant, three interleaved rounds
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/gemmflags_ab.log
: > $out
for r in 1 2 3; do
  for v in base maxilp memclause; do
    echo "round $r $v" >> $out
    AB_VARIANTS=w4 VSTYLER_LIB=$PWD/abl/g_$v/libvstyler.so timeout -k 10 150 python -u tests/probes/gemm_ab.py 59280 >> $out 2>&1 || { echo "FAILED $v"; tail -20 $out; exit 1; }
  done
done
grep -v amdgpu.ids $out
