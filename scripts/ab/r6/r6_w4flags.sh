#!/bin/bash
# attn_fwd_w4 code-generation flags A/B: the product library vs attention_w4.o rebuilt with each
# scheduler / MFMA-form flag (abl/w4_*/libvstyler.so), tests/probes/attn_bench.py per variant,
# three interleaved rounds
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/w4flags_ab.log
: > $out
for r in 1 2 3; do
  for v in base maxilp memclause vgprform; do
    echo "round $r $v" >> $out
    VSTYLER_LIB=$PWD/abl/w4_$v/libvstyler.so timeout -k 10 120 python -u tests/probes/attn_bench.py >> $out 2>&1 || { echo "FAILED $v"; tail -20 $out; exit 1; }
  done
done
grep -v amdgpu.ids $out
