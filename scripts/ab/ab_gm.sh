#!/bin/bash
# scratch: GEMM raster-group size (VS_GEMM_GM) A/B at the 14B SP=1 row count, then the SP graph
# capture probe under faulthandler (last: it may end in a segfault)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
L=video-styler_amd/vstyler/lib
for r in 1 2; do
  for v in default gm8 gm16 gm32; do
    if [ $v = default ]; then LIB=$L/libvstyler.so; else LIB=$L/diag_$v/libvstyler.so; fi
    echo "== GM $v round $r" | tee -a gpurun_out/gm_ab.log
    VSTYLER_LIB=$LIB timeout -k 10 120 python -u tests/probes/gemm_ab.py 59280 2>&1 | tee -a gpurun_out/gm_ab.log || exit 1
  done
done
PYTHONFAULTHANDLER=1 VSTYLER_SP_GRAPH=1 timeout -k 10 120 python -u -X faulthandler tests/probes/sp_graph_probe.py torch 3 > gpurun_out/sp_graph_fh.log 2>&1
echo "sp probe rc=$?"
