#!/bin/bash
# scratch: price the SP hipGraph on one GPU -- the per-rank 14B CFG step at SP = 8 / 4 and SP = 1,
# eager vs graph-replayed (tests/probes/sp_rank_compute.py, SPC_GRAPH=1; exchanges as device copies)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
SPC_GRAPH=1 SPC_REPS=4 timeout -k 10 500 python -u tests/probes/sp_rank_compute.py 8 4 1 2>&1 | grep -v amdgpu.ids | tee gpurun_out/sp_graph_price.log
