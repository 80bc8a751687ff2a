#!/bin/bash
# r6 step 4: the per-rank SP = 8 / SP = 4 step (exchanges as copies) with the held-CU reserve + piece pool vs without
set -o pipefail
mkdir -p gpurun_out
SPC_AB=piece_queue=1,0 timeout -k 10 600 python -u tests/probes/sp_rank_compute.py 8 > gpurun_out/r6_sp8_pieceq_s4.log 2>&1 || { tail -20 gpurun_out/r6_sp8_pieceq_s4.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r6_sp8_pieceq_s4.log
SPC_AB=piece_queue=1,0 timeout -k 10 600 python -u tests/probes/sp_rank_compute.py 4 > gpurun_out/r6_sp4_pieceq_s4.log 2>&1 || { tail -20 gpurun_out/r6_sp4_pieceq_s4.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r6_sp4_pieceq_s4.log
