#!/bin/bash
# r6 step 6 (pool 1 vs pool+reserve 2 vs blocks 0): SP = 8 per-rank step with the exchanges as G-workgroup copy kernels on a side stream
# (RCCL's CU footprint), piece pool + held-CU reserve on / off
set -o pipefail
mkdir -p gpurun_out
SPC_G=0,16,64 SPC_PERSIST=1 SPC_OVERLAP=1 SPC_ENV=piece_queue=2,1,0 timeout -k 10 900 python -u tests/probes/sp_contention.py > gpurun_out/r6_sp_contention_s6.log 2>&1 || { tail -20 gpurun_out/r6_sp_contention_s6.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r6_sp_contention_s6.log
