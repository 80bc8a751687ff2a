#!/bin/bash
# r5 GPU session 15: SP = 8 per-rank step with the exchanges as copy kernels of G workgroups on a side
# stream (the RCCL pattern), XCD queues vs static lists; per-rank compute at SP = 1/2/4/8 (r5 kernels).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
SPC_G=0,16,64 SPC_PERSIST=1 SPC_OVERLAP=1 SPC_QUEUE=1,0 timeout -k 10 400 python -u tests/probes/sp_contention.py > gpurun_out/r5_sp_contention_s15.log 2>&1 || { tail -20 gpurun_out/r5_sp_contention_s15.log; exit 1; }
grep -v "Warning\|amdgpu.ids" gpurun_out/r5_sp_contention_s15.log
bash scripts/sp_price.sh > gpurun_out/r5_sp_price_s15.log 2>&1 || { tail -20 gpurun_out/r5_sp_price_s15.log; exit 1; }
grep -v Warning gpurun_out/r5_sp_price_s15.log | tail -20
