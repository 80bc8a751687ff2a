#!/bin/bash
# per-rank compute of one CFG step under Ulysses SP = 1/2/4/8 on one GPU (exchanges replaced by
# device copies): BASELINE C4's 1280x720x121 and the headline 832x480x73
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
SPC_SIZE=720p SPC_REPS=2 timeout -k 10 600 python -u tests/probes/sp_rank_compute.py 1 2 4 8 2>&1 | grep -v amdgpu.ids | tee gpurun_out/sp_rank_720p.log || exit 1
SPC_REPS=2 timeout -k 10 300 python -u tests/probes/sp_rank_compute.py 1 2 4 8 2>&1 | grep -v amdgpu.ids | tee gpurun_out/sp_rank_480p.log || exit 1
