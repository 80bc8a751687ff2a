#!/bin/bash
# r5 GPU session 16: PMC passes of the r5 self-attention (attn_fwd_w4 with the XCD item queues) at
# the 14B shape -- the bench line's `traffic` source -- and the stamps of the cross-attention's last tiles.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
PMC_TAG=attn_w4_r5 timeout -k 10 900 bash scripts/pmc.sh attn > gpurun_out/pmc_attn_w4_r5.log 2>&1 || { tail -20 gpurun_out/pmc_attn_w4_r5.log; exit 1; }
python3 scripts/pmc_summary.py attn_w4_r5 attn_fwd_w4
VSTYLER_LIB=$R/video-styler_amd/vstyler/lib/diag_w4st/libvstyler.so W4S_SKV=512 timeout -k 10 200 python -u tests/probes/w4_stamps.py > gpurun_out/r5_w4_lasttile_s16.log 2>&1 || { tail -20 gpurun_out/r5_w4_lasttile_s16.log; exit 1; }
grep -v "Warning\|amdgpu.ids" gpurun_out/r5_w4_lasttile_s16.log
