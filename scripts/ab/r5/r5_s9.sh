#!/bin/bash
# r5 GPU session 9: attn_fwd_w4 item-switch stamps (-DVS_W4_STAMPS diagnostic build) on the
# cross-attention shape (512 keys = 8 tiles per item) and on the self-attention.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export VSTYLER_LIB=$R/video-styler_amd/vstyler/lib/diag_w4st/libvstyler.so
W4S_SKV=512 timeout -k 10 200 python -u tests/probes/w4_stamps.py > gpurun_out/r5_w4_switch_cross_s9.log 2>&1 || { tail -20 gpurun_out/r5_w4_switch_cross_s9.log; exit 1; }
grep -v Warning gpurun_out/r5_w4_switch_cross_s9.log
timeout -k 10 200 python -u tests/probes/w4_stamps.py > gpurun_out/r5_w4_switch_self_s9.log 2>&1 || { tail -20 gpurun_out/r5_w4_switch_self_s9.log; exit 1; }
grep -v Warning gpurun_out/r5_w4_switch_self_s9.log
