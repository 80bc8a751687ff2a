#!/bin/bash
# r5 GPU session 7: self / cross-attention on the 8-wave vs the 4-wave kernel (interleaved), the VAE
# encode/decode kernel-stats profile, and PMC passes of the cross-attention and the VAE convs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
ATTN_AB=8,4 timeout -k 10 300 python -u tests/probes/attn_bench.py > gpurun_out/r5_attn_impl_ab_s7.log 2>&1 || { tail -20 gpurun_out/r5_attn_impl_ab_s7.log; exit 1; }
grep -v Warning gpurun_out/r5_attn_impl_ab_s7.log
cd /tmp && export TMPDIR=/tmp
VAE_REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_vae_r5s7 -o run --output-format csv -- python3 $R/tests/probes/vae_bench.py > $R/gpurun_out/prof_vae_r5s7.log 2>&1 || { tail -20 $R/gpurun_out/prof_vae_r5s7.log; exit 1; }
grep -E "^(encode|decode)" $R/gpurun_out/prof_vae_r5s7.log
cd $R
PMC_TAG=cross_r5 timeout -k 10 900 bash scripts/pmc.sh cross > gpurun_out/pmc_cross_r5.log 2>&1 || { tail -20 gpurun_out/pmc_cross_r5.log; exit 1; }
python3 scripts/pmc_summary.py cross_r5 attn_fwd_d128
PMC_TAG=vae_r5 timeout -k 10 900 bash scripts/pmc.sh vae > gpurun_out/pmc_vae_r5.log 2>&1 || { tail -20 gpurun_out/pmc_vae_r5.log; exit 1; }
python3 scripts/pmc_summary.py vae_r5 vae_conv
