#!/bin/bash
# r5 GPU session 37: halo conv v2 + vectorised epilogue in the VAE -- 832x480x73 tiled encode / decode, VAE kernel stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u tests/probes/vae_bench.py > gpurun_out/r5_vae_bench_s37.log 2>&1 || { tail -20 gpurun_out/r5_vae_bench_s37.log; exit 1; }
grep -v "Warning\|amdgpu.ids" gpurun_out/r5_vae_bench_s37.log
cd /tmp && export TMPDIR=/tmp
VAE_REPS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/vae_prof_s37 -o vae -- python3 $R/tests/probes/vae_bench.py > $R/gpurun_out/r5_vae_prof_s37.log 2>&1 || { tail -20 $R/gpurun_out/r5_vae_prof_s37.log; exit 1; }
f=$(find $R/gpurun_out/vae_prof_s37 -name "*kernel_stats.csv" | head -1); cp $f $R/gpurun_out/kernel_stats_vae_r5s37.csv; head -8 $f | cut -c1-160
