set -o pipefail
cd $GRAFT_REPO_ROOT
PMC_TAG=attn_w4 bash scripts/pmc.sh attn && python3 scripts/pmc_summary.py attn_w4 attn_fwd_w4 > gpurun_out/pmc_attn_w4/summary.txt 2>&1; cat gpurun_out/pmc_attn_w4/summary.txt
