#!/bin/bash
# PMC of the benchmarked step itself (eager steps, so every dispatch is counted): MFMA busy, wave
# cycles, waits and the effective clock per kernel family (scripts/pmc_step_summary.py)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
OUT=$R/gpurun_out/pmc_step
mkdir -p $OUT
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
timeout -k 10 400 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d $OUT -o p1 -- python3 $R/bench.py --steps 1 --warmup 1 --no-graph --no-cpu-baseline --no-e2e > $OUT/p1.log 2>&1 || { tail -5 $OUT/p1.log; exit 1; }
cd $R && python3 scripts/pmc_step_summary.py $OUT
