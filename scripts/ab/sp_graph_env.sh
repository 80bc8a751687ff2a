#!/bin/bash
# scratch: the world-1 SP graph-capture probe (tests/probes/sp_graph_probe.py) under variants:
# the native communicator on the caller's stream (no side stream in the capture).  A probe may end
# in a segfault: the script stops at the first failure.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
for knobs in "VSTYLER_SP_COMM_STREAM=caller"; do
  echo "== native $knobs" >> gpurun_out/sp_graph_env2.log
  env $knobs PYTHONFAULTHANDLER=1 VSTYLER_SP_GRAPH=1 timeout -k 10 120 python -u -X faulthandler tests/probes/sp_graph_probe.py native 3 >> gpurun_out/sp_graph_env2.log 2>&1
  rc=$?; echo "rc=$rc" >> gpurun_out/sp_graph_env2.log; echo "$knobs rc=$rc"
  [ $rc -eq 0 ] || exit 0
done
