#!/bin/bash
# Round 3, profiles at HEAD for the small-box configs (bench line + rocprofv3
# kernel trace + steady-state summary each; graphs replayed with
# DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 under the profiler). Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in ${CFGS:-s1 s3 s4 s5}; do
  CFG=$cfg PKTCAP=0 BSTEPS=10 K=5 BTIME=240 PTIME=240 bash scripts/prof_cfg.sh || exit $?
done
