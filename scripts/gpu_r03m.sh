#!/bin/bash
# Round 3 final profiles at HEAD: bench line + rocprofv3 kernel trace +
# steady-state summary per config (graph packets built at launch under the
# profiler, PKTCAP=0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in ${CFGS:-s1-64 s1 s3 s4 s5}; do
  K=5; [ $cfg = s1-64 ] && K=4
  CFG=$cfg PKTCAP=0 BSTEPS=10 K=$K BTIME=300 PTIME=300 bash scripts/prof_cfg.sh || exit $?
done
