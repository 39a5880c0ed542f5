#!/bin/bash
# Round 4: pool addresses of alternating allocations vs the pair's mode
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
AFH_LOG_POOLS=1 timeout -k 10 400 python3 scripts/placement_probe.py 4 > gpurun_out/placement_log.txt 2>&1 ||
  { tail -5 gpurun_out/placement_log.txt; exit 1; }
grep -E "allocation|afh_pool" gpurun_out/placement_log.txt
echo DONE
