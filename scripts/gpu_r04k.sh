#!/bin/bash
# Round 4: the pair's speed mode across allocations in one process, twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for p in 1 2; do
  timeout -k 10 400 python3 scripts/placement_probe.py 5 > gpurun_out/placement_$p.log 2>&1 ||
    { tail -5 gpurun_out/placement_$p.log; exit 1; }
  cat gpurun_out/placement_$p.log
done
echo DONE
