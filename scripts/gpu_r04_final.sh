#!/bin/bash
# Round 4 end: rocprofv3 summaries of every bench config (PKTCAP=0 for the
# graph-replayed ones), the PMC traffic of the S1-64 pair, and N fresh S1-64
# bench processes. Each step under its own time limit; stops at the first
# failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PKTCAP=0 PROF="${PROF:-s1-64 s4 s3 s5 s1 2d}" TAG=r04g bash scripts/gpu_round.sh || exit $?
if [ -n "$PMC" ]; then
  CFG=s1-64 timeout -k 10 400 bash scripts/pmc.sh > gpurun_out/pmc_r04.log 2>&1 || { tail -5 gpurun_out/pmc_r04.log; exit 1; }
  # algorithmic bytes per leaf pair launch: 24 B x 512 boxes x 64^3 cells
  python3 scripts/pmc_summary.py gpurun_out/pmc 3221225472 gpurun_out/pmc_s1-64_r04.json \
    >> gpurun_out/pmc_r04.log 2>&1 || { tail -5 gpurun_out/pmc_r04.log; exit 1; }
  cat gpurun_out/pmc_s1-64_r04.json
fi
exit 0
