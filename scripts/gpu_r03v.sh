#!/bin/bash
# Round 3 end: bench line + rocprofv3 steady-state profile at HEAD for the
# headline (S1-64) and the small-box configs S1 and S3 (scripts/prof_cfg.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for c in s1-64 s1 s3; do
  CFG=$c PKTCAP=0 bash scripts/prof_cfg.sh || exit $?
done
