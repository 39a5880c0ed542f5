#!/bin/bash
# Round 3: 2x2 A/B of the fill pairing and the restriction column length
# (they measured faster each on its own but not together), plus the
# restriction workgroup size.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CFG=s1-64 REPS=3 bash scripts/ab_env_sets.sh "AFH_GC_XPAIR=0,AFH_RSTR_K=2" \
  "AFH_GC_XPAIR=1,AFH_RSTR_K=2" "AFH_GC_XPAIR=0,AFH_RSTR_K=4" "AFH_GC_XPAIR=1,AFH_RSTR_K=4" \
  "AFH_GC_XPAIR=0,AFH_RSTR_K=4,AFH_RSTR_BS=128" || exit $?
