#!/bin/bash
# Round 3: gradient column length variants with the |E|-only gradient.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CFG=s1-64 REPS=2 bash scripts/ab_kernels.sh default abv/gk2/libafivo_hip.so \
  abv/gk8/libafivo_hip.so || exit $?
