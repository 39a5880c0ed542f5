#!/bin/bash
# Round 3: flux kernel tile size / register budget variants (library builds
# under abv/, scripts/build_variant.sh), per-kernel totals under the profiler.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CFG=s1-64 REPS=2 bash scripts/ab_kernels.sh default abv/fnt1024/libafivo_hip.so \
  abv/fminw2/libafivo_hip.so abv/fnt256/libafivo_hip.so || exit $?
