#!/bin/bash
# Round 4: the GPU suite with k_gc_faces_r (8 values per thread) on; the
# S1-64 A/B of the fill form and the XR pair
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 \
  --timeout-method thread > gpurun_out/pytest_r04j.log 2>&1 ||
  { tail -30 gpurun_out/pytest_r04j.log; exit 1; }
tail -3 gpurun_out/pytest_r04j.log
KREGEX='gsrb_pair2|gc_faces|corners' REPS=2 bash scripts/env_sets_prof.sh \
  "AFH_GC_FACES_R=1,AFH_PAIR_XR=0" "AFH_GC_FACES_R=8,AFH_PAIR_XR=0" \
  "AFH_GC_FACES_R=1,AFH_PAIR_XR=1" "AFH_GC_FACES_R=8,AFH_PAIR_XR=1" || exit 1
echo DONE
