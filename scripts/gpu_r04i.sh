#!/bin/bash
# Round 4: the pair storing the fill's x ghost cells (AFH_PAIR_XR) -- bitwise
# tests, then the S1-64 A/B against the pair + full fill
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fusions.py -x -v --timeout 300 \
  --timeout-method thread -k "pair_xr" > gpurun_out/pytest_r04i.log 2>&1 ||
  { tail -30 gpurun_out/pytest_r04i.log; exit 1; }
tail -3 gpurun_out/pytest_r04i.log
KREGEX='gsrb_pair2|gc_faces|gc_corners' REPS=2 STEPS=4 bash scripts/env_ab.sh AFH_PAIR_XR "0 1" || exit 1
echo DONE
