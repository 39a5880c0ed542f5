#!/bin/bash
# Round 3: the line-per-thread one-workgroup direct coarse solve: bitwise
# tests (8^3, 16^3, 16x8x8 against the launches), then A/B of its size limit
# on S1 (16^3: the launches vs one workgroup) and on S3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fusions.py -m gpu -x -v -k "direct" \
  --timeout 300 --timeout-method thread > gpurun_out/pytest_p.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_p.log; [ $rc -eq 0 ] || exit $rc
CFG=s1 REPS=2 bash scripts/ab_env_sets.sh "AFH_CS_DS_CELLS=1024" "AFH_CS_DS_CELLS=4096" || exit $?
CFG=s3 REPS=2 bash scripts/ab_env_sets.sh "AFH_CS_DIRECT_SMALL=0" "AFH_CS_DIRECT_SMALL=1" || exit $?
