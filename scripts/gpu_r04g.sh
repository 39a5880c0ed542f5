#!/bin/bash
# Round 4: the pair's pushed face fills (AFH_PAIR2_PUSH) -- bitwise tests,
# then A/Bs of the round's push switches on their configs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fusions.py -x -v --timeout 300 \
  --timeout-method thread -k "pair2 or push or 2d_pair" > gpurun_out/pytest_r04g.log 2>&1 ||
  { tail -30 gpurun_out/pytest_r04g.log; exit 1; }
tail -3 gpurun_out/pytest_r04g.log
KREGEX='gsrb_pair2|gc_faces|gc_corners|flux_lds' REPS=2 STEPS=4 bash scripts/env_ab.sh AFH_PAIR2_PUSH "0 1" || exit 1
CFG=s3 REPS=2 bash scripts/ab_env_sets.sh default "AFH_PROLONG_PUSH=1,AFH_RSTR_PUSH=1" || exit 1
CFG=2d REPS=2 bash scripts/ab_env_sets.sh default "AFH_PAIR2D=1" || exit 1
echo DONE
