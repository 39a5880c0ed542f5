#!/bin/bash
# Round 3: the whole -m gpu suite at HEAD (one-launch refinement-boundary
# restriction, phi face field without divisions), then A/B of the face
# field source on S3 and S1 and the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v \
  --timeout 300 --timeout-method thread > gpurun_out/pytest_l.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_l.log; [ $rc -eq 0 ] || exit $rc
CFG=s3 REPS=2 bash scripts/ab_env_sets.sh "AFH_FACES_FROM_PHI=0" "AFH_FACES_FROM_PHI=1" || exit $?
CFG=s1 REPS=2 bash scripts/ab_env_sets.sh "AFH_FACES_FROM_PHI=0" "AFH_FACES_FROM_PHI=1" || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench_l.json 2> gpurun_out/bench_l.err || exit $?
cut -c1-400 gpurun_out/bench_l.json
