#!/bin/bash
# Round 3: the face field from phi in the flux (afh_fluid_set_field_source):
# the whole -m gpu suite, then A/B on the bench clock (S1-64, S1, S3).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v \
  --timeout 300 --timeout-method thread > gpurun_out/pytest_h.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_h.log; [ $rc -eq 0 ] || exit $rc
CFG=s1-64 REPS=2 bash scripts/env_bench_ab.sh AFH_FACES_FROM_PHI "0 1" || exit $?
CFG=s1 REPS=2 bash scripts/env_bench_ab.sh AFH_FACES_FROM_PHI "0 1" || exit $?
CFG=s3 REPS=1 bash scripts/env_bench_ab.sh AFH_FACES_FROM_PHI "0 1" || exit $?
timeout -k 10 300 python bench.py --config 2d --no-cpu-baseline > gpurun_out/bench_h_2d.json 2> gpurun_out/bench_h_2d.err || exit $?
cut -c1-300 gpurun_out/bench_h_2d.json
