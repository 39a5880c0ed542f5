#!/bin/bash
# Round 3: prolongation columns of 8 as an option (default 4) (default). The whole
# -m gpu suite, smoke(), then the default bench line and S1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v \
  --timeout 300 --timeout-method thread > gpurun_out/pytest_z2.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_z2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_z2.log 2>&1 || exit $?
tail -1 gpurun_out/smoke_z2.log
timeout -k 10 300 python bench.py > gpurun_out/bench_z2.json 2> gpurun_out/bench_z2.err || exit $?
cut -c1-300 gpurun_out/bench_z2.json
CFG=s1-64 REPS=2 bash scripts/ab_env_sets.sh default AFH_PROLONG_K=8
