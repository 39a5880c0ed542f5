#!/bin/bash
# Round 3 (re-entry): the whole -m gpu suite at HEAD (2-D build included),
# the default bench line and the 2-D bench line. Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v \
  --timeout 300 --timeout-method thread > gpurun_out/pytest_g.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_g.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_g.json 2> gpurun_out/bench_g.err || exit $?
cut -c1-400 gpurun_out/bench_g.json
timeout -k 10 300 python bench.py --config 2d --no-cpu-baseline > gpurun_out/bench_g_2d.json 2> gpurun_out/bench_g_2d.err || exit $?
cut -c1-400 gpurun_out/bench_g_2d.json
