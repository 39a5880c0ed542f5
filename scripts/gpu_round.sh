#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprof. Stops at the first
# crash / timeout (exit codes other than 0 = pass and 1 = test failures).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
ok $rc || exit $rc
timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 5 --warmup 1} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench.log
[ "$rc" -eq 0 ] || exit $rc
if [ -n "$PROFILE" ]; then
  export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/prof.log
fi
