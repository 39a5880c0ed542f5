#!/bin/bash
# Config 4 (electrode) on the GPU: parity tests, then S4 / S5 bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_rtest.py -k "s4" tests/test_hip_parity.py -k "s4 or electrode" > gpurun_out/t_s4.log 2>&1
rc=$?; tail -6 gpurun_out/t_s4.log; [ $rc -eq 0 ] || exit $rc
for c in s4 s5; do
  timeout -k 10 400 python bench.py --config $c --steps 10 --warmup 2 > gpurun_out/bench_$c.log 2>&1
  rc=$?; tail -1 gpurun_out/bench_$c.log; [ $rc -eq 0 ] || exit $rc
done
