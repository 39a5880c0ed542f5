#!/bin/bash
# Round-end evidence: GPU tests, smoke, the S1-64 bench line, then the bench
# lines of the other configurations (each printed as it finishes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BENCH_ARGS="--steps 10 --warmup 2" bash scripts/gpu_round.sh || exit 1
for c in s1 s3 s4 s5; do
  timeout -k 10 500 python bench.py --config $c --steps 20 --warmup 2 > gpurun_out/bench_$c.log 2>&1
  rc=$?; echo "bench $c rc=$rc"; grep -h '^{' gpurun_out/bench_$c.log | cut -c1-200
  [ $rc -eq 0 ] || exit $rc
done
