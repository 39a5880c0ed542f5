#!/bin/bash
# One GPU session, parameterised (replaces round 3's one-off gpu_r03*.sh).
# Steps run in this order, each under its own time limit; the session stops
# at the first crash / timeout (exit codes other than 0 = pass and
# 1 = test failures), and at a test failure too unless KEEP_GOING=1.
#   PYTEST=1      the whole -m gpu suite (PYTEST_ARGS: extra pytest args,
#                 e.g. "-k 2d" or a test file)
#   SMOKE=1       __graft_entry__.smoke()
#   BENCH=1       bench.py (BENCH_ARGS, default "--steps 20 --warmup 5")
#   AB="v1 v2"    scripts/ab_env_sets.sh over the variants (CFG, REPS, STEPS)
#   ENVPROF="v1 v2"  scripts/env_sets_prof.sh over the variants (rocprofv3
#                 kernel totals per run; CFG, REPS, STEPS, KREGEX)
#   LIBS="a.so b.so"  scripts/ab_kernels.sh over library builds ("default" =
#                 the in-tree one; scripts/build_variant.sh builds the others)
#   PLACEMENT=N   scripts/placement_probe.py: N allocations in one process
#   PROF="s1-64 s3"  scripts/prof_cfg.sh per config (PKTCAP=0 for graphs)
#   EXTRA="cmd"   one more command, last
# TAG names the logs under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-run}
ok() { local rc=$1; [ "$rc" -eq 0 ] || { [ "$rc" -eq 1 ] && [ -n "$KEEP_GOING" ]; }; }
if [ -n "$PYTEST" ]; then
  timeout -k 10 ${PYTEST_TIME:-1000} python -u -m pytest tests -m gpu -x -v --timeout 300 \
    --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -n 5 gpurun_out/pytest_$TAG.log
  ok $rc || exit $rc
fi
if [ -n "$SMOKE" ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -n 2 gpurun_out/smoke_$TAG.log
  [ "$rc" -eq 0 ] || exit $rc
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 20 --warmup 5} \
    > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
  rc=$?; echo "bench rc=$rc"; cut -c1-700 gpurun_out/bench_$TAG.json
  [ "$rc" -eq 0 ] || { tail -n 5 gpurun_out/bench_$TAG.err; exit $rc; }
fi
if [ -n "$AB" ]; then
  # shellcheck disable=SC2086
  bash scripts/ab_env_sets.sh $AB || exit $?
fi
if [ -n "$ENVPROF" ]; then
  # shellcheck disable=SC2086
  bash scripts/env_sets_prof.sh $ENVPROF || exit $?
fi
if [ -n "$LIBS" ]; then
  # shellcheck disable=SC2086
  bash scripts/ab_kernels.sh $LIBS || exit $?
fi
if [ -n "$PLACEMENT" ]; then
  timeout -k 10 400 python3 scripts/placement_probe.py $PLACEMENT \
    > gpurun_out/placement_$TAG.log 2>&1 || { tail -5 gpurun_out/placement_$TAG.log; exit 1; }
  grep -E "allocation|afh_pool" gpurun_out/placement_$TAG.log
fi
for cfg in $PROF; do
  CFG=$cfg BTIME=300 PTIME=300 bash scripts/prof_cfg.sh || exit $?
done
if [ -n "$EXTRA" ]; then
  bash -c "$EXTRA" || exit $?
fi
exit 0
