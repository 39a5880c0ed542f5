#!/bin/bash
# Round 3: x-interface pairing in the level fill (AFH_GC_XPAIR) -- the GPU
# tests that cover fills, an A/B on the bench clock -- and the steady-state
# profiles at HEAD (face field from phi) for S1-64 and S1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
AFH_GC_XPAIR=1 timeout -k 10 600 python -u -m pytest tests/test_ions.py tests/test_graphs.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > gpurun_out/pytest_i.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_i.log; [ $rc -eq 0 ] || exit $rc
CFG=s1-64 REPS=2 bash scripts/env_bench_ab.sh AFH_GC_XPAIR "0 1" || exit $?
CFG=s1-64 REPS=2 bash scripts/env_bench_ab.sh AFH_RSTR_K "2 4" || exit $?
CFG=s1-64 PKTCAP=0 BSTEPS=10 K=4 BTIME=300 PTIME=300 bash scripts/prof_cfg.sh || exit $?
CFG=s1 PKTCAP=0 BSTEPS=10 K=6 BTIME=240 PTIME=240 bash scripts/prof_cfg.sh || exit $?
