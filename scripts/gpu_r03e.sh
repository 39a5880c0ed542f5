#!/bin/bash
# Round 3: the line-pencil k_cs_direct_small (bitwise tests, A/B against the
# multi-launch direct solve) and the bench lines with one host sync per time
# step. Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fusions.py tests/test_full_size.py tests/test_graphs.py -m gpu -v \
  --timeout 300 --timeout-method thread > gpurun_out/pytest_e.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_e.log; [ $rc -eq 0 ] || exit $rc
CFG=s1 REPS=2 bash scripts/env_bench_ab.sh AFH_CS_DIRECT_SMALL "0 1" || exit $?
CFG=s5 REPS=1 bash scripts/env_bench_ab.sh AFH_CS_DIRECT_SMALL "0 1" || exit $?
for cfg in s1 s3; do
  CFG=$cfg PKTCAP=0 BSTEPS=10 K=6 BTIME=240 PTIME=240 bash scripts/prof_cfg.sh || exit $?
done
