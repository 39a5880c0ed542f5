#!/bin/bash
# Round 3: x-interface pairing and 4-cell restriction columns on by default:
# the whole -m gpu suite, the default bench line, steady profiles S1-64, S3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v \
  --timeout 300 --timeout-method thread > gpurun_out/pytest_j.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_j.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_j.json 2> gpurun_out/bench_j.err || exit $?
cut -c1-600 gpurun_out/bench_j.json
CFG=s1-64 REPS=2 bash scripts/env_bench_ab.sh AFH_RES_K "4 8" || exit $?
CFG=s1-64 PKTCAP=0 BSTEPS=10 K=4 BTIME=300 PTIME=300 bash scripts/prof_cfg.sh || exit $?
CFG=s3 PKTCAP=0 BSTEPS=10 K=6 BTIME=240 PTIME=240 bash scripts/prof_cfg.sh || exit $?
