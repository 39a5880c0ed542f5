#!/bin/bash
# Round-3 first GPU session: parity tests, smoke, headline bench, S1 profile
# (graphs on), S3 profile with graph packet capture off. Stops at the first
# crash / timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; cut -c1-600 gpurun_out/bench.log
[ $rc -eq 0 ] || exit $rc
CFG=s1 BTIME=300 PTIME=300 bash scripts/prof_cfg.sh || exit $?
CFG=s3 PKTCAP=0 BTIME=300 PTIME=180 bash scripts/prof_cfg.sh || exit $?
