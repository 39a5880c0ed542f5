#!/bin/bash
# Round 3, second GPU session: parity tests on the new fused kernels (one-launch
# level fill, pushed pair fill, one-workgroup coarse direct solve, armed
# reduction slots, one-launch gradient), then A/B of each on the S1 bench clock
# and all of them on S3; deferred reductions (one fetch per sub-step) on S1, S3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for v in AFH_GC_BOX AFH_PAIR_PUSH AFH_CS_DIRECT_SMALL; do
  CFG=s1 REPS=2 bash scripts/env_bench_ab.sh $v "0 1" || exit $?
done
CFG=s3 REPS=2 bash scripts/env_bench_ab.sh AFH_GC_BOX,AFH_PAIR_PUSH,AFH_CS_DIRECT_SMALL,AFH_UPD_NET "0 1" || exit $?
CFG=s3 REPS=2 bash scripts/env_bench_ab.sh AFH_UPD_NET "0 1" || exit $?
CFG=s3 REPS=2 bash scripts/env_bench_ab.sh AFH_ALL_LVL "0 1" || exit $?
CFG=s1 REPS=2 bash scripts/env_bench_ab.sh AFH_DEFER "0 1" || exit $?
CFG=s3 REPS=2 bash scripts/env_bench_ab.sh AFH_DEFER "0 1" || exit $?
CFG=s1-64 REPS=1 bash scripts/env_bench_ab.sh AFH_GC_BOX "1" || exit $?
