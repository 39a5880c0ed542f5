#!/bin/bash
# Round 3, profile session: bench line + rocprofv3 kernel trace + steady-state
# summary per config (scripts/prof_cfg.sh; graphs replayed with
# DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 under the profiler), then the counter passes
# for the small-box kernels VERDICT names (k_update<9>, k_gsrb_pair_box<8> on
# S3) and the S1-64 kernels (scripts/pmc_kernel.sh, one group per pass).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fusions.py tests/test_full_size.py -m gpu -v \
  --timeout 300 --timeout-method thread -k "DIRECT or s1" > gpurun_out/pytest_c.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_c.log; [ $rc -eq 0 ] || exit $rc
CFG=s1 REPS=2 bash scripts/env_bench_ab.sh AFH_CS_DIRECT_SMALL "0 1" || exit $?
for cfg in ${CFGS:-s1 s3 s4 s5 s1-64}; do
  CFG=$cfg PKTCAP=0 BSTEPS=10 K=5 bash scripts/prof_cfg.sh || exit $?
done
[ -n "$NO_PMC" ] && exit 0
CFG=s3 KREGEX="k_update|k_gsrb_pair_box|k_gc_box|k_gc_faces" PMC_STEPS=2 \
  bash scripts/pmc_kernel.sh || exit $?
CFG=s1-64 KREGEX="k_gsrb_pair2|k_flux_lds|k_update|k_gradient|k_gc_faces|k_rstr_fas|k_prolong|k_residual" \
  bash scripts/pmc_kernel.sh || exit $?
