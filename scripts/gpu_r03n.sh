#!/bin/bash
# Round 3 counters at HEAD: HBM bytes of the dominant kernel with the
# calibration copy (scripts/pmc.sh) and the per-kernel groups of S1-64 and
# S3 (scripts/pmc_kernel.sh, one group per pass).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/pmc.sh || exit $?
python3 scripts/pmc_summary.py gpurun_out/pmc 3221225472 gpurun_out/r03_pmc_s1-64.json || exit $?
CFG=s1-64 KREGEX="k_gsrb_pair2|k_flux_lds|k_update|k_gradient|k_gc_faces|k_rstr_fas|k_prolong|k_residual" \
  bash scripts/pmc_kernel.sh || exit $?
CFG=s3 KREGEX="k_update|k_gsrb_pair_box|k_gc_box|k_flux_staged" PMC_STEPS=2 \
  bash scripts/pmc_kernel.sh || exit $?
