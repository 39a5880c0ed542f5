#!/bin/bash
# PMC passes for the round's profile: HBM bytes of the dominant kernel with
# the calibration copy (scripts/pmc.sh), then instruction-mix / cycle / byte
# counters of the main kernels (scripts/pmc_kernel.sh), one group per pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/pmc.sh || exit $?
KREGEX=${KREGEX:-"k_flux|k_update|k_gradient|k_gsrb_pair|k_set_rhs|k_prolong|k_residual|k_rstr_fas"} \
  bash scripts/pmc_kernel.sh || exit $?
