#!/bin/bash
# HBM traffic of the dominant kernel from PMC counters: one counter per pass
# (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE do not fit one pass), each
# pass also profiling a calibration copy kernel with the same 8-B/lane access
# width (scripts/pmc_calib.hip). Summarised by scripts/pmc_summary.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
CFG=${CFG:-s1-64}
[ -x scripts/pmc_calib ] || hipcc --offload-arch=gfx950 -O3 scripts/pmc_calib.hip -o scripts/pmc_calib || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c --kernel-include-regex "${KREGEX:-k_gsrb_pair2}" \
    --output-format csv -d gpurun_out/pmc/$c -o run -- \
    python3 bench.py --config $CFG --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/pmc/$c.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"
  [ "$rc" -eq 0 ] || exit $rc
  timeout -k 10 120 rocprofv3 --pmc $c --kernel-include-regex k_calib \
    --output-format csv -d gpurun_out/pmc/calib_$c -o run -- \
    ./scripts/pmc_calib > gpurun_out/pmc/calib_$c.log 2>&1
  rc=$?; echo "pmc calib $c rc=$rc"
  [ "$rc" -eq 0 ] || exit $rc
done
