#!/bin/bash
# HBM traffic of the dominant kernel from PMC counters, one counter group per
# pass (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE do not fit one pass).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c --kernel-include-regex "${KREGEX:-k_gsrb}" \
    --output-format csv -d gpurun_out/pmc/$c -o run -- \
    python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/pmc/$c.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"
  [ "$rc" -eq 0 ] || exit $rc
done
