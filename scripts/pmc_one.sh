#!/bin/bash
# One PMC pass (counters in $1) over the bench for kernels matching $KREGEX.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc1
timeout -k 10 300 rocprofv3 --pmc $1 --kernel-include-regex "${KREGEX:-k_cs_small}" \
  --output-format csv -d gpurun_out/pmc1/${TAG:-p} -o run -- \
  python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc1/${TAG:-p}.log 2>&1
