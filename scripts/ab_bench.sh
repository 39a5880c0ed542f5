#!/bin/bash
# A/B of library builds on one box through bench.py lines (alternating, REPS
# rounds): each argument is a library path, "default" = the in-tree build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in $(seq ${REPS:-2}); do
  for lib in "$@"; do
    l=$lib; [ "$lib" = default ] && l=""
    AFH_HIP_LIB=$l timeout -k 10 300 python bench.py --config ${CFG:-s1-64} --steps ${STEPS:-6} --warmup 2 --no-cpu-baseline > gpurun_out/abb.json 2> gpurun_out/abb.err || { tail -3 gpurun_out/abb.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/abb.json')); print('%-28s %.4g cu/s %.3f ms/step' % ('$lib', d['value'], d['ms_per_step']))"
  done
done
