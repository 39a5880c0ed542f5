#!/bin/bash
# A/B timing on one box: rocprof kernel stats of the bench for each variant,
# alternating twice. A variant is a library path (a libafivo_hip.so build),
# optionally followed by :VAR=VALUE[,VAR=VALUE...] environment settings.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for rep in 1 2; do
  n=0
  for spec in "$@"; do
    n=$((n+1))
    lib=${spec%%:*}
    envs=""
    [ "$spec" != "$lib" ] && envs=$(echo "${spec#*:}" | tr ',' ' ')
    env $envs AFH_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/v${n}_r$rep -o run -- \
      python3 bench.py --steps ${STEPS:-4} --warmup 1 --no-cpu-baseline > gpurun_out/ab/v${n}_r$rep.log 2>&1 || exit $?
    echo "v$n r$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab/v${n}_r$rep.log)"
  done
done
