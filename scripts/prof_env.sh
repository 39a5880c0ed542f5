#!/bin/bash
# rocprofv3 kernel stats of a short bench run under extra environment
# settings: prof_env.sh TAG VAR=VALUE ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; shift
for kv in "$@"; do export "$kv"; done
mkdir -p gpurun_out/penv
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/penv/$tag -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/penv/$tag.log 2>&1
