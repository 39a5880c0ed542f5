#!/bin/bash
# A/B of whole environment sets on the bench clock: each argument is one
# variant, a comma-separated list of NAME=VALUE ("default" = none); REPS
# alternating rounds; prints ms/step and the smoother fraction per run.
# Usage: CFG=s1-64 REPS=2 ab_env_sets.sh "A=0,B=2" "A=1,B=2" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/envsets
for rep in $(seq ${REPS:-2}); do
  for v in "$@"; do
    tag=${CFG:-s1-64}_${v//,/+}_$rep
    envs=()
    [ "$v" = default ] || IFS=',' read -ra envs <<< "$v"
    env "${envs[@]}" timeout -k 10 400 python3 bench.py --config ${CFG:-s1-64} --steps ${STEPS:-10} \
      --warmup ${WARMUP:-2} --no-cpu-baseline > gpurun_out/envsets/$tag.log 2>&1 || { tail -3 gpurun_out/envsets/$tag.log; exit 1; }
    python3 -c "
import json
d = json.loads([l for l in open('gpurun_out/envsets/$tag.log') if l.startswith('{')][-1])
r = d['roofline'] or {}
print('%-52s %.3f ms/step  %.3f G  frac %.3f  pair %.1f us' % ('$tag', d['ms_per_step'], d['value'] / 1e9, r.get('frac', 0), r.get('avg_launch_us', 0)), flush=True)"
  done
done
