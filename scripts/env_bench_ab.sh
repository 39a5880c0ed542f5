#!/bin/bash
# A/B of a run-time switch on the bench's own clock (no profiler): bench.py
# per value, alternating, REPS rounds; prints ms/step and the smoother frac.
# Usage: CFG=s3 env_bench_ab.sh VAR[,VAR2...] "v1 v2 ..." (every VAR set to v)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
VAR=$1
mkdir -p gpurun_out/envbench
for rep in $(seq ${REPS:-2}); do
  for v in $2; do
    tag=${CFG:-s1-64}_${VAR//,/+}_${v}_$rep
    for var in ${VAR//,/ }; do export "$var=$v"; done
    timeout -k 10 400 python3 bench.py --config ${CFG:-s1-64} --steps ${STEPS:-10} --warmup 2 \
      --no-cpu-baseline > gpurun_out/envbench/$tag.log 2>&1 || { tail -3 gpurun_out/envbench/$tag.log; exit 1; }
    python3 -c "
import json, sys
d = json.loads([l for l in open('gpurun_out/envbench/$tag.log') if l.startswith('{')][-1])
print('%-44s %.3f ms/step  %.3f G  frac %.3f' % ('$tag', d['ms_per_step'], d['value'] / 1e9, d['roofline']['frac']), flush=True)"
  done
done
