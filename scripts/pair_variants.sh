#!/bin/bash
# k_gsrb_pair2 variants on the S1-64 workload (bench lines per variant)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-default AFH_GSRB_PAIR_DEPTH=2 AFH_GSRB_PAIR_NT=512 AFH_GSRB_PAIR_TJ=32}; do
  echo "variant: $v"
  [ "$v" = default ] && v=""
  env $v timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/pv.json 2> gpurun_out/pv.err || { tail -5 gpurun_out/pv.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/pv.json')); r=d['roofline']; print('  %.3e cu/s  %.2f ms/step  pair %.1f us frac %.3f' % (d['value'], d['ms_per_step'], r['avg_launch_us'], r['frac']))"
done
