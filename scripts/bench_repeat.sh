#!/bin/bash
# N fresh-process bench runs of one config (the step clock's spread across
# processes: DESIGN.md, the bimodal S1-64 clock). CFG, N, STEPS, WARMUP;
# extra bench arguments after the script name.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/rep
CFG=${CFG:-s1-64}; N=${N:-3}
for r in $(seq $N); do
  timeout -k 10 300 python bench.py --config $CFG --steps ${STEPS:-20} --warmup ${WARMUP:-5} \
    --no-cpu-baseline "$@" > gpurun_out/rep/${CFG}_$r.json 2> gpurun_out/rep/${CFG}_$r.err || exit $?
  python3 - gpurun_out/rep/${CFG}_$r.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["roofline"] or {}
print("%s  %.3f ms/step  %.4g cell-updates/s  %s %.1f us frac %.3f" % (
    sys.argv[1], d["ms_per_step"], d["value"], r.get("kernel", "")[:22],
    r.get("avg_launch_us", 0), r.get("frac", 0)), flush=True)
PY
done
