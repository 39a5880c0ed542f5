#!/bin/bash
# Round 3: per-kernel time of k_residual at column lengths 2, 4 (default) and
# 8 (AFH_RES_K) and of the gradient with and without non-temporal stores
# (AFH_GRAD_NT) on S1-64, rocprofv3 kernel stats, two rounds each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/rx
for rep in 1 2; do
  for v in AFH_RES_K=4 AFH_RES_K=2 AFH_RES_K=8 AFH_GRAD_NT=0 AFH_GRAD_NT=1; do
    d=gpurun_out/rx/${v}_$rep
    env $v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $d -o run -- python3 bench.py --config s1-64 --steps 5 --warmup 2 --no-cpu-baseline \
      > $d.log 2>&1 || { echo "rocprof $v rc=$?"; tail -5 $d.log; exit 1; }
    python3 - "$d" "$v" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "k_residual<true" in r["Name"] or "k_gradient_t" in r["Name"]:
        print("%-14s %-50s calls %4s avg %8.1f us" % (sys.argv[2], r["Name"][:50], r["Calls"],
              float(r["AverageNs"]) / 1e3), flush=True)
PY
  done
done
