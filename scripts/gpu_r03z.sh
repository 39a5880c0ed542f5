#!/bin/bash
# Round 3: per-kernel time of k_prolong at column lengths 4 (default) and 8
# (AFH_PROLONG_K) on S1-64, rocprofv3 kernel stats, two rounds; the bitwise
# test first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/rp
timeout -k 10 300 python -u -m pytest tests/test_fusions.py -k prolong_columns -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_z.log 2>&1 || { tail -20 gpurun_out/pytest_z.log; exit 1; }; tail -1 gpurun_out/pytest_z.log
export TMPDIR=/tmp
mkdir -p gpurun_out/rp
for rep in 1 2; do
  for v in AFH_PROLONG_K=4 AFH_PROLONG_K=8; do
    d=gpurun_out/rp/${v}_$rep
    env $v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $d -o run -- python3 bench.py --config s1-64 --steps 5 --warmup 2 --no-cpu-baseline \
      > $d.log 2>&1 || { echo "rocprof $v rc=$?"; tail -5 $d.log; exit 1; }
    python3 - "$d" "$v" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "k_prolong<" in r["Name"]:
        print("%-14s %-50s calls %4s avg %8.1f us" % (sys.argv[2], r["Name"][:50], r["Calls"],
              float(r["AverageNs"]) / 1e3), flush=True)
PY
  done
done
