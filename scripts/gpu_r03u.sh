#!/bin/bash
# Round 3: restriction columns of 8 coarse cells (AFH_RSTR_K=8). The bitwise
# test, then per-kernel time of k_rstr_fas_col at K = 4 and 8 on S1-64 and
# S1 (rocprofv3 kernel stats, two rounds each), then the bench clock.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/rk
timeout -k 10 300 python -u -m pytest tests/test_fusions.py -k restriction_columns -x -v \
  --timeout 200 --timeout-method thread > gpurun_out/rk/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/rk/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for cfg in s1-64 s1; do
    for k in 4 8; do
      d=gpurun_out/rk/${cfg}_k${k}_$rep
      AFH_RSTR_K=$k timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
        -d $d -o run -- python3 bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline \
        > $d.log 2>&1 || { echo "rocprof $cfg $k rc=$?"; tail -5 $d.log; exit 1; }
      python3 - "$d" "$cfg" "$k" <<'EOF'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "rstr_fas" in r["Name"] or r["Name"].startswith("void k_gsrb_pair2"):
        print("%-6s K=%s %-60s calls %5s avg %9.1f us total %9.1f us" % (
            sys.argv[2], sys.argv[3], r["Name"][:60], r["Calls"],
            float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e3), flush=True)
EOF
    done
  done
done
CFG=s1-64 REPS=2 bash scripts/ab_env_sets.sh AFH_RSTR_K=4 AFH_RSTR_K=8
