#!/bin/bash
# Per-kernel A/B of library builds: rocprofv3 --kernel-trace --stats of a
# short bench run per build (alternating, REPS rounds); prints the total
# kernel time per step of the largest kernels. Arguments: library paths
# ("default" = the in-tree build).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/abk
for rep in $(seq ${REPS:-2}); do
  for lib in "$@"; do
    l=$lib; [ "$lib" = default ] && l=""
    tag=$(echo "$lib" | tr '/.' '__')_$rep
    AFH_HIP_LIB=$l timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d gpurun_out/abk/$tag -o run -- python3 bench.py --config ${CFG:-s1-64} \
      --steps ${STEPS:-4} --warmup 1 --no-cpu-baseline > gpurun_out/abk/$tag.log 2>&1 || \
      { tail -3 gpurun_out/abk/$tag.log; exit 1; }
    python3 - "$lib" gpurun_out/abk/$tag/run_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[2])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
top = sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:9]
print("%-30s total %.2f ms | " % (sys.argv[1][-30:], tot / 1e6) +
      " ".join("%s=%.0f" % (r["Name"].split("(")[0].replace("void ", "").replace("afh::", "")[:18],
                            float(r["TotalDurationNs"]) / 1e3) for r in top), flush=True)
PY
  done
done
