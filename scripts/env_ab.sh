#!/bin/bash
# A/B of a run-time switch of the library (an AFH_* environment variable read
# at afh_mg_create / afh_fluid_create): rocprofv3 --kernel-trace --stats of a
# short bench run per value, alternating, REPS rounds; prints the kernels
# matching KREGEX (average us per launch of the largest launches) and the
# bench's ms/step. Usage: env_ab.sh VAR "v1 v2 ..."
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
VAR=$1
mkdir -p gpurun_out/envab
for rep in $(seq ${REPS:-2}); do
  for v in $2; do
    tag=${VAR}_${v}_$rep
    env_line="$VAR=$v"
    export "$env_line"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d gpurun_out/envab/$tag -o run -- python3 bench.py --config ${CFG:-s1-64} \
      --steps ${STEPS:-4} --warmup 1 --no-cpu-baseline > gpurun_out/envab/$tag.log 2>&1 || \
      { tail -3 gpurun_out/envab/$tag.log; exit 1; }
    python3 - "$tag" gpurun_out/envab/$tag/run_kernel_trace.csv gpurun_out/envab/$tag.log \
      "${KREGEX:-.}" <<'PY'
import csv, json, re, sys
tag, trace, log, rx = sys.argv[1:5]
acc = {}
tot = 0
for r in csv.DictReader(open(trace)):
    tot += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("afh::", "")
    if not re.search(rx, name):
        continue
    g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    a = acc.setdefault(name, {})
    a.setdefault(g, []).append(d)
line = json.loads([l for l in open(log) if l.startswith('{"metric"')][-1])
out = []
for name, by in sorted(acc.items()):
    g = max(by)
    out.append("%s=%.1fus(x%d)" % (name[:28], sum(by[g]) / len(by[g]) / 1e3, len(by[g])))
print("%-22s %.3f ms/step kernels %.2f ms | %s" % (tag, line["ms_per_step"], tot / 1e6,
                                                  " ".join(out)), flush=True)
PY
  done
done
