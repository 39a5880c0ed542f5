#!/bin/bash
# rocprofv3 --kernel-trace A/B of environment sets on one config: each
# argument one variant (comma-separated NAME=VALUE, "default" = none), REPS
# alternating rounds; prints ms/step, the summed kernel time and the largest
# kernels' totals per run (KREGEX filters the listed kernels).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/envprof
for rep in $(seq ${REPS:-2}); do
  for v in "$@"; do
    tag=${CFG:-s1-64}_${v//,/+}_$rep
    envs=()
    [ "$v" = default ] || IFS=',' read -ra envs <<< "$v"
    for e in "${envs[@]}"; do export "$e"; done
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/envprof/$tag \
      -o run -- python3 bench.py --config ${CFG:-s1-64} --steps ${STEPS:-4} --warmup 1 \
      --no-cpu-baseline > gpurun_out/envprof/$tag.log 2>&1 || { tail -3 gpurun_out/envprof/$tag.log; exit 1; }
    for e in "${envs[@]}"; do unset "${e%%=*}"; done
    python3 - "$tag" gpurun_out/envprof/$tag/run_kernel_trace.csv gpurun_out/envprof/$tag.log \
      "${KREGEX:-.}" <<'PY'
import csv, json, re, sys
tag, trace, log, rx = sys.argv[1:5]
tot, acc = 0, {}
for r in csv.DictReader(open(trace)):
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    tot += d
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("afh::", "")[:24]
    if re.search(rx, name):
        acc[name] = acc.get(name, 0) + d
line = json.loads([l for l in open(log) if l.startswith('{"metric"')][-1])
top = sorted(acc.items(), key=lambda x: -x[1])[:6]
print("%-44s %.3f ms/step kernels %.2f ms | %s" % (tag[:44], line["ms_per_step"], tot / 1e6,
      " ".join("%s=%.2f" % (n, d / 1e6) for n, d in top)), flush=True)
PY
  done
done
