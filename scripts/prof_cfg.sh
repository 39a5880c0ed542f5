#!/bin/bash
# bench line + rocprofv3 kernel trace of one config (CFG), steady-state summary
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CFG=${CFG:-s1-64}; K=${K:-5}
mkdir -p gpurun_out/prof_$CFG
timeout -k 10 600 python bench.py --config $CFG --steps ${BSTEPS:-10} --warmup 2 > gpurun_out/bench_$CFG.json 2> gpurun_out/bench_$CFG.err
rc=$?; echo "bench $CFG rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_$CFG.err; exit $rc; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$CFG -o run -- \
  python3 bench.py --config $CFG --steps $K --warmup 2 --no-cpu-baseline > gpurun_out/prof_$CFG.log 2>&1
rc=$?; echo "rocprof $CFG rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/prof_steady.py gpurun_out/prof_$CFG/run_kernel_trace.csv $K gpurun_out/steady_$CFG.json
