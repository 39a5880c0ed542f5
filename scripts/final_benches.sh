#!/bin/bash
# The round's bench lines: for every config in CFGS the default bench.py
# line (with its cpu_baseline), then the same command under rocprofv3
# --kernel-trace --stats (the summary the roofline line's launch time is
# checked against). Outputs gpurun_out/${TAG}_<cfg>_bench.json and
# gpurun_out/${TAG}_<cfg>_prof/. Each step under its own time limit; stops at
# the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r06z}; CFGS=${CFGS:-"s1-64 s1 s3 s4 s5 2d"}
for CFG in $CFGS; do
  timeout -k 10 ${BTIME:-400} python bench.py --config $CFG ${BENCH_EXTRA:-} \
    > gpurun_out/${TAG}_${CFG}_bench.json 2> gpurun_out/${TAG}_${CFG}_bench.err
  rc=$?; echo "bench $CFG rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_${CFG}_bench.err; exit $rc; }
  DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 ${PTIME:-400} rocprofv3 --kernel-trace --stats \
    --output-format csv -d gpurun_out/${TAG}_${CFG}_prof -o run -- \
    python3 bench.py --config $CFG --no-cpu-baseline ${BENCH_EXTRA:-} \
    > gpurun_out/${TAG}_${CFG}_prof.json 2> gpurun_out/${TAG}_${CFG}_prof.err
  rc=$?; echo "rocprof $CFG rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_${CFG}_prof.err; exit $rc; }
  rm -f gpurun_out/${TAG}_${CFG}_prof/run_kernel_trace.csv
done
