#!/bin/bash
# Bench lines of the driver configs on grown trees: the
# time loop advanced untimed until the tree holds GROW leaf cells (default
# 4.33e6, the reference's 3d_pos start) or GS seconds pass, then K timed unit
# steps with the cpu_baseline. PROF=1 also runs the same under rocprofv3
# --selected-regions (collection paused during the growth, resumed for
# --profile-steps 5 steps after the timed region) and writes the steady
# per-step profile. Each step under its own time limit; stops at the first
# failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CFGS=${CFGS:-"s3 s4 s5"}; GROW=${GROW:-4.33e6}; GS=${GS:-300}; K=${K:-20}
mkdir -p gpurun_out
for CFG in $CFGS; do
  timeout -k 10 ${BTIME:-900} python3 -u bench.py --config $CFG --grow-cells $GROW \
    --grow-seconds $GS --steps $K --warmup 3 > gpurun_out/grown_$CFG.json \
    2> gpurun_out/grown_$CFG.err
  rc=$?; echo "grown $CFG rc=$rc"; cut -c1-300 gpurun_out/grown_$CFG.json
  [ $rc -eq 0 ] || { tail -5 gpurun_out/grown_$CFG.err; exit $rc; }
  if [ -n "$PROF" ]; then
    D=gpurun_out/gprof_$CFG
    AFH_BENCH_TOPO=gpurun_out/gtopo_$CFG.json DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 \
      timeout -k 10 ${BTIME:-900} rocprofv3 --selected-regions ${MARKER:+--marker-trace} --kernel-trace --stats \
      --output-format csv -d $D -o run -- \
      python3 bench.py --config $CFG --grow-cells $GROW --grow-seconds $GS --steps 5 \
      --warmup 3 --no-cpu-baseline --profile-steps 5 > gpurun_out/gprof_$CFG.json \
      2> gpurun_out/gprof_$CFG.err
    rc=$?; echo "gprof $CFG rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/gprof_$CFG.err; exit $rc; }
    T="$(find $D -name "*kernel_trace.csv" | head -n 1)"
    [ -n "$T" ] || { echo "no kernel trace under $D"; exit 1; }
    python3 scripts/prof_steady.py "$T" 4 gpurun_out/gsteady_$CFG.json \
      gpurun_out/gtopo_$CFG.json > /dev/null || exit 1
    cp "$(find $D -name "*kernel_stats.csv" | head -n 1)" gpurun_out/gstats_$CFG.csv
    rm -f "$T"
  fi
done
