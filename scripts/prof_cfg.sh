#!/bin/bash
# bench line + rocprofv3 kernel trace of one config (CFG), steady-state summary
# (scripts/prof_steady.py with the run's own topology, AFH_BENCH_TOPO).
# PKTCAP=0 runs the profiled process with DEBUG_CLR_GRAPH_PACKET_CAPTURE=0:
# the HIP runtime then builds the AQL packets of a graph's kernel nodes at
# launch instead of replaying captured ones (the S3 abort of
# round 2 under the profiler).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CFG=${CFG:-s1-64}; K=${K:-5}
mkdir -p gpurun_out/prof_$CFG
timeout -k 10 ${BTIME:-600} python bench.py --config $CFG --steps ${BSTEPS:-10} --warmup 2 \
  ${BENCH_EXTRA:-} > gpurun_out/bench_$CFG.json 2> gpurun_out/bench_$CFG.err
rc=$?; echo "bench $CFG rc=$rc"; cat gpurun_out/bench_$CFG.json | cut -c1-400
[ $rc -eq 0 ] || { tail -5 gpurun_out/bench_$CFG.err; exit $rc; }
[ -n "$PKTCAP" ] && export DEBUG_CLR_GRAPH_PACKET_CAPTURE=$PKTCAP
AFH_BENCH_TOPO=gpurun_out/topo_$CFG.json timeout -k 10 ${PTIME:-600} rocprofv3 --kernel-trace \
  --stats --output-format csv -d gpurun_out/prof_$CFG -o run -- \
  python3 bench.py --config $CFG --steps $K --warmup 2 --no-cpu-baseline ${BENCH_EXTRA:-} \
  > gpurun_out/prof_$CFG.log 2>&1
rc=$?; echo "rocprof $CFG rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/prof_$CFG.log; exit $rc; }
unset DEBUG_CLR_GRAPH_PACKET_CAPTURE
python3 scripts/prof_steady.py gpurun_out/prof_$CFG/run_kernel_trace.csv $K \
  gpurun_out/steady_$CFG.json gpurun_out/topo_$CFG.json
# (the trace of a grown tree is large: keep the summaries)
rm -f gpurun_out/prof_$CFG/run_kernel_trace.csv
