#!/bin/bash
# Inputs of scripts/project_scaling.py for the configs in CFGS (default
# "s1-64 s5"): the N = 1 bench line + its rocprofv3 kernel trace, and for
# N in NS (default "2 4 8") the thread-rank bench (--transport local
# --shared-stream) + its kernel trace; then the projection. Each step under
# its own time limit; stops at the first failure. BENCH_EXTRA: more
# arguments of the thread-rank runs (e.g. --min-level-cells); TAG: a suffix
# of the output directory.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CFGS=${CFGS:-"s1-64 s5"}; NS=${NS:-"2 4 8"}; K=${K:-5}
for CFG in $CFGS; do
  D=gpurun_out/scale_$CFG${TAG}
  mkdir -p $D
  DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 ${PTIME:-400} rocprofv3 --kernel-trace \
    --output-format csv -d $D/prof_n1 -o run -- \
    python3 bench.py --config $CFG --steps $K --warmup 2 --no-cpu-baseline \
    > $D/n1.json 2> $D/n1.err
  rc=$?; echo "n1 $CFG rc=$rc"; [ $rc -eq 0 ] || { tail -5 $D/n1.err; exit $rc; }
  cp "$(find $D/prof_n1 -name "*kernel_trace.csv" | head -n 1)" $D/n1_trace.csv || exit 1
  for N in $NS; do
    timeout -k 10 ${PTIME:-400} rocprofv3 --kernel-trace --output-format csv \
      -d $D/prof_n$N -o run -- \
      python3 bench.py --config $CFG --transport local --gpus $N --shared-stream \
      --steps $K --warmup 2 ${BENCH_EXTRA} > $D/n$N.json 2> $D/n$N.err
    rc=$?; echo "n$N $CFG rc=$rc"; [ $rc -eq 0 ] || { tail -5 $D/n$N.err; exit $rc; }
    cp "$(find $D/prof_n$N -name "*kernel_trace.csv" | head -n 1)" $D/n${N}_trace.csv || exit 1
  done
  rm -rf $D/prof_n*
  python3 scripts/project_scaling.py $CFG $D $D/projection.json > /dev/null || exit 1
  # (the traces are large: keep the bench lines and the projection)
  for f in $D/n*_trace.csv; do wc -l $f; done
  rm -f $D/n*_trace.csv
  python3 -c "import json; d = json.load(open('$D/projection.json')); \
print('$CFG', {n: round(v['projected_speedup'], 2) for n, v in d['ranks'].items()})"
done
