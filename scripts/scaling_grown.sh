#!/bin/bash
# Scaling projection of a grown driver tree (scripts/scaling_grown.py under
# one kernel trace; then scripts/project_scaling.py per size floor).
# CFG (s5), CELLS (4.4e6), FLOORS ("0 1048576"), NS ("2 4 8"), K (5).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CFG=${CFG:-s5}; CELLS=${CELLS:-4.4e6}; FLOORS=${FLOORS:-"0 1048576"}; NS=${NS:-"2 4 8"}
D=gpurun_out/scale_grown_$CFG
mkdir -p $D
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 ${PTIME:-900} rocprofv3 --kernel-trace --output-format csv -d $D/prof -o run -- \
  python3 scripts/scaling_grown.py $CFG $CELLS $D --ns $NS --floors $FLOORS --steps ${K:-5} \
  > $D/run.log 2> $D/run.err
rc=$?; echo "grown $CFG rc=$rc"; [ $rc -eq 0 ] || { tail -5 $D/run.err; exit $rc; }
T="$(find $D/prof -name "*kernel_trace.csv" | head -n 1)"
for F in $FLOORS; do
  for n in 1 $NS; do ln -sf "$(realpath "$T")" $D/f$F/n${n}_trace.csv; done
  python3 scripts/project_scaling.py $CFG $D/f$F $D/f$F/projection.json > /dev/null || exit 1
  python3 -c "import json; d = json.load(open('$D/f$F/projection.json')); \
print('$CFG floor $F', {n: (round(v['projected_speedup'], 2), round(v['projected_speedup_per_link'] or 0, 2)) for n, v in d['ranks'].items()})"
  rm -f $D/f$F/n*_trace.csv
done
rm -rf $D/prof
