#!/bin/bash
# Round 4, session b: the -m gpu suite (partition frontier, direct electrode
# solve), streaming bandwidth of contiguous allocations, and the S1-64 step
# clock under placement variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PYTEST=1 KEEP_GOING=1 TAG=r04b bash scripts/gpu_round.sh || exit $?
for g in x 0 4096 65536 1048576; do
  if [ $g = x ]; then timeout -k 5 60 ./scripts/stream_bw
  else STREAM_CONTIG=1 STREAM_GAP=$g timeout -k 5 60 ./scripts/stream_bw; fi || exit 1
done > gpurun_out/stream_contig.txt 2>&1
cat gpurun_out/stream_contig.txt
CFG=s1-64 REPS=2 STEPS=20 WARMUP=5 bash scripts/ab_env_sets.sh default AFH_PAIR_KS_LEAF=2 \
  AFH_PAIR_KS_LEAF=4 AFH_POOL_CONTIG=1,AFH_POOL_PAD=4096 AFH_POOL_CONTIG=1,AFH_POOL_PAD=65536 \
  AFH_POOL_CONTIG=1,AFH_POOL_PAD=1048576 AFH_POOL_CONTIG=1,AFH_ALT_OFF=65536 \
  AFH_POOL_CONTIG=1,AFH_PAIR_KS_LEAF=2
