#!/bin/bash
# Round 3: in-process A/B of the pair's non-temporal plane loads (one box,
# interleaved V-cycles), then the counter passes of scripts/gpu_r03n.sh.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROUNDS=6 timeout -k 10 300 python3 scripts/pair_ab.py default AFH_GSRB_PAIR_NTL=1 \
  > gpurun_out/pair_ab_ntl.log 2>&1 || { tail -5 gpurun_out/pair_ab_ntl.log; exit 1; }
tail -n 2 gpurun_out/pair_ab_ntl.log
bash scripts/gpu_r03n.sh || exit $?
