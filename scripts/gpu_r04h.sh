#!/bin/bash
# Round 4: the whole GPU suite with the push defaults on; store-type variants
# of the pushing 64^3 pair (AFH_PAIR2_PUSH) against the pair + fill
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 \
  --timeout-method thread > gpurun_out/pytest_r04h.log 2>&1 ||
  { tail -30 gpurun_out/pytest_r04h.log; exit 1; }
tail -3 gpurun_out/pytest_r04h.log
AFH_PAIR2_PUSH=0 REPS=1 STEPS=4 bash scripts/ab_kernels.sh default || exit 1
AFH_PAIR2_PUSH=1 REPS=2 STEPS=4 bash scripts/ab_kernels.sh default abv/psplain/libafivo_hip.so \
  abv/psrowplain/libafivo_hip.so || exit 1
timeout -k 10 300 python bench.py --config 2d --steps 10 --warmup 2 > gpurun_out/bench_2d_r04h.json || exit 1
cat gpurun_out/bench_2d_r04h.json
echo DONE
