#!/bin/bash
# Counter passes for one kernel of the bench (KREGEX), one group per pass:
# VALU / memory instruction mix and HBM bytes. Output: gpurun_out/pmck/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmck
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $grp --kernel-include-regex "${KREGEX:-k_flux}" \
    --output-format csv -d gpurun_out/pmck/p$i -o run -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmck/p$i.log 2>&1
  rc=$?; echo "pmc pass $i ($grp) rc=$rc"
  [ "$rc" -eq 0 ] || exit $rc
done
