#!/bin/bash
# SQ counter passes (one group per pass) for one kernel of the S1-64 bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcsq
timeout -k 10 60 rocprofv3 -L > gpurun_out/pmcsq/avail.txt 2>&1 || true
i=0
IFS=';' read -ra GRPS <<< "${GROUPS_SQ:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAIT_ANY}"
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  timeout -k 10 -s KILL 300 rocprofv3 --pmc $grp --kernel-include-regex "${KREGEX:-k_gsrb_pair2}" \
    --output-format csv -d gpurun_out/pmcsq/${TAG:-x}p$i -o run -- \
    python3 bench.py --config ${CFG:-s1-64} --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/pmcsq/${TAG:-x}p$i.log 2>&1
  rc=$?; echo "pmc pass $i rc=$rc"
  [ "$rc" -eq 0 ] || exit $rc
done
