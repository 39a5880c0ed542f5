#!/bin/bash
# Counter passes for the kernels of one bench config (CFG, default s1-64)
# matching KREGEX, one group per pass: VALU / memory instruction mix, cycles
# and HBM bytes. V-cycle graphs are off (AFH_GRAPHS=0: the same kernels,
# dispatched one by one, so each dispatch carries its own counters).
# Output: gpurun_out/pmck_$CFG/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CFG=${CFG:-s1-64}
out=gpurun_out/pmck_$CFG
mkdir -p $out
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  AFH_GRAPHS=0 timeout -k 10 -s KILL ${PMC_TIME:-300} rocprofv3 --pmc $grp \
    --kernel-include-regex "${KREGEX:-k_flux}" \
    --output-format csv -d $out/p$i -o run -- \
    python3 bench.py --config $CFG --steps ${PMC_STEPS:-1} --warmup 0 --no-cpu-baseline \
    > $out/p$i.log 2>&1
  rc=$?; echo "pmc $CFG pass $i ($grp) rc=$rc"
  [ "$rc" -eq 0 ] || { tail -5 $out/p$i.log; exit $rc; }
done
python3 scripts/pmc_kernels_summary.py $out gpurun_out/pmc_kernels_$CFG.json
