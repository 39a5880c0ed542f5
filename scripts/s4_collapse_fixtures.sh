#!/bin/bash
# Fixtures of tests/test_s4_collapse.py (build container; about three hours
# of CPU on 4 threads): the reference's own streamer.f90 on config 4 through
# the shim on the C oracle (oracle/_ref/dropin_streamer, `make -C oracle
# dropin`) from its set-up to the end of its time loop, and afh.driver's rows
# of the same run from the GPU box (scripts/s4_timeloop_rows.py, copied here
# from gpurun_out/).
#   bash scripts/s4_collapse_fixtures.sh [device rows json]
set -e
REPO=$(cd "$(dirname "$0")/.." && pwd)
W=${W:-/tmp/s4dropin}
mkdir -p $W
if [ ! -f $W/s4_rtest.log ] || [ -n "$RERUN" ]; then
  cd /root/reference/programs/standard_3d
  OMP_NUM_THREADS=${OMP_NUM_THREADS:-4} OMP_STACKSIZE=512M timeout 36000 \
    $REPO/oracle/_ref/dropin_streamer streamer_3d.cfg \
    -input_data%file=../../transport_data/air_chemistry_v2.txt -input_data%old_style=f \
    -use_electrode=T -field_electrode_grounded=T "-field_rod_r0=0.5 0.5 0.0" \
    "-field_rod_r1=0.5 0.5 0.15" -field_rod_radius=1e-3 -refine_electrode_dx=2e-4 \
    -refine_min_dx=1e-4 -output%name=$W/s4 -output%regression_test=T -silo_write=f \
    -end_time=2.5e-9 -output%dt=0.05e-9 > $W/stdout.txt 2>&1 || true
fi
cp $W/s4_rtest.log $REPO/tests/golden/s4_collapse_ref_rtest.txt
tail -n 12 $W/stdout.txt > $REPO/tests/golden/s4_collapse_ref_stop.txt
cp ${1:-$REPO/gpurun_out/s4_rows_hip.json} $REPO/tests/golden/s4_collapse_hip_rows.json
python3 $REPO/scripts/s4_collapse_compare.py $REPO/tests/golden/s4_collapse_hip_rows.json \
  $REPO/tests/golden/s4_collapse_ref_rtest.txt $W/stdout.txt $REPO/profiles/r06_s4_collapse.json
