#!/usr/bin/env python3
"""Debug aid: test_3d on the device twice in lockstep, split small levels (A)
and every level fused (B, AFH_GSRB_FUSED_MIN_BOXES=1, read whenever a
multigrid is created); stops at the first step whose state differs and
reports the levels and variables."""
import os
import sys
sys.path[:0] = ["afivo-streamer_amd", "tests"]
import numpy as np
import golden
from afh import capi
from afh.driver import Simulation


# argv: extra VAR=value settings for run B; "cap=<f>" sets both runs'
# capacity factor (1.0: every regrid out of place)
EXTRA = [a.split("=", 1) for a in sys.argv[1:] if not a.startswith("cap=")]
CAP = [float(a[4:]) for a in sys.argv[1:] if a.startswith("cap=")] or [2.0]


def env(on):
    if on:
        os.environ["AFH_GSRB_FUSED_MIN_BOXES"] = "1"
        for k, v in EXTRA:
            os.environ[k] = v
    else:
        os.environ.pop("AFH_GSRB_FUSED_MIN_BOXES", None)
        for k, _ in EXTRA:
            os.environ.pop(k, None)


sims = []
for on in (False, True):
    env(on)
    s = Simulation(capi.hip_library(), golden.load("rtest_test_3d"), device=0,
                   capacity_factor=CAP[0])
    s.start()
    sims.append(s)
A, B = sims
for n in range(1, 2000):
    for on, s in ((False, A), (True, B)):
        env(on)
        more = s.step()
    if n >= 60:
        print("step", n, "boxes", A.af.highest_id, "regrid" if n % A.c.i("refine_per_steps") == 0 else "", flush=True)
    if A.af.highest_id != B.af.highest_id:
        print("step", n, "topology differs", A.af.highest_id, B.af.highest_id, flush=True)
        break
    bad = []
    for iv in [A.i_phi, A.i_efld] + list(A.densities):
        a, b = A.tree.get_cc(iv), B.tree.get_cc(iv)
        if not np.array_equal(a, b):
            diff = np.abs(a - b).reshape(len(a), -1).max(axis=1)
            boxes = np.nonzero(diff > 0)[0] + 1
            lv = sorted(set(A.af.lvl[b] for b in boxes if A.af.in_use[b]))
            bad.append((A.cc_names[iv - 1], len(boxes), lv, float(diff.max())))
    if bad:
        print("step", n, "t %.4e" % A.time, "levels", A.af.highest_lvl, bad, flush=True)
        break
    if n % 20 == 0:
        print("step", n, "t %.4e same, levels %d boxes %d" % (A.time, A.af.highest_lvl, A.af.highest_id), flush=True)
    if not more:
        break
