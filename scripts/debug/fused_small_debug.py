#!/usr/bin/env python3
"""Debug aid: one V-cycle on a regression-run tree with the small levels
split (default) and fused (AFH_GSRB_FUSED_MIN_BOXES=1), HIP, from the same
state; per level, the boxes whose phi differs."""
import os
import sys
sys.path[:0] = ["afivo-streamer_amd", "tests"]
import numpy as np
import golden
from afh import capi
from afh.driver import Simulation

sim = Simulation(capi.hip_library(), golden.load("rtest_test_3d"), device=0)
sim.start()
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 8):
    sim.step()
print("levels", sim.af.highest_lvl, "boxes", sim.af.highest_id, flush=True)
out = {}
for mode, env in (("split", "0"), ("fused", "1")):
    os.environ["AFH_GSRB_FUSED_MIN_BOXES"] = env
    s = sim.clone(capi.hip_library(), device=0)
    ops = sys.argv[2] if len(sys.argv) > 2 else "v"
    for op in ops:
        if op == "v":
            s.mg.fas_vcycle(True)
        elif op == "m":
            s.mg.fas_vcycle_maxres()
        elif op == "g":
            s.mg.fas_fmg(True, have_guess=True)
        elif op == "f":
            s.mg.fas_fmg(True, have_guess=False)
        elif op == "c":
            s.field_compute(0, True)
    out[mode] = (s.tree.get_cc(s.i_phi), s.tree.get_cc(s.i_tmp))
    os.environ.pop("AFH_GSRB_FUSED_MIN_BOXES")
for l in range(1, sim.af.highest_lvl + 1):
    ids = sim.af.lvls[l]["ids"]
    bad = [b for b in ids if not np.array_equal(out["split"][0][b - 1], out["fused"][0][b - 1])]
    d = max((np.max(np.abs(out["split"][0][b - 1] - out["fused"][0][b - 1])) for b in bad), default=0)
    nbs = [sim.af.neighbors[b] for b in bad[:3]]
    print("lvl %d: %d boxes, %d differ, max %.3e, e.g. %s nbs %s" % (l, len(ids), len(bad), d, bad[:3], nbs), flush=True)
