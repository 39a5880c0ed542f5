#!/usr/bin/env python3
"""Debug aid: test_3d to step 65 (split), then the state cloned twice (split
/ every level fused) and step 66's parts replayed on both: the Heun step,
the field solve, the regrid, the field solve after it; phi compared after
each part."""
import os
import sys
sys.path[:0] = ["afivo-streamer_amd", "tests"]
import numpy as np
import golden
from afh import capi
from afh.driver import Simulation


# argv: the B run's settings (default AFH_GSRB_FUSED_MIN_BOXES=1)
B_ENV = [a.split("=", 1) for a in sys.argv[1:]] or [["AFH_GSRB_FUSED_MIN_BOXES", "1"]]


def env(on):
    for k, v in B_ENV:
        if on:
            os.environ[k] = v
        else:
            os.environ.pop(k, None)


S = Simulation(capi.hip_library(), golden.load("rtest_test_3d"), device=0)
S.start()
for _ in range(65):
    S.step()
sims = []
for on in (False, True):
    env(on)
    sims.append(S.clone(capi.hip_library(), device=0))
env(False)


def cmp(tag):
    a, b = sims[0].tree.get_cc(sims[0].i_phi), sims[1].tree.get_cc(sims[1].i_phi)
    d = np.abs(a - b).reshape(len(a), -1).max(axis=1)
    lv = sorted(set(sims[0].af.lvl[q + 1] for q in np.nonzero(d > 0)[0]))
    print("%-28s phi max diff %.3e levels %s boxes %d" % (tag, d.max(), lv, sims[0].af.highest_id),
          flush=True)


def each(fn):
    for on, s in zip((False, True), sims):
        env(on)
        fn(s)
    env(False)


print("B:", B_ENV, "level boxes", [len(S.af.lvls[l]["ids"]) for l in range(1, S.af.highest_lvl + 1)], flush=True)
cmp("cloned at step 65")
each(lambda s: s.copy_current_state())
each(lambda s: s.advance(s.dt))
cmp("after advance")
each(lambda s: s.field_compute(0, True))
cmp("after field_compute")
for s in sims:
    for iv in s.densities:
        s.tree.restrict_tree(iv)
        s.tree.gc_tree(iv)
each(lambda s: s.adjust_refinement())
cmp("after regrid")
print("level boxes after regrid", [len(sims[0].af.lvls[l]["ids"]) for l in range(1, sims[0].af.highest_lvl + 1)], flush=True)
each(lambda s: s.field_compute(0, True))
cmp("after field_compute 2")
each(lambda s: s.field_compute(0, True))
cmp("after field_compute 3")
