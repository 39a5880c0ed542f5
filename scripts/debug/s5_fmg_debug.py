#!/usr/bin/env python3
"""Debug aid: Helmholtz FMG, HIP against the C oracle, on the sprite
(config 5) tree after its initial refinement, over lambda^2, coarse solver
and smoother variants (env read at afh_mg_create)."""
import os
import sys
sys.path[:0] = ["afivo-streamer_amd", "tests"]
import numpy as np
import golden
from afh import capi
from afh.driver import Simulation
from afh.model import Multigrid
from afh.users import Sprite3D


def rel(a, b):
    return np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300)


sim = Simulation(capi.hip_library(), golden.load("case_s5"), device=0, user=Sprite3D)
sim.start()
osim = sim.clone(capi.oracle_library())
for s in (sim, osim):
    s.fluid.photoi_set_src(s.i_rhs, s.photoi_coeff, alpha_col=3)
rhs0 = osim.tree.get_cc(osim.i_rhs)
iv = sim.helm_iv[0]
VARS = [("default", {}), ("split", {"AFH_GSRB_FUSED_MIN_BOXES": "0", "AFH_GSRB_PAIR_BOX": "0"}),
        ("nobox", {"AFH_GSRB_PAIR_BOX": "0"}), ("fused_all", {"AFH_GSRB_FUSED_MIN_BOXES": "1"})]
for lam2 in (0.0, 1.7e-3, 0.45, 1e3):
    for cc in (0, 8):
        for name, env in VARS:
            os.environ.update(env)
            out = []
            for s in (sim, osim):
                s.tree.put_cc(s.i_rhs, rhs0)
                s.tree.put_cc(iv, np.zeros(s.tree.cc_shape))
                m = Multigrid(s.tree, iv, s.i_rhs, s.i_tmp, helmholtz_lambda=lam2,
                              coarse_cycles=cc,
                              coarse_mode=capi.COARSE_DIRECT if cc == 0 else capi.COARSE_CYCLES)
                m.fas_fmg(True, have_guess=False)
                out.append(s.tree.get_cc(iv))
                m.close()
            for k in env:
                os.environ.pop(k)
            print("lam2 %-8g coarse %s %-10s rel %.3g" % (lam2, "direct" if cc == 0 else "mg%d" % cc,
                                                         name, rel(out[0], out[1])), flush=True)
