import sys
sys.path[:0] = ["afivo-streamer_amd", "tests"]
import numpy as np
import golden
from afh import capi
from afh.driver import Simulation
from afh.users import Sprite3D
sim = Simulation(capi.hip_library(), golden.load("case_s5"), device=0, user=Sprite3D)
sim.start()
for _ in range(3):
    sim.step()
osim = sim.clone(capi.oracle_library())
def rel(a, b):
    return np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300)
for s in (sim, osim):
    s.fluid.photoi_set_src(s.i_rhs, s.photoi_coeff, alpha_col=3)
print("src rel", rel(sim.tree.get_cc(sim.i_rhs), osim.tree.get_cc(osim.i_rhs)), flush=True)
from afh.model import photoi_helmh_compute
for s in (sim, osim):
    n = photoi_helmh_compute(s.helm, s.helm_coeffs, s.i_photo, s.c.r("photoi_helmh%max_rel_residual"), 10)
    print("fmg counts", n, flush=True)
for iv in sim.helm_iv + [sim.i_photo]:
    print(sim.cc_names[iv - 1], rel(sim.tree.get_cc(iv), osim.tree.get_cc(iv)), flush=True)
print("max_rel_residual", sim.c.r("photoi_helmh%max_rel_residual"))
