"""BASELINE config 1's species step against the reference's own forward_euler.

tests/state2d.py builds a 2-D state deterministically (an AMR tree with
refinement boundaries on three levels, smooth densities of every species,
phi, |E| and the face field); oracle/make_replay2d.py handed it, in the build
container, to the reference's forward_euler compiled with NDIM = 2
(oracle/_ref/2d/replay_step: flux_upwind_tree with the m_fluid callbacks,
af_gc2_box and af_consistent_fluxes, flux_update_densities with
add_source_terms and get_rates) for both Heun sub-steps, and committed
dt_lim and the new densities (tests/golden/replay2d_*.npz). Here the same
state goes through libafivo_hip_2d.so's afh_fluid_forward_euler:

* streamer_2d.cfg (programs/standard_2d: air_chemistry_v1, 8 species, 25
  reactions with the field table, constant and both exponential rate forms);
* tests/test_2d.cfg (the old-style td_air_siglo_swarm model).

The bar is the reference's output bitwise. The exponential rate forms of
air_chemistry_v1 call exp, whose device (ocml) and host (glibc) results can
differ in the last ulp; those densities are held to 1e-13 relative, as the
3-D temperature forms are (tests/test_rtest.py), and the test reports how
many differ at all.
"""
import os

import numpy as np
import pytest

import golden
import state2d

HERE = os.path.dirname(os.path.abspath(__file__))


def _fixture(name):
    return np.load(os.path.join(HERE, "golden", "replay2d_%s.npz" % name))


@pytest.mark.parametrize("name", sorted(state2d.SPECS))
def test_2d_replay_fixture_matches_state(name):
    """The committed outputs belong to the state the code builds now: the
    leaves and their count."""
    _, af, cc, fc, _ = state2d.build_state(name)
    fx = _fixture(name)
    for k in range(len(state2d.STAGES)):
        leaves = sorted(af.leaves())
        assert sorted(fx["stage%d_leaves" % k].tolist()) == leaves
        assert af.highest_lvl == state2d.SPECS[name][2]


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(state2d.SPECS))
def test_2d_species_step_equals_reference(name):
    from afh import capi
    from afh.driver import Simulation
    c, af, cc, fc, dt = state2d.build_state(name)
    fx = _fixture(name)
    worst, n_diff = 0.0, 0
    for k, (s_deriv, s_prev, w_prev, s_out) in enumerate(state2d.STAGES):
        sim = Simulation(capi.hip_library_2d(), c, device=0)
        sim.af = af
        sim._bind(sim._create_tree())
        for iv, a in cc.items():
            sim.tree.put_cc(iv, a)
        for iv, a in fc.items():
            sim.tree.put_fc(iv, a)
        lim = sim.fluid.forward_euler(dt, s_deriv, s_prev, w_prev, s_out, True)
        ours = min(sim.dt_max, min(lim[0] * sim.cfl, lim[1], lim[2], lim[3]))
        ref_lim = float(fx["stage%d_dt_lim" % k][0])
        assert abs(ours - ref_lim) <= 1e-13 * abs(ref_lim), (k, ours, ref_lim)
        leaves = fx["stage%d_leaves" % k]
        for iv in c.ia("all_densities"):
            mine = sim.tree.get_cc(iv + s_out)[leaves - 1][:, 1:-1, 1:-1]
            theirs = fx["stage%d_iv%d" % (k, iv)]
            rel = np.abs(mine - theirs) / np.abs(theirs)
            worst = max(worst, float(rel.max()))
            n_diff += int(np.count_nonzero(mine != theirs))
            assert rel.max() <= 1e-13, (k, c.sa("cc_names")[iv - 1], rel.max())
        sim.tree.close()
    print("%s: max rel %.3g, %d values not bitwise" % (name, worst, n_diff))
    if name == "test_2d":  # no exp / pow in the old-style model: bitwise
        assert n_diff == 0
