"""field_set_rhs folded into the density update (afh_fluid_set_rhs_output):
the rhs and max|rhs| the update writes for its output state must be bitwise
those of a separate field_set_rhs_maxabs call on that state (ghost cells
included; without the ghost option the interiors, whose values are all the
solver reads), for both Heun stages, on uniform and AMR trees and on the rod
electrode tree (level-set operators read the rhs of their boxes); the Heun
step that consumes them must be bitwise that of the unfused step. The library
tracks whether the fused rhs is still current (afh_fluid_rhs_valid): writing a
density of its state invalidates it. CPU: the C oracle; GPU: the HIP library
(and HIP == oracle)."""
import numpy as np
import pytest

import golden
from afh import capi
from afh.streamer import IV, StreamerCase, tables_from
from afh.tree import build_tree, uniform_tree
from test_dist import seed_state

TOPOS = {
    "uni8_l3": lambda: uniform_tree(8, (16, 16, 16), (2e-3, 2e-3, 2e-3), 3),
    "amr8": lambda: build_tree(
        8, (16, 16, 16), (2e-3, 2e-3, 2e-3), 2,
        refine=lambda lvl, r0, r1: lvl < 4 and np.all(r0 < 1.2e-3) and np.all(r1 > 0.7e-3)),
    # the reference's rod electrode fixture: level-set stencils on 15 boxes
    "rod8": lambda: "rod8",
}


def make(lib, topo, device, fused, ghosts=True):
    if isinstance(topo, str):
        c = golden.make_case(lib, golden.load(topo), coarse_cycles=0, device=device)
    else:
        g = golden.load("uni8")
        td, chem = tables_from(g)
        c = StreamerCase(lib, topo, td, chem, float(g["current_voltage"]),
                         coarse_cycles=0, device=device)
    seed_state(c)
    if fused:
        c.fuse_rhs(True, ghosts)
    return c


def leaf_rhs(c, ghosts=True):
    ids = []
    for l in range(1, int(c.topo["highest_lvl"]) + 1):
        ids += list(c.topo["lvl_leaves_%d" % l])
    r = c.tree.get_cc(IV["rhs"])[np.asarray(ids) - 1]
    return r if ghosts else r[:, 1:-1, 1:-1, 1:-1]


def check(lib, device, name, ghosts=True):
    topo = TOPOS[name]()
    a, b = make(lib, topo, device, True, ghosts), make(lib, topo, device, False)
    for c in (a, b):
        c.field_compute(0, check_residual=False)
    for s_deriv, s_prev, w_prev, s_out, last in [(0, [0], [1.0], 1, False),
                                                 (1, [0, 1], [0.5, 0.5], 0, True)]:
        la = a.fluid.forward_euler(1e-12, s_deriv, s_prev, w_prev, s_out, last, False)
        lb = b.fluid.forward_euler(1e-12, s_deriv, s_prev, w_prev, s_out, last, False)
        assert list(la) == list(lb)
        ma = a.fluid.rhs_maxabs(s_out)
        mb = b.fluid.field_set_rhs_maxabs(IV["rhs"], s_out)
        assert ma == mb
        assert np.array_equal(leaf_rhs(a, ghosts), leaf_rhs(b, ghosts))
        with pytest.raises(capi.AfhError):  # another state's rhs was not written
            a.fluid.rhs_maxabs(1 - s_out)
        assert a.fluid.rhs_valid(s_out) and not a.fluid.rhs_valid(1 - s_out)
    # any write of a density of that state makes the fused rhs stale
    a.tree.copy_cc(IV["pos"], IV["pos"])
    assert not a.fluid.rhs_valid(0)
    with pytest.raises(capi.AfhError):
        a.fluid.rhs_maxabs(0)
    # a whole Heun step through field_compute reuses the fused rhs
    for c in (a, b):
        c.field_compute(0)
    la, lb = a.heun_step(1e-12), b.heun_step(1e-12)
    assert la == lb
    # the fused update already wrote rhs(state 0); the field_compute after
    # af_advance (streamer.f90) consumes it, the unfused case recomputes it
    for c in (a, b):
        c.field_compute(0)
    for iv in (IV["e"], IV["pos"], IV["neg"], IV["phi"], IV["efld"]):
        assert np.array_equal(a.tree.get_cc(iv), b.tree.get_cc(iv)), iv
    assert np.array_equal(leaf_rhs(a, ghosts), leaf_rhs(b, ghosts))
    return a


@pytest.mark.parametrize("ghosts", [True, False])
@pytest.mark.parametrize("name", sorted(TOPOS))
def test_oracle_fused_rhs_equals_set_rhs(name, ghosts):
    check(capi.oracle_library(), -1, name, ghosts)


@pytest.mark.gpu
@pytest.mark.parametrize("ghosts", [True, False])
@pytest.mark.parametrize("name", sorted(TOPOS))
def test_hip_fused_rhs_equals_set_rhs(name, ghosts):
    a = check(capi.hip_library(), 0, name, ghosts)
    o = check(capi.oracle_library(), -1, name, ghosts)
    for iv in (IV["e"], IV["phi"], IV["efld"]):
        assert np.array_equal(a.tree.get_cc(iv), o.tree.get_cc(iv)), iv
    assert np.array_equal(leaf_rhs(a, ghosts), leaf_rhs(o, ghosts))
