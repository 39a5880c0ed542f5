"""Regrid (af_adjust_refinement's data movement, m_af_core.f90:697-881)
against tests/golden/regrid8.npz: the reference refined boxes near a point
and derefined boxes far from it (oracle/harness/golden_gen.f90, case
regrid8); the densities are prolonged with af_prolong_limit (gminmod43),
phi and |E| with af_prolong_linear. Every box of the new tree must hold the
reference's bits: restricted parents, copied boxes, prolonged new boxes with
their ghost cells."""
import numpy as np
import pytest

import golden
from afh import capi
from afh.model import Tree
from afh.streamer import IV, N_VAR_FACE, StreamerCase

VARS = ["e0", "pos0", "neg0", "phi", "efld"]


def _old_tree(lib):
    g = golden.load("regrid8")
    t = Tree(lib, g, int(g["n_var_cell"]), N_VAR_FACE)
    neumann0 = [(capi.BC_NEUMANN, 0.0)] * 6
    for sp in ("e", "pos", "neg"):
        for s in range(3):
            t.set_cc_methods(IV[sp] + s, neumann0, capi.RB_GC_INTERP_LIM,
                             capi.LIM_GMINMOD43)
    t.set_cc_methods(IV["efld"], neumann0, capi.RB_GC_INTERP)
    for s in (0, 1):
        t.set_cc_methods(IV["phi"] + s, StreamerCase.phi_bc(float(g["current_voltage"])),
                         capi.RB_MG_SIDES)
    # tree%cc_auto_vars in af_set_cc_methods order (the originals only)
    for sp in ("e", "pos", "neg"):
        t.set_cc_prolong(IV[sp], capi.PROLONG_LIMIT, capi.LIM_GMINMOD43)
    t.set_cc_prolong(IV["efld"], capi.PROLONG_LINEAR)
    t.set_cc_prolong(IV["phi"], capi.PROLONG_LINEAR)
    for v in VARS:
        t.put_cc(golden.IVS[v], g["regrid_in__" + v])
    return g, t


def _regrid(lib):
    g, t = _old_tree(lib)
    after = {k[len("after_"):]: g[k] for k in g if k.startswith("after_")}
    t2 = t.regrid(after)
    ids = np.concatenate([np.asarray(after["lvl_ids_%d" % l]) for l in
                          range(1, int(after["highest_lvl"]) + 1)]) - 1
    return g, t2, ids


def test_regrid_topology_changed():
    g = golden.load("regrid8")
    before = set(np.concatenate([g["lvl_ids_%d" % l] for l in range(1, int(g["highest_lvl"]) + 1)]))
    after = set(np.concatenate([g["after_lvl_ids_%d" % l]
                                for l in range(1, int(g["after_highest_lvl"]) + 1)]))
    derefined = [i for i in before & after if g["meta_children"][i - 1][0] > 0
                 and g["after_meta_children"][i - 1][0] == 0]
    assert len(after - before) > 0 and len(before - after) > 0 and derefined


def test_oracle_regrid_matches_reference():
    g, t2, ids = _regrid(capi.oracle_library())
    for v in VARS:
        a = t2.get_cc(golden.IVS[v])[ids]
        b = g["regrid__" + v][ids]
        assert np.array_equal(a, b), (v, np.max(np.abs(a - b)))


@pytest.mark.gpu
def test_hip_regrid_matches_reference_and_oracle():
    g, th, ids = _regrid(capi.hip_library())
    _, to, _ = _regrid(capi.oracle_library())
    for v in VARS:
        a = th.get_cc(golden.IVS[v])[ids]
        assert np.array_equal(a, g["regrid__" + v][ids]), v
        assert np.array_equal(a, to.get_cc(golden.IVS[v])[ids]), v
