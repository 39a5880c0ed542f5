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


def _old_tree(lib, box_capacity=0):
    g = golden.load("regrid8")
    t = Tree(lib, g, int(g["n_var_cell"]), N_VAR_FACE, box_capacity=box_capacity)
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


def _regrid(lib, box_capacity=0):
    g, t = _old_tree(lib, box_capacity)
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
@pytest.mark.parametrize("capacity", [0, 128])
def test_hip_regrid_matches_reference_and_oracle(capacity):
    """capacity 0: new pools (copy); 128: the 73 new boxes fit the old
    pools, the regrid works in place."""
    g, th, ids = _regrid(capi.hip_library(), capacity)
    _, to, _ = _regrid(capi.oracle_library())
    for v in VARS:
        a = th.get_cc(golden.IVS[v])[ids]
        assert np.array_equal(a, g["regrid__" + v][ids]), v
        assert np.array_equal(a, to.get_cc(golden.IVS[v])[ids]), v


def refine_desc(g):
    """The harness' default_refinement parameters (golden_gen.f90
    dump_refine_flags), in afh_refine_desc."""
    from afh.streamer import IV
    p = g["refine_params"]
    d = capi.RefineDesc()
    d.i_electron, d.i_efld = IV["e"], IV["efld"]
    d.td_alpha_col, d.td_eta_col = 3, 4
    d.use_alpha_effective = 0
    d.buffer_width = int(g["refine_buffer"][0])
    d.adx, d.adx_fac, d.min_dens, d.derefine_dx, d.max_dx, d.min_dx = p[:6]
    d.init_fac = p[6]
    d.electrode_dx = 1e99
    d.n_seeds = 1
    d.seed_r0[0][:] = list(p[7:10])
    d.seed_r1[0][:] = list(p[10:13])
    d.seed_width[0] = p[13]
    d.n_regions = 1
    d.region_dr[0] = p[14]
    d.region_rmin[0][:] = list(p[15:18])
    d.region_rmax[0][:] = list(p[18:21])
    d.n_limits = 1
    d.limit_dr[0] = p[21]
    d.limit_rmin[0][:] = list(p[22:25])
    d.limit_rmax[0][:] = list(p[25:28])
    return d


def _flags(lib):
    g = golden.load("regrid8")
    case = golden.make_case(lib, g)
    for v in VARS:
        case.tree.put_cc(golden.IVS[v], g["regrid_in__" + v])
    return g, case.fluid.refine_flags(refine_desc(g))


def test_oracle_refine_flags_match_harness():
    """afo_refine_flags == default_refinement + cell_to_ref_flags as the
    harness evaluates them (reference LT_get_col / GM_dist_line / af_r_cc)."""
    g, (flags, masks) = _flags(capi.oracle_library())
    assert np.array_equal(flags, g["refine_flags"])
    assert np.array_equal(masks.astype(np.int64), g["refine_masks"].astype(np.int64) & 0xffffffff)
    assert len(set(flags.tolist())) == 3


@pytest.mark.gpu
def test_hip_refine_flags_match_harness():
    g, (flags, masks) = _flags(capi.hip_library())
    assert np.array_equal(flags, g["refine_flags"])
    assert np.array_equal(masks.astype(np.int64), g["refine_masks"].astype(np.int64) & 0xffffffff)


def _summary(cf, bw):
    """cell_to_ref_flags (m_af_core.f90:1111-1146) of cell flags cf[k][j][i]."""
    nc = cf.shape[0]
    flag = 1 if (cf == 1).any() else 0 if (cf == 0).any() else -1
    m = 0
    if bw > 0:
        for dk in (-1, 0, 1):
            for dj in (-1, 0, 1):
                for di in (-1, 0, 1):
                    if not (di or dj or dk):
                        continue
                    sl = []
                    for d in (dk, dj, di):
                        sl.append(slice(nc - bw, nc) if d == 1 else
                                  slice(0, bw) if d == -1 else slice(0, nc))
                    if (cf[tuple(sl)] == 1).any():
                        m |= 1 << ((dk + 1) * 9 + (dj + 1) * 3 + (di + 1))
    return flag, m


@pytest.mark.parametrize("which", ["oracle", "hip"])
def test_refine_cell_flags_reproduce_summary(which):
    """afh_refine_cell_flags: the cells a driver hands af_adjust_refinement
    give back the device summary exactly (random cell flags, several buffer
    widths, including slabs that cover the whole box)."""
    import ctypes as C
    lib = capi.oracle_library() if which == "oracle" else capi.hip_library()
    rng = np.random.default_rng(7)
    for nc, bw in [(8, 0), (8, 2), (8, 4), (16, 4), (16, 8), (4, 3)]:
        for trial in range(40):
            p = rng.choice([0.0, 0.002, 0.02, 0.3])
            cf = rng.choice([-1, 0], size=(nc, nc, nc), p=[0.5, 0.5]).astype(np.int32)
            if trial % 3 == 0:
                cf[:] = -1
            cf[rng.random((nc, nc, nc)) < p] = 1
            flag, mask = _summary(cf, bw)
            out = np.zeros(nc ** 3, np.int32)
            lib.call("refine_cell_flags", int(flag), C.c_uint32(mask), nc, bw,
                     out.ctypes.data_as(capi.P_i32))
            assert _summary(out.reshape(nc, nc, nc), bw) == (flag, mask)
