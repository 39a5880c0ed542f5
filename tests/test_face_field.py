"""The flux's face field from the potential (afh_fluid_set_field_source).

field_from_potential stores the face field fac / dr * (phi_f - phi_{f-1})
(mg_box_lpl_gradient, m_af_multigrid.f90:1882-1900) and the flux reads it
(m_fluid.f90:160-205). With the field source set, the gradient writes |E|
only (afh_mg_compute_phi_gradient with i_fc = 0) and the flux kernels form
the same expression from phi and its ghost cells. Both Heun stages must be
bitwise the stored-field run: |E|, the face fluxes, the densities and the dt
limits, on uniform trees of every flux kernel's box size (8: k_flux_staged;
16, 32, 64: k_flux_lds) and on an AMR tree (refinement boundaries, where the
fine box's face field reads phi's mg_sides_rb ghost cells). The electrode's
gradient needs the stored face field: i_fc = 0 is refused there. CPU: the C
oracle; GPU: the HIP library, and HIP == oracle in the new mode."""
import numpy as np
import pytest

import golden
from afh import capi
from afh.streamer import FV, IV, StreamerCase, tables_from
from afh.tree import build_tree, uniform_tree
from test_dist import seed_state

TOPOS = {
    "uni8_l3": lambda: uniform_tree(8, (16, 16, 16), (2e-3, 2e-3, 2e-3), 3),
    "amr8": lambda: build_tree(
        8, (16, 16, 16), (2e-3, 2e-3, 2e-3), 2,
        refine=lambda lvl, r0, r1: lvl < 4 and np.all(r0 < 1.2e-3) and np.all(r1 > 0.7e-3)),
    "uni16_l3": lambda: uniform_tree(16, (32, 32, 32), (2e-3, 2e-3, 2e-3), 3),
    "amr16": lambda: build_tree(
        16, (32, 32, 32), (2e-3, 2e-3, 2e-3), 2,
        refine=lambda lvl, r0, r1: lvl < 3 and np.all(r0 < 1.2e-3) and np.all(r1 > 0.7e-3)),
    "uni32_l2": lambda: uniform_tree(32, (64, 64, 64), (2e-3, 2e-3, 2e-3), 2),
}
# 8 leaf boxes of 64^3 (k_flux_lds<64>): the oracle takes a few seconds
GPU_TOPOS = dict(TOPOS, uni64_l2=lambda: uniform_tree(64, (128, 128, 128),
                                                      (2e-3, 2e-3, 2e-3), 2))


def make(lib, topo, device, from_phi):
    g = golden.load("uni8")
    td, chem = tables_from(g)
    c = StreamerCase(lib, topo, td, chem, float(g["current_voltage"]),
                     coarse_cycles=0, device=device)
    seed_state(c)
    if from_phi:
        c.faces_from_phi(True)
    return c


def run(lib, device, topo):
    """Two Heun stages from the same state, face field from phi (a) and
    stored (b); returns a after checking a == b bitwise."""
    a, b = make(lib, topo, device, True), make(lib, topo, device, False)
    for c in (a, b):
        c.field_compute(0, check_residual=False)
    assert np.array_equal(a.tree.get_cc(IV["efld"]), b.tree.get_cc(IV["efld"]))
    for s_deriv, s_prev, w_prev, s_out, last in [(0, [0], [1.0], 1, False),
                                                 (1, [0, 1], [0.5, 0.5], 0, True)]:
        if s_deriv == 1:
            for c in (a, b):
                c.field_compute(1, check_residual=False)
        la = a.fluid.forward_euler(1e-12, s_deriv, s_prev, w_prev, s_out, last, True)
        lb = b.fluid.forward_euler(1e-12, s_deriv, s_prev, w_prev, s_out, last, True)
        assert list(la) == list(lb)
        fa, fb = a.tree.get_fc(FV["flux"]), b.tree.get_fc(FV["flux"])
        leaves = leaf_ids(a)
        assert np.array_equal(fa[leaves], fb[leaves])
        for sp in ("e", "pos", "neg"):
            assert np.array_equal(a.tree.get_cc(IV[sp] + s_out),
                                  b.tree.get_cc(IV[sp] + s_out)), sp
    return a


def leaf_ids(c):
    ids = []
    for l in range(1, int(c.topo["highest_lvl"]) + 1):
        ids += list(c.topo["lvl_leaves_%d" % l])
    return np.asarray(ids) - 1


@pytest.mark.parametrize("name", sorted(TOPOS))
def test_oracle_faces_from_phi_equal_stored(name):
    run(capi.oracle_library(), -1, TOPOS[name]())


def test_oracle_norm_only_gradient_refused_with_electrode():
    lib = capi.oracle_library()
    c = golden.make_case(lib, golden.load("rod8"), coarse_cycles=0)
    with pytest.raises(capi.AfhError):
        c.mg.compute_phi_gradient(0, -1.0, IV["efld"])
    c = make(lib, TOPOS["uni8_l3"](), -1, True)
    with pytest.raises(capi.AfhError):  # the norm only needs a norm
        c.mg.compute_phi_gradient(0, -1.0, 0)
    with pytest.raises(capi.AfhError):  # no such potential variable
        c.fluid.set_field_source(c.tree.n_var_cell + 1, -1.0)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(GPU_TOPOS))
def test_hip_faces_from_phi_equal_stored(name):
    topo = GPU_TOPOS[name]()
    a = run(capi.hip_library(), 0, topo)
    o = make(capi.oracle_library(), topo, -1, True)
    o.field_compute(0, check_residual=False)
    lo = o.fluid.forward_euler(1e-12, 0, [0], [1.0], 1, False, True)
    h = make(capi.hip_library(), topo, 0, True)
    h.field_compute(0, check_residual=False)
    lh = h.fluid.forward_euler(1e-12, 0, [0], [1.0], 1, False, True)
    assert list(lo) == list(lh)
    leaves = leaf_ids(h)
    assert np.array_equal(h.tree.get_fc(FV["flux"])[leaves], o.tree.get_fc(FV["flux"])[leaves])
    for sp in ("e", "pos", "neg"):
        assert np.array_equal(h.tree.get_cc(IV[sp] + 1), o.tree.get_cc(IV[sp] + 1)), sp
    del a


@pytest.mark.gpu
def test_hip_norm_only_gradient_refused_with_electrode():
    c = golden.make_case(capi.hip_library(), golden.load("rod8"), coarse_cycles=0, device=0)
    with pytest.raises(capi.AfhError):
        c.mg.compute_phi_gradient(0, -1.0, IV["efld"])
