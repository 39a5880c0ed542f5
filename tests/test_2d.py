"""BASELINE config 1: the 2-D build (libafivo_hip_2d.so, include/afivo_hip_2d.h).

The reference builds its 2-D library from the same sources with NDIM=2
(afivo/lib_2d/Makefile). oracle/Makefile (target ref2d) compiles those
sources the same way and oracle/harness/golden_gen2d.f90 drives them through
one Heun step of the hot path, an FMG and a Helmholtz FMG on two trees
(tests/golden/uni2d.npz: uniform, 2 x 2 level-1 boxes of 8^2, 3 levels;
amr2d.npz: 16 x 8 coarse cells refined around a point to level 5, with
refinement boundaries on every level); the fixtures are packed by
oracle/make_golden.py. The reference's compiled code is the oracle here: the
GPU tests compare the 2-D library stage by stage with those vectors, each
stage started from the reference's own input state -- bitwise for every stage
that does not involve the level-1 solve, within the north-star bounds (1e-10
on phi, 1e-8 on densities) for those that do (HYPRE PFMG, absent, is
replaced by an exact solve on both sides).

CPU: the library loads and exports exactly the entry points of
afivo_hip_2d.h (all of them part of afivo_hip.h's ABI); the fixtures are
self-consistent with a numpy restatement of two per-cell stages (the rhs,
the gradient with |E|).
"""
import numpy as np
import pytest

import golden
from afh import capi

CASES_2D = ["uni2d", "amr2d"]


def test_2d_header_is_a_subset_of_the_abi():
    sub = set(capi.header_symbols("afivo_hip_2d.h"))
    assert sub and sub <= set(capi.header_symbols())


def test_2d_library_exports_every_header_symbol():
    import ctypes
    lib = ctypes.CDLL(capi.HIP_LIB_2D)
    missing = [s for s in capi.header_symbols("afivo_hip_2d.h") if not hasattr(lib, s)]
    assert not missing, missing
    # loading through the product loader binds exactly those (no compute
    # call without a GPU)
    assert sorted(capi.hip_library_2d().symbols()) == capi.header_symbols("afivo_hip_2d.h")


def test_2d_uniform_tree_is_the_reference_topology():
    """afh.tree.uniform_tree_2d builds, id for id, the topology the reference's
    2-D af_init + af_refine_up_to_lvl built for the uni2d fixture (ids,
    children, neighbours, neighbor_mat, r_min, dr, level lists)."""
    from afh.tree import uniform_tree_2d
    g = golden.load("uni2d")
    t = uniform_tree_2d(8, (16, 16), g["domain"], 3)
    keys = [k for k in t if k in g]
    assert len(keys) >= 20
    for k in keys:
        assert np.asarray(t[k]).shape == np.asarray(g[k]).shape, k
        assert np.array_equal(t[k], g[k]), k


@pytest.mark.parametrize("case", CASES_2D)
def test_2d_fixture_rhs_and_gradient(case):
    """field_set_rhs (src/m_field.f90:363-401) on the leaves, whole blocks,
    and mg_box_lpl_gradient + mg_box_field_norm (m_af_multigrid.f90:1882-2010)
    restated in numpy reproduce the reference's stages bitwise."""
    g = golden.load(case)
    assert int(g["ndim"]) == 2
    ini = golden.stage_outputs(g, "init")
    rhs = golden.stage_outputs(g, "rhs")["rhs"]
    fac = -1.6022e-19 / 8.8541878176e-12
    leaves = np.concatenate([g["lvl_leaves_%d" % l] for l in range(1, int(g["highest_lvl"]) + 1)]) - 1
    # e, M+, M- in species order: 0 + q1 n1 + q2 n2 + q3 n3, left to right
    r = np.zeros_like(ini["e0"])
    for q, n in ((-1, "e0"), (1, "pos0"), (-1, "neg0")):
        r = r + (q * fac) * ini[n]
    assert np.array_equal(rhs[leaves], r[leaves])
    # gradient of the V-cycled potential (vcycle2's phi -> field0)
    phi = golden.stage_outputs(g, "vcycle2")["phi"]
    f0 = golden.stage_outputs(g, "field0")
    nc = int(g["nc"])
    dr = g["meta_dr"]
    ix = (-1.0 / dr[:, 0])[:, None, None]
    iy = (-1.0 / dr[:, 1])[:, None, None]
    fx = ix * (phi[:, 1:nc + 1, 1:nc + 2] - phi[:, 1:nc + 1, 0:nc + 1])
    fy = iy * (phi[:, 1:nc + 2, 1:nc + 1] - phi[:, 0:nc + 1, 1:nc + 1])
    ids = np.concatenate([g["lvl_ids_%d" % l] for l in range(1, int(g["highest_lvl"]) + 1)]) - 1
    assert np.array_equal(f0["fc_field"][ids, 0, :nc, :], fx[ids])
    assert np.array_equal(f0["fc_field"][ids, 1, :, :nc], fy[ids])
    sx = fx[:, :, :nc] + fx[:, :, 1:]
    sy = fy[:, :nc, :] + fy[:, 1:, :]
    en = 0.5 * np.sqrt(sx * sx + sy * sy)
    assert np.array_equal(f0["efld"][ids, 1:nc + 1, 1:nc + 1], en[ids])


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES_2D)
def test_2d_hip_matches_reference(case):
    """Every stage of the 2-D golden chain on libafivo_hip_2d.so: the rhs, the
    gradient, the flux (with af_gc2_box, af_consistent_fluxes) and the
    density updates bitwise; V-cycles, FMG and Helmholtz FMG within 1e-10
    (the level-1 solve); the dt limits to the 16 digits the harness logs."""
    report, dts, g = golden.run_golden(capi.hip_library_2d(), case, isolated=True,
                                       coarse_cycles=0, device=0)
    print(case, {s: {v: float(e) for v, e in r.items()} for s, r in report.items()})
    bad = []
    for stage, errs in report.items():
        for var, e in errs.items():
            tol = 0.0
            if stage in golden.SOLVE_STAGES:
                tol = 1e-10
            if not e <= tol:
                bad.append((stage, var, e))
    assert not bad, bad
    # (the harness log prints 16 digits)
    for stage, key in (("flux1", "log_flux1_dt"), ("flux2", "log_flux2_dt")):
        np.testing.assert_allclose(dts[stage], g[key], rtol=1e-15)
    np.testing.assert_allclose(dts["update2"][0], g["log_update2_dt"][0], rtol=1e-15)


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES_2D)
def test_2d_heun_step_chained(case):
    """The same chain run continuously (no re-upload between stages): the
    field solves with the threshold test of field_compute and the Heun step
    stay within the north-star bounds of the reference's states."""
    report, _, _ = golden.run_golden(capi.hip_library_2d(), case, isolated=False,
                                     coarse_cycles=0, device=0)
    for stage, errs in report.items():
        for var, e in errs.items():
            tol = 1e-10 if var in ("phi", "tmp", "rhs", "efld") or var.startswith("fc_") else 1e-8
            assert e <= tol, (stage, var, e)
