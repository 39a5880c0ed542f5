"""GPU parity: the HIP library (libafivo_hip.so) against the reference golden
vectors and against the C oracle on the same seeded inputs.

* golden: every stage of the reference's Heun step, per stage from the
  reference's own inputs -- bitwise for everything except the V-cycle (whose
  level-1 solve is HYPRE in the reference; both sides converge it), bounded
  by the north-star tolerances 1e-10 (potential) and 1e-8 (densities);
* oracle: HIP and C oracle run the identical algorithm including our coarse
  solver; results must be bitwise identical (max |diff| == 0), at sizes the
  oracle finishes in seconds, uniform and AMR;
* size-independent properties at larger sizes: V-cycles reduce the residual,
  ghost cells of a linear field are exact, the Heun step conserves charge
  flux-wise (interior fluxes cancel).
"""
import numpy as np
import pytest

import golden
from afh import capi
from afh.streamer import IV, FV, StreamerCase, seed_state, tables_from
from afh.tree import build_tree, uniform_tree

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hip():
    return capi.hip_library()


@pytest.fixture(scope="module")
def oracle():
    return capi.oracle_library()


# smoother variants: "split" = one launch per half-sweep with the level ghost
# fill in between (the reference's sequence); "fused" = k_gsrb_pair on every
# level (AFH_GSRB_FUSED_MIN_BOXES=1), which must give the same bits
# ("fused_tiles": the same with NC/4-row tiles per workgroup, the geometry of
# levels with 64..255 boxes, AFH_GSRB_TILES=1)
SMOOTHERS = {"split": ("0", "0"), "fused": ("1", "0"), "fused_tiles": ("1", "1")}


@pytest.fixture(params=sorted(SMOOTHERS))
def smoother(request, monkeypatch):
    fused_min, tiles = SMOOTHERS[request.param]
    monkeypatch.setenv("AFH_GSRB_FUSED_MIN_BOXES", fused_min)
    monkeypatch.setenv("AFH_GSRB_TILES", tiles)
    return request.param


# level-1 solve: 40 MG cycles, or the exact separable solve (AFH_COARSE_DIRECT)
COARSE = {"mg": 40, "direct": 0}


@pytest.mark.parametrize("coarse", sorted(COARSE))
@pytest.mark.parametrize("case", golden.CASES)
def test_hip_matches_reference_golden(hip, case, smoother, coarse):
    report, dts, g = golden.run_golden(hip, case, isolated=True,
                                       coarse_cycles=COARSE[coarse])
    bad = []
    for stage, errs in report.items():
        for var, e in errs.items():
            tol = 0.0
            if stage in golden.SOLVE_STAGES:
                tol = 1e-10
            if stage.startswith("update"):
                tol = 1e-8
            if not e <= tol:
                bad.append((stage, var, e, tol))
    assert not bad, bad
    if "flux1" in dts:
        np.testing.assert_allclose(dts["flux1"], g["log_flux1_dt"], rtol=1e-15)


def _pair(lib_a, lib_b, topo, g, coarse_cycles=12):
    td, chem = tables_from(g)
    v = float(g["current_voltage"])
    ca = StreamerCase(lib_a, topo, td, chem, v, coarse_cycles=coarse_cycles)
    cb = StreamerCase(lib_b, topo, td, chem, v, coarse_cycles=coarse_cycles)
    seed_state(ca)
    seed_state(cb)
    return ca, cb


def _assert_same(ca, cb, ivs=(), fvs=()):
    for iv in ivs:
        a, b = ca.tree.get_cc(iv), cb.tree.get_cc(iv)
        assert np.array_equal(a, b), (iv, np.max(np.abs(a - b)))
    for fv in fvs:
        a, b = ca.tree.get_fc(fv), cb.tree.get_fc(fv)
        fa, fb = golden.faces(a), golden.faces(b)
        for x, y in zip(fa, fb):
            assert np.array_equal(x, y), (fv, np.max(np.abs(x - y)))


TOPOS = {
    "uni16_l3": lambda: uniform_tree(16, (16, 16, 16), (2e-3, 2e-3, 2e-3), 3),
    "uni8_l4_2x1x1": lambda: uniform_tree(8, (16, 8, 8), (2e-3, 1e-3, 1e-3), 4),
    "uni64_l2": lambda: uniform_tree(64, (64, 64, 64), (4e-3, 4e-3, 4e-3), 2),
    "uni32_l2": lambda: uniform_tree(32, (32, 32, 32), (2e-3, 2e-3, 2e-3), 2),
    "amr16": lambda: build_tree(
        16, (32, 32, 32), (2e-3, 2e-3, 2e-3), 2,
        refine=lambda lvl, r0, r1: lvl < 3 and np.all(r0 < 1.2e-3) and np.all(r1 > 0.7e-3)),
    "amr8": lambda: build_tree(
        8, (16, 16, 16), (2e-3, 2e-3, 2e-3), 2,
        refine=lambda lvl, r0, r1: lvl < 4 and np.all(r0 < 1.2e-3) and np.all(r1 > 0.7e-3)),
}


@pytest.mark.parametrize("coarse", ["mg12", "direct"])
@pytest.mark.parametrize("name", sorted(TOPOS))
def test_hip_bitwise_equals_oracle_heun_step(hip, oracle, name, smoother, coarse):
    g = golden.load("uni8")
    topo = TOPOS[name]()
    ca, cb = _pair(hip, oracle, topo, g, 12 if coarse == "mg12" else 0)
    for c in (ca, cb):
        c.field_compute(0, check_residual=False)
    _assert_same(ca, cb, [IV["phi"], IV["tmp"], IV["rhs"], IV["efld"]], [FV["field"]])
    ca.store_flux = True  # the fused species step keeps the face fluxes
    la = ca.heun_step(1e-12, check_residual=False)
    lb = cb.heun_step(1e-12, check_residual=False)
    assert la == lb
    _assert_same(ca, cb, [IV["e"], IV["e"] + 1, IV["pos"], IV["neg"], IV["phi"]],
                 [FV["flux"], FV["field"]])


# forward_euler species sub-steps (s_deriv, s_prev, w_prev, s_out): the two
# Heun stages, a derivative state that is no previous state (one and two
# previous states), and the in-place step (which must take the two-call path)
FE_STEPS = [(0, [0], [1.0], 1), (1, [0, 1], [0.5, 0.5], 0), (1, [0], [1.0], 2),
            (2, [0, 1], [0.25, 0.75], 1), (1, [1], [1.0], 1)]


@pytest.mark.parametrize("fused", ["0", "2"])
@pytest.mark.parametrize("store", [0, 1])
@pytest.mark.parametrize("name", ["uni16_l3", "uni32_l2", "uni64_l2", "amr16"])
def test_forward_euler_equals_oracle(hip, oracle, name, store, fused, monkeypatch):
    """afh_fluid_forward_euler (with AFH_FE_FUSED=2: k_fe_lds on trees
    without coarse-fine flux corrections) gives the bits of the oracle's
    flux_upwind_tree + flux_update_densities: every species state, the dt
    limits, and with store_flux the face fluxes."""
    monkeypatch.setenv("AFH_FE_FUSED", fused)
    g = golden.load("uni8")
    ca, cb = _pair(hip, oracle, TOPOS[name](), g)
    for c in (ca, cb):
        c.field_compute(0, check_residual=False)
    states = [IV[sp] + s for sp in ("e", "pos", "neg") for s in range(3)]
    for n, (sd, sp, wp, so) in enumerate(FE_STEPS):
        last = n % 2 == 1
        la = ca.fluid.forward_euler(1e-12, sd, sp, wp, so, last, store_flux=store)
        lb = cb.fluid.forward_euler(1e-12, sd, sp, wp, so, last, store_flux=store)
        assert la == lb, (n, la, lb)
        _assert_same(ca, cb, states, [FV["flux"]] if store else [])


@pytest.mark.parametrize("helm", [0.0, 44081.25])
@pytest.mark.parametrize("name", sorted(TOPOS))
def test_hip_bitwise_equals_oracle_fmg(hip, oracle, name, smoother, helm):
    """mg_fas_fmg from phi = 0 and then with the result as guess; helm > 0:
    a photoionization Helmholtz mode (lambda^2 in the operator, Dirichlet 0
    on the z faces, m_photoi_helmh.f90:149-204)."""
    g = golden.load("uni8")
    ca, cb = _pair(hip, oracle, TOPOS[name](), g)
    mgs = []
    for c in (ca, cb):
        c.fluid.field_set_rhs(IV["rhs"], 0)
        if helm:
            c.set_voltage(0.0)
            mgs.append(c.helmholtz_mg(helm ** 2))
        else:
            mgs.append(c.mg)
    for mg in mgs:
        mg.fas_fmg(True, have_guess=False)
    _assert_same(ca, cb, [IV["phi"], IV["tmp"], IV["rhs"]])
    for mg in mgs:
        mg.fas_fmg(True, have_guess=True)
    _assert_same(ca, cb, [IV["phi"], IV["tmp"], IV["rhs"]])


@pytest.mark.parametrize("name", ["uni8_l4_2x1x1", "uni16_l3"])
def test_multigrids_sharing_a_tree(hip, oracle, name, smoother):
    """Several multigrids on one tree (the field solver and the Helmholtz
    photoionization modes): each one's fused pairs and the level fills that
    follow them use the tree's one spare image, whichever was created last
    (a per-multigrid image left the fills of the earlier ones filling
    another's). Interleaved FMGs, bitwise the oracle."""
    g = golden.load("uni8")
    ca, cb = _pair(hip, oracle, TOPOS[name](), g)
    mgs = []
    for c in (ca, cb):
        c.fluid.field_set_rhs(IV["rhs"], 0)
        c.set_voltage(0.0)
        mgs.append([c.mg, c.helmholtz_mg(1e6), c.helmholtz_mg(4e8)])
    for rnd in range(2):
        for k in (0, 2, 1):
            for m in mgs:
                m[k].fas_fmg(True, have_guess=rnd > 0)
            _assert_same(ca, cb, [IV["phi"], IV["tmp"], IV["rhs"]])
    mgs[0][2].close()  # the last-created one goes first
    mgs[1][2].close()
    for m in mgs:
        m[1].fas_fmg(True, have_guess=True)
    _assert_same(ca, cb, [IV["phi"], IV["tmp"], IV["rhs"]])


@pytest.mark.parametrize("name", ["amr8", "uni16_l3"])
def test_vcycle_from_stale_ghost_cells(hip, oracle, name, smoother):
    """A V-cycle whose phi has stale ghost cells (as after a regrid: afivo
    fills the ghost cells of the new boxes only, not those of their
    neighbours) runs its top level's first leg split, as
    the reference does: the fused pair's phase B would take this box's stale
    ghost column for the neighbour's boundary column. Seeded phi with zero
    ghost cells, uploaded; then V-cycles and an upload between them, bitwise
    the oracle."""
    g = golden.load("uni8")
    ca, cb = _pair(hip, oracle, TOPOS[name](), g)
    rng = np.random.default_rng(7)
    phi = rng.standard_normal(ca.tree.get_cc(IV["phi"]).shape) * 1e3
    phi[:, 0, :, :] = phi[:, -1, :, :] = 0.0
    phi[:, :, 0, :] = phi[:, :, -1, :] = 0.0
    phi[:, :, :, 0] = phi[:, :, :, -1] = 0.0
    for c in (ca, cb):
        c.fluid.field_set_rhs(IV["rhs"], 0)
        c.tree.put_cc(IV["phi"], phi)
        c.mg.fas_vcycle(True)
        c.mg.fas_vcycle(True)
    _assert_same(ca, cb, [IV["phi"], IV["tmp"]])
    for c in (ca, cb):
        c.tree.put_cc(IV["phi"], phi)
        c.mg.fas_vcycle(True)
    _assert_same(ca, cb, [IV["phi"], IV["tmp"]])


def test_vcycles_converge_large(hip, smoother):
    """Size-independent property at a larger size: each V-cycle reduces the
    max residual on the leaves by a large factor."""
    g = golden.load("uni8")
    topo = uniform_tree(32, (32, 32, 32), (4e-3, 4e-3, 4e-3), 4)
    td, chem = tables_from(g)
    c = StreamerCase(hip, topo, td, chem, 1e4, coarse_cycles=10)
    seed_state(c)
    c.fluid.field_set_rhs(IV["rhs"], 0)
    res = []
    for _ in range(5):
        c.mg.fas_vcycle(True)
        res.append(c.tree.maxabs_cc(IV["tmp"]))
    for a, b in zip(res, res[1:]):
        assert b < 0.35 * a, res


def test_ghost_cells_exact_for_linear_field(hip):
    """Face/edge/corner ghost cells of a field linear in z with matching
    Dirichlet values reproduce the field (copy, extrapolation and BC paths)."""
    g = golden.load("uni8")
    topo = uniform_tree(8, (16, 16, 16), (1.0, 1.0, 1.0), 3)
    td, chem = tables_from(g)
    c = StreamerCase(hip, topo, td, chem, 1.0)
    nc = 8
    idx = np.arange(nc + 2) - 0.5
    z = topo["meta_r_min"][:, 2, None] + idx[None, :] * topo["meta_dr"][:, 2, None]
    phi = np.ascontiguousarray(np.broadcast_to(z[:, :, None, None], c.tree.cc_shape))
    inner = phi.copy()
    inner[:, 0, :, :] = inner[:, -1, :, :] = 0
    inner[:, :, 0, :] = inner[:, :, -1, :] = 0
    inner[:, :, :, 0] = inner[:, :, :, -1] = 0
    c.tree.put_cc(IV["phi"], inner)
    c.tree.gc_tree(IV["phi"])
    out = c.tree.get_cc(IV["phi"])
    assert np.max(np.abs(out - phi)) < 1e-13


@pytest.mark.parametrize("name", ["amr8", "uni16_l3"])
def test_fused_maxabs_equals_separate(hip, oracle, name):
    """afh_field_set_rhs_maxabs / afh_mg_fas_vcycle_maxres (the reductions of
    field_compute folded into the rhs and residual passes) give the values of
    field_set_rhs + af_tree_maxabs_cc and mg_fas_vcycle + af_tree_maxabs_cc."""
    g = golden.load("uni8")
    ca, cb = _pair(hip, oracle, TOPOS[name](), g)
    ma = ca.fluid.field_set_rhs_maxabs(IV["rhs"], 0)
    cb.fluid.field_set_rhs(IV["rhs"], 0)
    mb = cb.tree.maxabs_cc(IV["rhs"])
    assert ma == mb and ma == ca.tree.maxabs_cc(IV["rhs"])
    _assert_same(ca, cb, [IV["rhs"]])
    for _ in range(2):
        ra = ca.mg.fas_vcycle_maxres()
        cb.mg.fas_vcycle(True)
        rb = cb.tree.maxabs_cc(IV["tmp"])
        assert ra == rb and ra == ca.tree.maxabs_cc(IV["tmp"])
    _assert_same(ca, cb, [IV["phi"], IV["tmp"]])


@pytest.mark.parametrize("coarse", [12, 0])
def test_electrode_bitwise_equals_oracle(hip, oracle, smoother, coarse):
    """The rod-electrode field solve (level-set stencils of the reference,
    tests/golden/rod8.npz) chained: two V-cycles, the gradient with the
    electrode faces, FMG without and with guess -- HIP == C oracle bitwise
    (the level-1 grid holds electrode boxes: Gauss-Seidel to stationarity)."""
    g = golden.load("rod8")
    cases = [golden.make_case(lib, g, coarse_cycles=coarse) for lib in (hip, oracle)]
    state = {**golden.stage_outputs(g, "init"), **golden.stage_outputs(g, "rhs")}
    names = ["phi", "tmp", "rhs", "efld", "fc_field"]
    for c in cases:
        golden.upload(c, state)
        c.mg.fas_vcycle(True)
        c.mg.fas_vcycle(True)
        c.field_from_potential()
    ra, rb = (golden.download(c, names) for c in cases)
    for n in names:
        assert np.array_equal(ra[n], rb[n]), n
    for c in cases:
        c.mg.fas_fmg(True, have_guess=False)
        c.mg.fas_fmg(True, have_guess=True)
    ra, rb = (golden.download(c, names[:3]) for c in cases)
    for n in names[:3]:
        assert np.array_equal(ra[n], rb[n]), n


@pytest.mark.gpu
def test_pair_ksplit16_bitwise_split(monkeypatch):
    """The fused pair on a 64^3 level of at most 16 boxes (a rank's share of
    a sharded level: S1-64's level 3 on 8 ranks) splits each box's march into
    16 chunks of 4 planes (k_gsrb_pair2<64, 64, 1, 16>, round 6): bitwise the
    split half-sweeps with their fills, over two V-cycles."""
    from afh.streamer import IV, StreamerCase, seed_state, tables_from
    from afh.tree import uniform_tree
    from afh import decks
    td, chem = tables_from(decks.load("tables_air_siglo"))
    topo = uniform_tree(64, (64, 64, 64), (2e-3, 2e-3, 2e-3), 2)  # 1 + 8 boxes
    out = []
    for fused in ("0", "1"):
        monkeypatch.setenv("AFH_GSRB_FUSED_MIN_BOXES", fused)
        monkeypatch.setenv("AFH_GRAPHS", "0")
        c = StreamerCase(capi.hip_library(), topo, td, chem, 5e3, device=0, coarse_cycles=0)
        seed_state(c, width=1e-4)
        res = c.field_compute(0, n_vcycles=2, check_residual=False)
        out.append((np.asarray(res), c.tree.get_cc(IV["phi"])))
        c.tree.close()
    assert np.array_equal(out[0][0], out[1][0])
    assert np.array_equal(out[0][1], out[1][1])
