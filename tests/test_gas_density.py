"""Variable gas density (gas_constant_density = .false.) on the species path.

flux_upwind (src/m_fluid.f90:146-154) then takes 1/N per face as
N_inv = 2 / (N_{f-1} + N_f) from the cc variable i_gas_dens, and
add_source_terms (src/m_fluid.f90:339-348) evaluates the reduced field per
cell as E / N and gives the gas species (first in the reactions' species
list, m_chemistry.f90:193-197) the densities gas_fractions * N; they enter the
reaction products and the chemistry time-step limit.

No reference-generated vectors cover this mode (the harness builds the
constant-density case only), so it is pinned by the numpy restatement below
(each expression citing its m_fluid.f90 line), by the property that a uniform
N field reproduces the constant-density fluxes bitwise, and -- on the GPU --
by bitwise equality of the HIP library with the C oracle."""
import numpy as np
import pytest

from afh import capi
from afh.model import Fluid, Tree
from afh.tree import uniform_tree

NP = 64
X = np.linspace(0.0, 1000.0, NP)
# mobility, diffusion (x in Td), both scaled by N in the table
TD = np.stack([1e24 * (1 + X / 500), 1e24 + X * 1e20], axis=1)
CHEM = np.stack([1e-16 * (1 + X / 100)], axis=1)
INV_FAC = (NP - 1) / 1000.0
N0 = 2.414e25
FRAC = (0.79, 0.21)
K_ION, K_ATT = (1.0e-18, 50.0), 2.0e-17


def lt(col, x):
    """LT_get_col, vectorised (m_lookup_table.f90:330-406)."""
    frac = x * INV_FAC
    low = np.clip(np.ceil(frac), 1, NP - 1).astype(int)
    lf = np.where(frac <= 0, 1.0, np.where(frac >= NP - 1, 0.0, low - frac))
    return lf * col[low - 1] + (1 - lf) * col[low]


def make_case(lib, device, gas, limiter=capi.LIM_ZERO, uniform_n=False, seed=3):
    """Two-level uniform tree (64 leaf boxes of 4^3); e, M+, M- (2 states
    each), |E|, N. Returns (tree, fluid)."""
    rng = np.random.default_rng(seed)
    topo = uniform_tree(4, (8, 8, 8), (2e-3, 2e-3, 2e-3), 2)
    t = Tree(lib, topo, 8, 2, device=device)
    neu = [(capi.BC_NEUMANN, 0.0)] * 6
    for iv in range(1, 9):
        t.set_cc_methods(iv, neu, capi.RB_GC_INTERP_LIM)
    shp = t.cc_shape
    t.put_cc(1, 1e15 * (1 + rng.random(shp)))
    t.put_cc(3, 1e15 * (1 + rng.random(shp)))
    t.put_cc(5, 1e14 * (1 + rng.random(shp)))
    for iv in (2, 4, 6):
        t.put_cc(iv, np.zeros(shp))
    t.put_cc(7, 3e6 * (1 + rng.random(shp)))         # |E|: 120..250 Td
    if uniform_n:
        t.put_cc(8, np.full(shp, N0))
    else:
        t.put_cc(8, N0 * (0.6 + 0.8 * rng.random(shp)))
    t.put_fc(2, 3e6 * (rng.random(t.fc_shape) - 0.5))
    t.put_fc(1, np.zeros(t.fc_shape))
    for iv in (1, 7, 8):
        t.gc_tree(iv)
    td = {"rows_cols": TD, "x_min": 0.0, "inv_fac": INV_FAC}
    chem = {"rows_cols": CHEM, "x_min": 0.0, "inv_fac": INV_FAC}
    g = len(FRAC) if gas else 0
    # N2 + e -> 2e + M+ (linear form), O2 + e -> M- (constant form)
    reac = [{"rate_type": capi.RATE_LINEAR, "c": list(K_ION), "ix_in": [1, g + 1],
             "ix_out": [g + 1, g + 2], "mult_out": [2, 1]},
            {"rate_type": capi.RATE_CONSTANT, "c": [K_ATT], "ix_in": [2, g + 1],
             "ix_out": [g + 3], "mult_out": [1]}]
    if not gas:  # without gas species the inputs are the electrons alone
        for r in reac:
            r["ix_in"] = [1]
    kw = dict(i_gas_dens=8, gas_fractions=FRAC) if gas else {}
    f = Fluid(t, [1, 3, 5], [-1, 1, -1], 1, 7, 1, 2, N0, td, chem, reac,
              limiter=limiter, **kw)
    return t, f, topo


def flux_restated(t, topo):
    """flux_upwind with LIM_ZERO (first-order upwind) on every leaf face,
    src/m_fluid.f90:146-205; fc array of the leaves."""
    nc = t.nc
    ne, E, N = t.get_cc(1), t.get_cc(7), t.get_cc(8)
    Ef = t.get_fc(2)
    dx = 2e-3 / 8 / 2  # domain / coarse cells / 2 (level 2)
    inv_dx = 1 / dx
    out = {}
    for b in topo["lvl_leaves_2"]:
        q = b - 1
        F = np.zeros((3, nc + 1, nc + 1, nc + 1))
        for d in range(3):
            # move dimension d to the last axis (arrays are [k][j][i])
            ax = 2 - d
            n_ = np.moveaxis(ne[q], ax, -1)[1:-1, 1:-1]
            e_ = np.moveaxis(E[q], ax, -1)[1:-1, 1:-1]
            g_ = np.moveaxis(N[q], ax, -1)[1:-1, 1:-1]
            ex = np.moveaxis(Ef[q, d], ax, -1)[:-1, :-1]
            n_inv = 2 / (g_[..., :-1] + g_[..., 1:])                     # :151-153
            tfc = 0.5 * (e_[..., :-1] + e_[..., 1:]) * 1e21 * n_inv      # :172
            mu = lt(TD[:, 0], tfc) * n_inv                               # :173
            dc = lt(TD[:, 1], tfc) * n_inv                               # :174
            v = -mu * ex                                                 # :178
            u = np.where(-1 * ex > 0, n_[..., :-1], n_[..., 1:])
            fl = v * u - dc * inv_dx * (n_[..., 1:] - n_[..., :-1])      # :181
            full = np.zeros((nc + 1,) * 3)
            np.moveaxis(full, ax, -1)[:-1, :-1] = fl
            F[d] = full
        out[q] = F
    return out


def flux_case(lib, device, gas, **kw):
    t, f, topo = make_case(lib, device, gas, **kw)
    dt = f.flux_upwind_tree(0)
    F = t.get_fc(1)
    t.sync()
    return t, topo, dt, F


def test_oracle_flux_restated():
    t, topo, dt, F = flux_case(capi.oracle_library(), -1, True)
    want = flux_restated(t, topo)
    nc = t.nc
    for q, W in want.items():
        for d in range(3):
            sl = [slice(0, nc)] * 3
            sl[2 - d] = slice(0, nc + 1)
            got = F[q, d][tuple(sl)]
            np.testing.assert_allclose(got, W[d][tuple(sl)], rtol=1e-13,
                                       atol=1e-13 * np.abs(W[d]).max())


def test_oracle_uniform_n_matches_constant_density():
    """2 / (N + N) == 1 / N exactly: a uniform N field gives the constant-
    density fluxes and dt limits bitwise (Koren limiter)."""
    lib = capi.oracle_library()
    _, _, dt_a, Fa = flux_case(lib, -1, True, limiter=capi.LIM_KOREN, uniform_n=True)
    _, _, dt_b, Fb = flux_case(lib, -1, False, limiter=capi.LIM_KOREN, uniform_n=True)
    assert np.array_equal(Fa, Fb)
    assert dt_a == dt_b


def chem_restated(t, topo):
    """add_source_terms with gas species (src/m_fluid.f90:339-348, 398-470):
    the new densities of e, M+, M- and the chemistry dt limit."""
    E, N = t.get_cc(7), t.get_cc(8)
    ne, ni, nm = t.get_cc(1), t.get_cc(3), t.get_cc(5)
    ids = np.asarray(topo["lvl_leaves_2"]) - 1
    s = (ids, slice(1, -1), slice(1, -1), slice(1, -1))
    field = 1e21 * (E[s] / N[s])                                          # :346
    gas = [np.maximum(fr * N[s], 0.0) for fr in FRAC]                     # :340-343
    e = np.maximum(ne[s], 0.0)
    k1 = 1.0 * K_ION[0] * (field - K_ION[1])      # m_chemistry.f90:603
    k2 = 1.0 * K_ATT                              # m_chemistry.f90:601
    r1 = k1 * (1.0 * gas[0] * e)
    r2 = k2 * (1.0 * gas[1] * e)
    der = {"N2": -r1, "O2": -r2, "e": -r1 + 2 * r1 - r2, "M+": r1, "M-": r2}
    eps = 1e-100
    dens = {"N2": gas[0], "O2": gas[1], "e": e, "M+": np.maximum(ni[s], 0),
            "M-": np.maximum(nm[s], 0)}
    lim = min((np.maximum(dens[k], eps) / np.maximum(-der[k], eps)).min()
              for k in dens)                                              # :407-409
    return {"e": ne[s] + 1e-12 * der["e"], "M+": ni[s] + 1e-12 * der["M+"],
            "M-": nm[s] + 1e-12 * der["M-"]}, lim


def chem_case(lib, device):
    t, f, topo = make_case(lib, device, True)
    dt = 1e-12
    lim = f.flux_update_densities(dt, 0, [0], [1.0], 1, True)
    got = {"e": t.get_cc(2), "M+": t.get_cc(4), "M-": t.get_cc(6)}
    ids = np.asarray(topo["lvl_leaves_2"]) - 1
    got = {k: v[ids, 1:-1, 1:-1, 1:-1] for k, v in got.items()}
    t.sync()
    return t, topo, got, lim


def test_oracle_chemistry_restated():
    t, topo, got, lim = chem_case(capi.oracle_library(), -1)
    want, want_lim = chem_restated(t, topo)
    for k in want:
        np.testing.assert_allclose(got[k], want[k], rtol=1e-13, atol=0)
    # the gas species set the limit: their loss is the only negative derivative
    assert np.isclose(lim[0], want_lim, rtol=1e-13), (lim[0], want_lim)


def test_bad_gas_density_rejected():
    lib = capi.oracle_library()
    topo = uniform_tree(4, (4, 4, 4), (1e-3,) * 3, 1)
    t = Tree(lib, topo, 4, 2)
    t.set_cc_methods(1, [(capi.BC_NEUMANN, 0.0)] * 6, capi.RB_GC_INTERP_LIM)
    td = {"rows_cols": TD, "x_min": 0.0, "inv_fac": INV_FAC}
    chem = {"rows_cols": CHEM, "x_min": 0.0, "inv_fac": INV_FAC}
    with pytest.raises(capi.AfhError):
        Fluid(t, [1], [-1], 1, 3, 1, 2, N0, td, chem, [], i_gas_dens=9,
              gas_fractions=FRAC)
    with pytest.raises(capi.AfhError):  # species index beyond gas + plasma
        Fluid(t, [1], [-1], 1, 3, 1, 2, N0, td, chem,
              [{"rate_type": capi.RATE_CONSTANT, "c": [1.0], "ix_in": [4],
                "ix_out": [3], "mult_out": [1]}], i_gas_dens=2, gas_fractions=FRAC)


@pytest.mark.gpu
@pytest.mark.parametrize("limiter", [capi.LIM_ZERO, capi.LIM_KOREN])
def test_hip_flux_equals_oracle(limiter):
    _, _, dt_h, Fh = flux_case(capi.hip_library(), 0, True, limiter=limiter)
    _, _, dt_o, Fo = flux_case(capi.oracle_library(), -1, True, limiter=limiter)
    assert np.array_equal(Fh, Fo)
    assert dt_h == dt_o


@pytest.mark.gpu
def test_hip_chemistry_equals_oracle():
    _, _, gh, lh = chem_case(capi.hip_library(), 0)
    _, _, go, lo = chem_case(capi.oracle_library(), -1)
    for k in gh:
        assert np.array_equal(gh[k], go[k]), k
    assert lh[0] == lo[0]
