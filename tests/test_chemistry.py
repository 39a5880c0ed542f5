"""Reaction-rate forms of get_rates (src/m_chemistry.f90:565-650) on the
density-update path: every rate type, one reaction A -> B per case on a
one-box tree, checked against a numpy restatement of the reference formulas
(CPU: the C oracle; GPU: the HIP library, which must also agree with the
oracle). Parity with reference-generated vectors exists only for the
tabulated form (tests/golden); the analytic forms are pinned by the formulas
restated below (each citing its line in m_chemistry.f90)."""
import numpy as np
import pytest

from afh import capi
from afh.model import Fluid, Tree
from afh.tree import uniform_tree

KB, EV = 1.3806503e-23, 1.6022e-19      # m_units_constants.f90:16,22
EV_TO_K = 2 * EV / (3 * KB)             # m_chemistry.f90:577-578
N_GAS = 2.414e25
TG = 320.0
NP = 64
E_TD = 120.0                            # reduced field in every cell (Td)

# transport table (mobility, diffusion, alpha, eta, mean energy) on
# [0, 1000] Td and one chemistry column, linear in x
X = np.linspace(0.0, 1000.0, NP)
TD = np.stack([1e24 + 0 * X, 1e24 + X * 1e20, 0 * X, 0 * X, 1.0 + 0.01 * X], axis=1)
CHEM = np.stack([1e-16 * (1 + X / 100)], axis=1)


def lt(col, x):
    """LT_get_col, linear x spacing (m_lookup_table.f90:330-406)."""
    inv = (NP - 1) / 1000.0
    frac = (x - 0.0) * inv
    low = int(np.ceil(frac))
    lf = low - frac
    return lf * col[low - 1] + (1 - lf) * col[low]


def te():
    return EV_TO_K * lt(TD[:, 4], E_TD)


C = [2.0e-16, 1.5, 310.0, 2.2]
# rate type -> numpy restatement of m_chemistry.f90:594-649 (c0 = 1)
FORMS = {
    capi.RATE_TABULATED_FIELD: lambda: lt(CHEM[:, 0], E_TD),                # :598
    capi.RATE_CONSTANT: lambda: C[0],                                          # :601
    capi.RATE_LINEAR: lambda: C[0] * (E_TD - C[1]),                            # :603
    capi.RATE_EXP_V1: lambda: C[0] * np.exp(-(C[1] / (C[2] + E_TD)) ** 2),    # :605
    capi.RATE_EXP_V2: lambda: C[0] * np.exp(-(E_TD / C[1]) ** 2),             # :607
    capi.RATE_K1: lambda: C[0] * (300 / te()) ** C[1],                        # :609-615
    capi.RATE_K3: lambda: (C[0] * ((KB / EV) * te() + C[1]) ** 2 - C[2]) * C[3],  # :616-621
    capi.RATE_K4: lambda: C[0] * (TG / 300) ** C[1] * np.exp(-C[2] / TG),     # :622
    capi.RATE_K5: lambda: C[0] * np.exp(-C[1] / TG),                           # :624
    capi.RATE_K6: lambda: C[0] * TG ** C[1],                                   # :626
    capi.RATE_K7: lambda: C[0] * (TG / C[1]) ** C[2],                          # :628
    capi.RATE_K8: lambda: C[0] * (300 / TG) ** C[1],                           # :630
    capi.RATE_K9: lambda: C[0] * np.exp(-C[1] * TG),                           # :632
    capi.RATE_K10: lambda: 10 ** (C[0] + C[1] * (TG - 300)),                  # :634
    capi.RATE_K11: lambda: C[0] * (300 / TG) ** C[1] * np.exp(-C[2] / TG),    # :636
    capi.RATE_K12: lambda: C[0] * TG ** C[1] * np.exp(-C[2] / TG),            # :638
    capi.RATE_K13: lambda: C[0] * np.exp(-(C[1] / (C[2] + E_TD)) ** C[3]),    # :640
    capi.RATE_K14: lambda: C[0] * np.exp(-(E_TD / C[1]) ** C[2]),             # :642
    capi.RATE_K15: lambda: C[0] * np.exp(-(C[1] / (KB * (TG + E_TD / C[2]))) ** C[3]),  # :644-649
}
# K10 takes c1 as an exponent, K15 needs c2 in joule: their own constants
CONST = {capi.RATE_K10: [-15.0, 0.01, 0.0, 0.0],
         capi.RATE_K15: [2.0e-16, 3.0e-21, 0.18, 2.0],
         capi.RATE_K1: [2.0e-16, 0.7, 0.0, 0.0], capi.RATE_K3: [2.0e-16, 0.5, 1e-3, 3.0],
         capi.RATE_K7: [2.0e-16, 300.0, 0.8, 0.0], capi.RATE_K9: [2.0e-16, 0.01, 0.0, 0.0],
         capi.RATE_K14: [2.0e-16, 150.0, 2.2, 0.0]}


def run_rate(lib, rate_type, device=-1):
    """One update step with the single reaction A -> B; returns (dt * rate
    from B, the expected dt * rate)."""
    global C
    c = CONST.get(rate_type, [2.0e-16, 1.5, 310.0, 2.2])
    C = c
    topo = uniform_tree(4, (4, 4, 4), (1e-3, 1e-3, 1e-3), 1)
    t = Tree(lib, topo, 6, 2, device=device)  # A (2 states), B (2), |E|, spare
    neu = [(capi.BC_NEUMANN, 0.0)] * 6
    for iv in (1, 2, 3, 4):
        t.set_cc_methods(iv, neu, capi.RB_GC_INTERP_LIM)
    td = {"rows_cols": TD, "x_min": 0.0, "inv_fac": (NP - 1) / 1000.0}
    chem = {"rows_cols": CHEM, "x_min": 0.0, "inv_fac": (NP - 1) / 1000.0}
    reac = [{"rate_type": rate_type, "table_col": 1, "rate_factor": 1.0, "c": c,
             "ix_in": [1], "ix_out": [2], "mult_out": [1]}]
    f = Fluid(t, [1, 3], [0, 0], 1, 5, 1, 2, N_GAS, td, chem, reac,
              gas_temperature=TG, td_energy_col=5)
    one = np.ones(t.cc_shape)
    t.put_cc(1, one)
    t.put_cc(3, 0 * one)
    t.put_cc(5, one * E_TD / 1e21 * N_GAS)  # |E| such that Td = E_TD
    dt = 1e-9
    f.flux_update_densities(dt, 0, [0], [1.0], 1, False)
    b = t.get_cc(4)[:, 1:-1, 1:-1, 1:-1]
    t.sync()
    return b, dt * FORMS[rate_type]()


@pytest.mark.parametrize("rate_type", sorted(FORMS))
def test_oracle_rate_forms(rate_type):
    got, want = run_rate(capi.oracle_library(), rate_type)
    assert np.allclose(got, want, rtol=1e-12, atol=0), (got.max(), want)


def test_energy_form_is_rejected():
    """rate_tabulated_energy (LEA, m_chemistry.f90:594) is not on the path."""
    with pytest.raises(capi.AfhError):
        run_rate(capi.oracle_library(), 0)


@pytest.mark.gpu
@pytest.mark.parametrize("rate_type", sorted(FORMS))
def test_hip_rate_forms(rate_type):
    got, want = run_rate(capi.hip_library(), rate_type, device=0)
    ref, _ = run_rate(capi.oracle_library(), rate_type)
    assert np.allclose(got, want, rtol=1e-12, atol=0), (got.max(), want)
    # exp / pow of the device math library may differ from glibc by an ulp
    assert np.allclose(got, ref, rtol=1e-14, atol=0)
