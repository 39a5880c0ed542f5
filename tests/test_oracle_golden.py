"""Pin the C oracle (oracle/lib/libafo.so) to the reference's own numerics.

The golden vectors were produced by afivo modules compiled from the reference
sources (oracle/Makefile, oracle/make_golden.py). Stages that do not involve
the level-1 solve must agree to rounding; V-cycle results depend on the exact
coarse solve (HYPRE in the reference, absent: both sides solve the level-1
problem to machine precision) and must agree within the north-star bound
1e-10 relative on the potential; densities within 1e-8 per sub-step.
"""
import numpy as np
import pytest

import golden
from afh import capi

TOL_EXACT = 1e-13   # pure per-cell arithmetic (rounding-level differences)
TOL_PHI = 1e-10     # north-star potential bound
TOL_DENS = 1e-8     # north-star species-density bound per RK sub-step


@pytest.fixture(scope="module")
def lib():
    return capi.oracle_library()


@pytest.mark.parametrize("coarse_cycles", [40, 0])
@pytest.mark.parametrize("case", golden.CASES)
def test_oracle_matches_reference(lib, case, coarse_cycles):
    """coarse_cycles 0: the exact separable level-1 solve (AFH_COARSE_DIRECT)."""
    report, dts, g = golden.run_golden(lib, case, isolated=True,
                                       coarse_cycles=coarse_cycles)
    bad = []
    for stage, errs in report.items():
        for var, e in errs.items():
            tol = TOL_EXACT
            if stage in golden.SOLVE_STAGES:
                tol = TOL_PHI
            if stage.startswith("update"):
                tol = TOL_DENS
            if not e <= tol:
                bad.append((stage, var, e, tol))
    assert not bad, bad
    # dt limits (m_af_flux_schemes.f90 / m_fluid.f90)
    if "flux1" in dts:
        np.testing.assert_allclose(dts["flux1"], g["log_flux1_dt"], rtol=1e-13)
    if "flux2" in dts:
        np.testing.assert_allclose(dts["flux2"], g["log_flux2_dt"], rtol=1e-13)
        np.testing.assert_allclose(dts["update2"], g["log_update2_dt"], rtol=1e-13)


def test_oracle_chained_heun_step(lib):
    """The whole Heun step chained from the initial state (no re-upload)."""
    report, _, _ = golden.run_golden(lib, "uni8", isolated=False)
    assert report["update2"]["e0"] < 1e-8
    assert report["field1"]["phi"] < 1e-10


@pytest.mark.parametrize("bc", [(-11, -11), (-10, -10), (-11, -10), (-10, -11)])
def test_direct_coarse_tables_diagonalise_folded_operator(bc):
    """The eigenbases of AFH_COARSE_DIRECT: Q orthonormal and
    T Q = Q diag(e) for the folded 1-D operator (ends -h Neumann / -3h
    Dirichlet, stencil_handle_boundaries)."""
    import ctypes as C
    lib = C.CDLL(capi.ORACLE_LIB)
    n, h = 12, 3.0
    q = np.zeros(n * n)
    e = np.zeros(n)
    lib.afo_cs_direct_tables(C.c_int(n), C.c_int(bc[0]), C.c_int(bc[1]), C.c_double(h),
                             q.ctypes.data_as(C.POINTER(C.c_double)),
                             e.ctypes.data_as(C.POINTER(C.c_double)))
    Q = q.reshape(n, n)
    T = h * (np.diag(-2 * np.ones(n)) + np.diag(np.ones(n - 1), 1) + np.diag(np.ones(n - 1), -1))
    T[0, 0] += h if bc[0] == -11 else -h
    T[-1, -1] += h if bc[1] == -11 else -h
    assert np.allclose(Q.T @ Q, np.eye(n), atol=1e-13)
    assert np.allclose(T @ Q, Q * e[None, :], atol=1e-12)
