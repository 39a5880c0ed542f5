"""The one-box electrode level-1 solve as a dense product (round 4,
afivo-streamer_amd/csrc/afh_cs_direct.h; AFH_CS_ELEC_DIRECT, default on).

BASELINE config 4's level 1 is one 8^3 box with the rod's level-set stencil
and six physical faces. Round 3 solved it by red-black Gauss-Seidel until
phi was stationary, in one workgroup (465 us, a third of the S4 step,
profiles/r03_steady_s4_final.json). The fixed point of that iteration is the
solution of one 512-unknown linear system; its inverse is built on the host
when the stencil or the boundary conditions change, and every coarse solve
is one dense product. Both are our algorithms (the reference hands the
stencils to HYPRE, afivo/src/m_coarse_solver.f90:286-338, absent here), and
they solve the same discrete problem:

* CPU: on the C oracle the direct solve equals the iteration to 1e-13 after
  S4's initial refinement (field solves, a Heun step);
* GPU: libafivo_hip's direct solve equals the oracle's bitwise (the same
  inverse from the same host arithmetic, the same product order), and the
  device iteration to 1e-13.
"""
import os

import numpy as np
import pytest

import golden
from afh import capi
from afh.driver import Simulation


def _s4(lib, device=-1):
    sim = Simulation(lib, golden.load("case_s4"), device=device)
    sim.set_initial_conditions()
    return sim


def _run(sim):
    res = sim.field_compute(0, True)
    lim = sim.advance(1e-12)
    res += sim.field_compute(0, True)
    return res, lim, {iv: sim.tree.get_cc(iv) for iv in (sim.i_phi, sim.i_efld, sim.i_electron)}


def _rel(a, b):
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


@pytest.fixture
def direct_env(monkeypatch):
    def set_(on):
        monkeypatch.setenv("AFH_CS_ELEC_DIRECT", "1" if on else "0")
    return set_


def test_direct_equals_iteration_oracle(direct_env):
    base = _s4(capi.oracle_library())
    out = {}
    for on in (False, True):
        direct_env(on)
        out[on] = _run(base.clone(capi.oracle_library()))
    for iv in out[True][2]:
        assert _rel(out[True][2][iv], out[False][2][iv]) <= 1e-13, iv


@pytest.mark.gpu
def test_direct_hip_equals_oracle_and_iteration(direct_env):
    direct_env(True)
    sim = _s4(capi.hip_library(), device=0)
    osim = sim.clone(capi.oracle_library())
    gsim = sim.clone(capi.hip_library(), device=0)
    a, b = _run(sim), _run(osim)
    assert a[0] == b[0] and a[1] == b[1]
    for iv in a[2]:
        assert np.array_equal(a[2][iv], b[2][iv]), iv
    direct_env(False)
    c = _run(gsim)  # (multigrids created by the clone read the switch now)
    for iv in a[2]:
        assert _rel(a[2][iv], c[2][iv]) <= 1e-13, iv
