"""Mobile ions: the flux species after the electrons (input_data%mobile_ions
/ ion_mobilities, m_transport_data.f90:195-215, m_streamer.f90:253-282).

Each ion's face flux is sign(q) mu N_inv E_f u_f with the Koren-limited
upwind value u_f along sign(q) E_f and no diffusion; its mu u_f adds to the
electrons' in the dielectric relaxation limit and its CFL is ignored
(m_fluid.f90:207-214); flux_update_densities applies every flux species'
divergence. The case is test_3d_chem with N2+, O2+ and O2- mobile
(tests/golden/case_ions.npz, oracle/make_cases.py "ions"); the C oracle is
pinned to the reference's own forward_euler on it by
tests/test_reference_replay.py::test_species_step_replay_mobile_ions.
CPU: the descriptor is validated the same way by both libraries. GPU: the
HIP driver's state after three steps, handed to the oracle: Heun stage 1
fluxes of every species and the CFL and dielectric limits bitwise, the
densities to 1e-13 (rate forms with exp: ocml vs glibc in the last ulp);
stage 2 as test_rtest's S5 to 1e-12."""
import numpy as np
import pytest

import golden
from afh import capi
from afh.driver import Simulation
from afh.model import Fluid


def bad_ion_fluids(lib, device=-1):
    """Every malformed ion list is refused (afh_fluid_create)."""
    sim = Simulation(lib, golden.load("case_ions"), device=device)
    sim.start()
    c = sim.c
    plasma_iv = [sim.species_itree[n] for n in sim.plasma]
    e_sp = plasma_iv.index(sim.i_electron) + 1
    mob = sim.ions[0][2]
    cases = [[(e_sp, 3, mob)],                     # the electrons are no ion
             [(len(plasma_iv) + 1, 3, mob)],        # no such species
             [(sim.ions[0][0], sim.f_flux, mob)],   # the electrons' flux variable
             [(sim.ions[0][0], 99, mob)],           # no such face variable
             [sim.ions[0]] * (capi.MAX_IONS + 1)]   # too many
    for ions in cases:
        with pytest.raises(capi.AfhError):
            Fluid(sim.tree, plasma_iv, [sim.species_charge[n] for n in sim.plasma],
                  sim.i_electron, sim.i_efld, sim.f_flux, sim.f_field, sim.N, sim.td,
                  sim.chem, sim.reactions, ions=ions)
    del c


def test_oracle_refuses_bad_ion_lists():
    bad_ion_fluids(capi.oracle_library())


def test_case_declares_three_mobile_ions():
    sim = Simulation(capi.oracle_library(), golden.load("case_ions"))
    assert len(sim.ions) == 3
    names = [sim.species_list[sim.plasma[sp - 1]] for sp, _, _ in sim.ions]
    assert names == ["N2+", "O2+", "O2-"] or names == ["N2_plus", "O2_plus", "O2_min"], names


def test_cases_without_mobile_ions():
    """Cases exported before the flux-species fields (and configs without
    mobile ions) give an electrons-only fluid."""
    for name in ("rtest_test_3d", "case_s3"):
        sim = Simulation(capi.oracle_library(), golden.load(name))
        assert sim.ions == []


@pytest.mark.gpu
def test_hip_refuses_bad_ion_lists():
    bad_ion_fluids(capi.hip_library(), device=0)


@pytest.mark.gpu
def test_hip_mobile_ions_equal_oracle():
    sim = Simulation(capi.hip_library(), golden.load("case_ions"), device=0)
    sim.start()
    for _ in range(3):
        sim.step()
    osim = sim.clone(capi.oracle_library())
    x = [s.fluid.forward_euler(1e-12, 0, [0], [1.0], 1, False) for s in (sim, osim)]
    assert list(x[0])[:2] == list(x[1])[:2]
    leaves = np.array(sim.af.leaves()) - 1
    for fv in [sim.f_flux] + [q[1] for q in sim.ions]:
        a, b = sim.tree.get_fc(fv)[leaves], osim.tree.get_fc(fv)[leaves]
        assert np.array_equal(a, b), fv
        assert np.max(np.abs(a)) > 0
    # the densities: the rate forms with exp (air_chemistry_small_v1: O- + O2
    # + M -> O3- + M, c1 exp(-(Td/c2)^2)) may differ in the last ulp
    for iv in sim.densities:
        a, b = sim.tree.get_cc(iv + 1), osim.tree.get_cc(iv + 1)
        assert np.max(np.abs(a - b)) <= 1e-13 * np.max(np.abs(b)), sim.cc_names[iv - 1]
    y = [s.fluid.forward_euler(5e-13, 1, [0, 1], [0.5, 0.5], 0, True) for s in (sim, osim)]
    assert np.allclose(list(y[0]), list(y[1]), rtol=1e-12, atol=0)
    for iv in sim.densities:
        a, b = sim.tree.get_cc(iv), osim.tree.get_cc(iv)
        assert np.max(np.abs(a - b)) <= 1e-12 * np.max(np.abs(b)), sim.cc_names[iv - 1]


@pytest.mark.gpu
def test_hip_ion_se_equal_oracle():
    """Secondary emission from ions at the walls (input_data%ion_se_yield =
    0.5; handle_ion_se_flux, m_fluid.f90:584-663, the oracle pinned to the
    reference by tests/test_reference_replay.py::
    test_species_step_replay_ion_se): the HIP driver's state after three
    steps, handed to the oracle; Heun stage 1's face fluxes (the electrons'
    with the emission) and CFL / dielectric limits bitwise, the densities to
    1e-13 (exp in the rate forms)."""
    g = dict(golden.load("case_ions"))
    g["ion_se_yield"] = np.array([0.5])
    sim = Simulation(capi.hip_library(), g, device=0)
    sim.start()
    for _ in range(3):
        sim.step()
    osim = sim.clone(capi.oracle_library())
    x = [s.fluid.forward_euler(1e-12, 0, [0], [1.0], 1, False) for s in (sim, osim)]
    assert list(x[0])[:2] == list(x[1])[:2]
    leaves = np.array(sim.af.leaves()) - 1
    for fv in [sim.f_flux] + [q[1] for q in sim.ions]:
        assert np.array_equal(sim.tree.get_fc(fv)[leaves], osim.tree.get_fc(fv)[leaves]), fv
    for iv in sim.densities:
        a, b = sim.tree.get_cc(iv + 1), osim.tree.get_cc(iv + 1)
        assert np.max(np.abs(a - b)) <= 1e-13 * np.max(np.abs(b)), sim.cc_names[iv - 1]
