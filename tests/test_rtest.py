"""End-to-end regression against the reference's own regression logs.

The reference's 3D regression tests (programs/standard_3d/tests/test_3d*.cfg,
run by run_test.sh and compared by tools/compare_logs.py with rtol 1e-5,
atol 1e-8) ran the whole streamer program and committed one log row per
output time (0.2 ns): it, time, dt and the volume-averaged sums of n, n^2 and
the maxima of every species (output_regression_log, src/m_output.f90:783-837).
afh.driver.Simulation reruns the same program -- set-up from the reference's
own initializers (tests/golden/rtest_*.npz, oracle/make_cases.py), AMR set-up,
3 ns of Heun steps with step control, regrids every 2 steps, Helmholtz
photoionization every 5 steps -- over the C oracle (CPU) and the HIP library
(GPU), and compares against those committed rows.

What is expected, and why:
* the reference's level-1 solve is HYPRE StructPFMG stopped at a relative
  residual of 1e-6 (afivo/src/m_coarse_solver.f90:393-439), and
  field_compute stops at a residual of 1e-4 max|rhs|, so the rows depend on
  the level-1 solver at the 1e-5 level (profiles/r03_rtest_coarse_sensitivity.json:
  other level-1 solves move them by up to 3e-5);
* with HYPRE's PFMG restated (round 5, AFH_COARSE_PFMG,
  afivo-streamer_amd/csrc/afh_pfmg.h) every row of all three logs matches
  within 5e-8 -- the logs' print precision (E20.8, src/m_output.f90:829) --
  so the bound is 1e-7, a hundred times tighter than compare_logs' 1e-5;
* with our exact level-1 solve (the bench's) the rows are within 4e-5.
Until round 3 the rows diverged by 1e-3 .. 2e-2 after 1.4 ns: the field
solve after the first regrid (level 6 created at step 46) started from
phi = 0 in the new boxes, because the driver did not make phi an auto
variable as mg_init does (m_af_multigrid.f90:102-105: af_set_cc_methods
without a prolongation method, so af_prolong_linear into every new box,
m_af_core.f90:387-391, 420-425, 842-881).
"""
import numpy as np
import pytest

import golden
from afh import capi
from afh.driver import Simulation

CASES = ["test_3d", "test_3d_chem", "test_3d_photoi_chem"]
# level-1 solves: (max cycles, tolerance, mode) -- our exact solve
# (AFH_COARSE_DIRECT), and the reference's HYPRE PFMG restated (50, 1e-6:
# the reference's settings, m_af_types.f90:560-565)
EXACT, PFMG = (0, 0.0, None), (50, 1e-6, capi.COARSE_PFMG)
# bound on every row's relative deviation from the reference, per level-1
# solve: PFMG 1e-7 (measured 4.8e-8, the print precision); exact: measured
# max + the coarse-solve spread, rounded up
BOUND = {("test_3d", PFMG): 1e-7, ("test_3d", EXACT): 2.5e-5,
         ("test_3d_chem", PFMG): 1e-7, ("test_3d_chem", EXACT): 5e-5,
         ("test_3d_photoi_chem", PFMG): 1e-7, ("test_3d_photoi_chem", EXACT): 5e-5}


def load(name):
    return golden.load("rtest_" + name)


def run(lib, name, device=-1, solve=EXACT):
    d = load(name)
    sim = Simulation(lib, d, device=device, coarse_cycles=solve[0], coarse_tol=solve[1],
                     coarse_mode=solve[2])
    return sim, sim.run(), d["rtest_log"]


def check_against_reference(name, log, ref, solve=EXACT):
    assert log.shape == ref.shape, (log.shape, ref.shape)
    # it and time columns exactly (output times are hit exactly)
    assert np.array_equal(log[:, 0], ref[:, 0])
    assert np.allclose(log[:, 1], ref[:, 1], rtol=1e-12, atol=0)
    # every row, compare_logs.py's atol 1e-8 and the case's rtol
    rtol = BOUND[(name, solve)]
    bad = ~np.isclose(log, ref, rtol=rtol, atol=1e-8)
    assert not bad.any(), (rtol, np.argwhere(bad)[:5],
                           np.max(np.abs(log - ref) / np.maximum(np.abs(ref), 1e-300)))


SOLVES = {"exact": EXACT, "pfmg": PFMG}


# (the CPU suite runs the chemistry cases with the reference's PFMG solve
# only; their exact-solve runs, 4 minutes of oracle time, run in the GPU
# suite's test_rtest_hip, which checks the oracle's rows too)
@pytest.mark.parametrize("name,solve", [(n, s) for s in sorted(SOLVES) for n in CASES
                                        if s != "exact" or n == "test_3d"])
def test_rtest_oracle(name, solve):
    _, log, ref = run(capi.oracle_library(), name, solve=SOLVES[solve])
    check_against_reference(name, log, ref, SOLVES[solve])


@pytest.mark.gpu
@pytest.mark.parametrize("solve", sorted(SOLVES))
@pytest.mark.parametrize("name", CASES)
def test_rtest_hip(name, solve):
    """The device time loop: the reference rows as above, and the oracle's
    rows (same algorithms on the CPU) to 1e-9."""
    sim, log, ref = run(capi.hip_library(), name, device=0, solve=SOLVES[solve])
    check_against_reference(name, log, ref, SOLVES[solve])
    _, olog, _ = run(capi.oracle_library(), name, solve=SOLVES[solve])
    rel = np.abs(log - olog) / np.maximum(np.abs(olog), 1e-300)
    assert rel.max() <= 1e-9, rel.max(axis=1)


@pytest.mark.gpu
def test_s3_hip_equals_oracle():
    """BASELINE config 3 (streamer_3d.cfg + air_chemistry_v2, the reference's
    set-up exported by oracle/_ref/export_case): the 10-level AMR tree
    set_initial_conditions builds on the device (8873 boxes of 8^3), then one
    Heun step (two forward_euler sub-steps, field solves included) on the HIP
    library and on the C oracle from the same state. The oracle's species
    step on this tree is bitwise the reference's forward_euler
    (test_reference_replay.test_species_step_replay_s3)."""
    sim = Simulation(capi.hip_library(), golden.load("case_s3"), device=0)
    sim.set_initial_conditions()
    assert sim.af.highest_lvl >= 5 and len(sim.af.leaves()) > 1000
    osim = sim.clone(capi.oracle_library())
    for s in (sim, osim):
        s.advance(1e-12)
        s.field_compute(0, True)
    for iv in list(sim.densities) + [sim.i_phi, sim.i_efld]:
        a, b = sim.tree.get_cc(iv), osim.tree.get_cc(iv)
        rel = np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300)
        assert rel <= 1e-12, (sim.cc_names[iv - 1], rel)


@pytest.mark.gpu
def test_s3_species_step_hip_equals_oracle():
    """One forward_euler species step (flux + air_chemistry_v2 update, both
    Heun stages) on the S3 tree, HIP against the C oracle (whose step is the
    reference's forward_euler bitwise, test_reference_replay): the fluxes and
    dt limits bitwise; the densities to 1e-13 relative -- the temperature
    forms of air_chemistry_v2 call pow / exp, whose device (ocml) and host
    (glibc) results may differ in the last ulp."""
    sim = Simulation(capi.hip_library(), golden.load("case_s3"), device=0)
    sim.set_initial_conditions()
    osim = sim.clone(capi.oracle_library())
    lims = []
    for s in (sim, osim):
        a = s.fluid.forward_euler(1e-12, 0, [0], [1.0], 1, False)
        b = s.fluid.forward_euler(5e-13, 1, [0, 1], [0.5, 0.5], 0, True)
        lims.append((list(a), list(b)))
    assert lims[0][0][:2] == lims[1][0][:2] and lims[0][1][:2] == lims[1][1][:2]
    assert np.allclose(lims[0][1], lims[1][1], rtol=1e-13, atol=0)
    for iv in range(1, sim.n_var_face + 1):
        assert np.array_equal(sim.tree.get_fc(iv), osim.tree.get_fc(iv))
    for iv in sim.densities:
        for st in (0, 1):
            a, b = sim.tree.get_cc(iv + st), osim.tree.get_cc(iv + st)
            rel = np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300)
            assert rel <= 1e-13, (sim.cc_names[iv + st - 1], rel)


@pytest.mark.gpu
def test_s5_sprite_hip_equals_oracle():
    """BASELINE config 5 (sprite_3d.cfg: variable gas density, sprite
    chemistry, Helmholtz photoionization) on the device driver: after the
    initial refinement and three steps on the GPU, the same state on the C
    oracle (whose species step is the reference's forward_euler bitwise,
    test_reference_replay) -- the photoionization source to 1e-12; Heun
    stage 1 with fluxes and CFL / dielectric limits bitwise, stage 2 (on
    stage-1 densities that may differ in the last ulp: exp in the rate forms,
    ocml vs glibc) to 1e-12, densities to 1e-12; the refinement flags (E/N
    per cell) equal."""
    from afh.users import Sprite3D
    sim = Simulation(capi.hip_library(), golden.load("case_s5"), device=0, user=Sprite3D)
    sim.start()
    for _ in range(3):
        sim.step()
    assert sim.af.highest_lvl >= 6
    osim = sim.clone(capi.oracle_library())
    for s in (sim, osim):
        s.photoi_set_src()
    a, b = sim.tree.get_cc(sim.i_photo), osim.tree.get_cc(osim.i_photo)
    assert np.max(np.abs(a - b)) <= 1e-12 * np.max(np.abs(b))
    x = [s.fluid.forward_euler(1e-12, 0, [0], [1.0], 1, False) for s in (sim, osim)]
    assert list(x[0])[:2] == list(x[1])[:2]
    for iv in range(1, sim.n_var_face + 1):  # stage 1 reads state 0: identical inputs
        assert np.array_equal(sim.tree.get_fc(iv), osim.tree.get_fc(iv))
    # stage 2 reads state 1, whose densities may differ in the last ulp
    y = [s.fluid.forward_euler(5e-13, 1, [0, 1], [0.5, 0.5], 0, True) for s in (sim, osim)]
    assert np.allclose(list(y[0]), list(y[1]), rtol=1e-12, atol=0)
    for iv in range(1, sim.n_var_face + 1):
        a, b = sim.tree.get_fc(iv), osim.tree.get_fc(iv)
        assert np.max(np.abs(a - b)) <= 1e-12 * np.max(np.abs(b))
    for iv in sim.densities:
        for st in (0, 1):
            a, b = sim.tree.get_cc(iv + st), osim.tree.get_cc(iv + st)
            rel = np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300)
            assert rel <= 1e-12, (sim.cc_names[iv + st - 1], rel)
    fa = sim.fluid.refine_flags(sim.refine_desc())
    fb = osim.fluid.refine_flags(osim.refine_desc())
    assert np.array_equal(fa[0], fb[0]) and np.array_equal(fa[1], fb[1])


def _s4_checks(sim):
    """The electrode of config 4 as the set-up leaves it: boxes tagged,
    a grounded rod (phi ~ 0 inside it, leaf interiors), refined to
    refine_electrode_dx around it."""
    assert len(sim.electrode_ids) > 10
    lsf, phi = sim.tree.get_cc(sim.i_lsf), sim.tree.get_cc(sim.i_phi)
    inner = (slice(None),) + (slice(1, -1),) * 3
    leaves = np.asarray(sim.af.leaves()) - 1
    li, lp = lsf[leaves][inner], phi[leaves][inner]
    assert np.max(np.abs(lp[li < 0])) < 1e-3 * abs(sim.voltage)
    assert np.min(lp[li > 0]) > -1e-3 * abs(sim.voltage)
    dx = min(float(np.max(sim.af.dr[b])) for b in sim.electrode_ids if b - 1 in set(leaves))
    assert dx <= sim.c.r("refine_electrode_dx")


def test_s4_electrode_oracle():
    """BASELINE config 4 on one device (streamer_3d.cfg + air_chemistry_v2
    with the grounded rod of SURVEY 8(d) S4, exported by oracle/make_cases.py)
    through the driver on the C oracle: the host electrode operators
    (afh.electrode, pinned to the reference's own stencils in
    test_electrode_ops) in the set-up's field solves and two time steps."""
    sim = Simulation(capi.oracle_library(), golden.load("case_s4"))
    sim.start()
    _s4_checks(sim)
    for _ in range(2):
        sim.step()
    assert np.all(np.isfinite(sim.log[-1]))


@pytest.mark.gpu
def test_s4_electrode_hip_equals_oracle():
    """Config 4 on the GPU: the set-up (electrode field solves on the device,
    level-set stencils, electrode refinement) on the HIP library, then the
    same state on the C oracle; two Heun steps with electrode_species_bc
    and field solves through the electrode stencils on both: densities,
    potential and field to 1e-12 relative (the air_chemistry_v2 rate forms'
    pow / exp may differ in the last ulp between ocml and glibc), the
    refinement flags equal."""
    sim = Simulation(capi.hip_library(), golden.load("case_s4"), device=0)
    sim.start()
    _s4_checks(sim)
    osim = sim.clone(capi.oracle_library())
    for s in (sim, osim):
        s.fluid.electrode_species_bc(s.i_lsf, s.i_1pos_ion, s.electrode_ids, True)
        s.advance(1e-12)
        s.field_compute(0, True)
    for iv in list(sim.densities) + [sim.i_phi, sim.i_efld]:
        a, b = sim.tree.get_cc(iv), osim.tree.get_cc(iv)
        rel = np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300)
        assert rel <= 1e-12, (sim.cc_names[iv - 1], rel)
    fa = sim.fluid.refine_flags(sim.refine_desc(), sim.electrode_box)
    fb = osim.fluid.refine_flags(osim.refine_desc(), osim.electrode_box)
    assert np.array_equal(fa[0], fb[0]) and np.array_equal(fa[1], fb[1])
