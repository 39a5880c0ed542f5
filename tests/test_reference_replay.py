"""The device driver's ingredients replayed through the reference's own code.

Build-container only (needs /root/reference and the oracle/_ref programs that
oracle/Makefile compiles from it; skipped elsewhere, e.g. on the GPU box):

* refinement: every af_adjust_refinement call of a regression run
  (default_refinement evaluated on the device data, afh.amr's topology) is
  replayed by oracle/_ref/replay_refine, which loads the same electron
  density and |E| into a tree built by the reference and calls the
  reference's af_adjust_refinement with refine_routine => default_refinement
  (m_af_core.f90:697-822, src/m_refine.f90:198-298); the resulting
  topology must be ours, box id for box id, after every call;
* species step: the state before a forward-Euler sub-step of a regression
  run is handed to oracle/_ref/replay_step, which runs the reference's
  forward_euler (src/m_fluid.f90:21-99: flux_upwind_tree with flux_upwind /
  flux_direction, flux_update_densities with add_source_terms, get_rates,
  get_derivatives and the photoionization source) on it; the new densities
  and dt_lim must equal the C oracle's bitwise (the HIP library equals the
  oracle bitwise in the -m gpu tests).
"""
import os
import resource
import struct
import subprocess

import numpy as np
import pytest

import golden
from afh import capi
from afh.driver import Simulation

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_TESTS = "/root/reference/programs/standard_3d/tests"
REPLAY_REFINE = os.path.join(REPO, "oracle", "_ref", "replay_refine")
REPLAY_STEP = os.path.join(REPO, "oracle", "_ref", "replay_step")

pytestmark = pytest.mark.skipif(
    not (os.path.isdir(REF_TESTS) and os.path.exists(REPLAY_REFINE)
         and os.path.exists(REPLAY_STEP)),
    reason="needs the reference sources and oracle/_ref (build container)")


def _run_ref(exe, args, name, cwd=REF_TESTS):
    def unlimited_stack():
        resource.setrlimit(resource.RLIMIT_STACK,
                           (resource.RLIM_INFINITY, resource.RLIM_INFINITY))
    env = dict(os.environ, OMP_STACKSIZE="512M", OMP_NUM_THREADS="4")
    subprocess.run([exe] + args[:2] + [name + ".cfg"] + args[2:], cwd=cwd, check=True,
                   stdout=subprocess.DEVNULL, preexec_fn=unlimited_stack, env=env)


def _replay_refinements(name, tmp_path, full_calls=()):
    """Record every af_adjust_refinement call of the regression run `name`
    (the electron density and |E|; the whole state for the calls in
    full_calls), replay them through the reference and compare the
    topologies; returns [(our new boxes' data, the reference's)] of the full
    calls."""
    sim = Simulation(capi.oracle_library(), golden.load("rtest_" + name))
    rec, topo, ours = tmp_path / "rec.bin", [], []
    f = open(rec, "wb")
    f.write(struct.pack("<i", 0))
    n_calls = [0]
    changed = []
    orig = sim.adjust_refinement

    def recorded():
        af = sim.af
        full = n_calls[0] in full_calls
        f.write(struct.pack("<idi", af.highest_id, sim.global_time, int(full)))
        if full:
            cc = [sim.tree.get_cc(iv) for iv in range(1, sim.n_var_cell + 1)]
        else:
            e = sim.tree.get_cc(sim.i_electron)[:, 1:-1, 1:-1, 1:-1]
            E = sim.tree.get_cc(sim.i_efld)[:, 1:-1, 1:-1, 1:-1]
        for b in range(1, af.highest_id + 1):
            f.write(struct.pack("<i", int(af.in_use[b])))
            if af.in_use[b] and full:
                f.write(np.ascontiguousarray(np.stack([c[b - 1] for c in cc])).tobytes())
            elif af.in_use[b]:
                f.write(np.ascontiguousarray(e[b - 1]).tobytes())
                f.write(np.ascontiguousarray(E[b - 1]).tobytes())
        info = orig()
        if info.n_add or info.n_rm:
            changed.append(n_calls[0])
        topo.append((af.highest_id, [(int(af.in_use[b]), af.lvl[b], af.parent[b],
                                      list(af.children[b]) if af.in_use[b] else None)
                                     for b in range(1, af.highest_id + 1)]))
        if full:
            ours.append([sim.tree.get_cc(iv) for iv in range(1, sim.n_var_cell + 1)])
        n_calls[0] += 1
        return info

    sim.adjust_refinement = recorded
    sim.run()
    f.seek(0)
    f.write(struct.pack("<i", n_calls[0]))
    f.close()
    out = tmp_path / "rep.bin"
    _run_ref(REPLAY_REFINE, [str(rec), str(out)], name)
    raw, p = out.read_bytes(), 0
    ng = sim.af.nc + 2
    pairs = []
    for k, (hid, boxes) in enumerate(topo):
        rhid, _ = struct.unpack_from("<ii", raw, p)
        p += 8
        rows = np.frombuffer(raw, np.int32, rhid * 20, p).reshape(rhid, 20)
        p += rhid * 80
        assert rhid == hid, (k, rhid, hid)
        for b, (use, lvl, parent, children) in enumerate(boxes):
            assert rows[b, 0] == use, (k, b + 1)
            if use:
                assert (rows[b, 1], rows[b, 5]) == (lvl, parent), (k, b + 1)
                assert list(rows[b, 6:14]) == children, (k, b + 1)
        if k in full_calls:
            n_auto = struct.unpack_from("<i", raw, p)[0]
            auto = np.frombuffer(raw, np.int32, n_auto, p + 4)
            p += 4 * (n_auto + 1)
            n_add = struct.unpack_from("<i", raw, p)[0]
            p += 4
            mine = ours[full_calls.index(k)]
            for _ in range(n_add):
                bid = struct.unpack_from("<i", raw, p)[0]
                box = np.frombuffer(raw, np.float64, sim.n_var_cell * ng ** 3, p + 4)
                p += 4 + 8 * sim.n_var_cell * ng ** 3
                box = box.reshape(sim.n_var_cell, ng, ng, ng)
                for iv in auto:
                    pairs.append(((k, bid, sim.cc_names[iv - 1]), mine[iv - 1][bid - 1],
                                  box[iv - 1]))
    return n_calls[0], changed, pairs


@pytest.mark.parametrize("name", ["test_3d", "test_3d_chem"])
def test_refinement_replay(name, tmp_path):
    n_calls, _, _ = _replay_refinements(name, tmp_path)
    assert n_calls > 40


def test_regrid_data_replay(tmp_path):
    """The data af_adjust_refinement moves (auto_prolong into the new boxes:
    every auto variable -- the densities with af_prolong_limit, phi, |E| and
    the others with af_prolong_linear -- and the ghost cells of the new
    boxes, m_af_core.f90:842-881), replayed through the reference at the
    first three regrids of test_3d that add boxes: bitwise ours, ghost cells
    included. (Round 2's driver left phi out of the auto variables; the
    field solve after a regrid then started from phi = 0 in the new boxes.)"""
    _, changed, _ = _replay_refinements("test_3d", tmp_path)
    assert len(changed) >= 3
    _, _, pairs = _replay_refinements("test_3d", tmp_path, tuple(changed[:3]))
    names = {key[2] for key, _, _ in pairs}
    assert "phi" in names and "electric_fld" in names, names
    for key, mine, theirs in pairs:
        assert np.array_equal(mine, theirs), (key, np.max(np.abs(mine - theirs)))


def _replay_state(sim, name, s_deriv, s_prev, w_prev, s_out, dt, tmp_path, cwd=REF_TESTS,
                  cfg_args=None):
    """Hand the state of `sim` to oracle/_ref/replay_step (the reference's
    forward_euler) and compare its new densities and dt_lim with the oracle's."""
    if sim.photoi:
        sim.photoi_set_src()
    t, af = sim.tree, sim.af
    if sim.faces_from_phi:
        # our flux forms the face field from phi; the reference's
        # forward_euler reads the stored one (the same values)
        sim.mg.compute_phi_gradient(sim.f_field, -1.0, 0)
    hid = af.highest_id
    used = [b for b in range(1, hid + 1) if af.in_use[b]]
    rec = tmp_path / "step.bin"
    with open(rec, "wb") as f:
        f.write(struct.pack("<4i", hid, sim.n_var_cell, sim.n_var_face, af.nc))
        for b in range(1, hid + 1):
            ix = af.ix[b] if af.in_use[b] else (0, 0, 0)
            f.write(struct.pack("<6i", af.parent[b], af.lvl[b], *ix, int(af.in_use[b])))
        f.write(struct.pack("<ddii", dt, sim.time, s_deriv, len(s_prev)))
        f.write(struct.pack("<%di" % len(s_prev), *s_prev))
        f.write(struct.pack("<%dd" % len(w_prev), *w_prev))
        f.write(struct.pack("<i", s_out))
        for iv in range(1, sim.n_var_cell + 1):
            a = t.get_cc(iv)
            for b in used:
                f.write(np.ascontiguousarray(a[b - 1]).tobytes())
        for iv in range(1, sim.n_var_face + 1):
            a = t.get_fc(iv)
            for b in used:
                f.write(np.ascontiguousarray(a[b - 1]).tobytes())
    out = tmp_path / "out.bin"
    args = cfg_args or [name + ".cfg"]
    _run_ref(REPLAY_STEP, [str(rec), str(out)] + args[1:], args[0].replace(".cfg", ""),
             cwd=cwd)
    lim = sim.fluid.forward_euler(dt, s_deriv, s_prev, w_prev, s_out, True)
    ours = min(sim.dt_max, min(lim[0] * sim.cfl, lim[1], lim[2], lim[3]))
    raw = out.read_bytes()
    assert struct.unpack_from("<d", raw, 0)[0] == ours
    ng = af.nc + 2
    ref = np.frombuffer(raw, np.float64, offset=8).reshape(
        sim.n_var_cell, len(used), ng, ng, ng)
    leaves = set(af.leaves())
    li = [k for k, b in enumerate(used) if b in leaves]
    for iv in sim.densities:
        mine = t.get_cc(iv + s_out)[np.array(used) - 1][li][:, 1:-1, 1:-1, 1:-1]
        theirs = ref[iv + s_out - 1][li][:, 1:-1, 1:-1, 1:-1]
        assert np.array_equal(mine, theirs), sim.cc_names[iv - 1]


def replay_species_step(name, n_steps, s_deriv, s_prev, w_prev, s_out, dt, tmp_path):
    sim = Simulation(capi.oracle_library(), golden.load("rtest_" + name))
    sim.start()
    while sim.it < n_steps:
        sim.step()
    _replay_state(sim, name, s_deriv, s_prev, w_prev, s_out, dt, tmp_path)


@pytest.mark.parametrize("name", ["test_3d", "test_3d_chem", "test_3d_photoi_chem"])
def test_species_step_replay(name, tmp_path):
    # Heun stage 1 on the AMR tree after 5 steps, stage 2 after 40 (the second
    # with the photoionization source of that step)
    replay_species_step(name, 5, 0, [0], [1.0], 1, 1e-11, tmp_path)
    replay_species_step(name, 40, 1, [0, 1], [0.5, 0.5], 0, 2e-11, tmp_path)


def test_species_step_replay_s3(tmp_path):
    """BASELINE config 3 (streamer_3d.cfg + air_chemistry_v2: 9 species, 25
    reactions) on the 10-level AMR tree set_initial_conditions builds: one
    species step bitwise equal to the reference's forward_euler."""
    from afh.driver import Simulation as Sim
    sim = Sim(capi.oracle_library(), golden.load("case_s3"))
    sim.set_initial_conditions()
    _replay_state(sim, "s3", 0, [0], [1.0], 1, 1e-12, tmp_path,
                  cwd="/root/reference/programs/standard_3d",
                  cfg_args=["streamer_3d.cfg",
                            "-input_data%file=../../transport_data/air_chemistry_v2.txt",
                            "-input_data%old_style=f"])


def test_species_step_replay_s5(tmp_path):
    """BASELINE config 5 (programs/3d_sprite/sprite_3d.cfg: sprite_chemistry_v0,
    Helmholtz photoionization, the exponential atmosphere of its m_user.f90 as
    the gas density variable "M"): after the initial refinement and three time
    steps, Heun stages 1 and 2 -- with the photoionization source -- bitwise
    equal to the reference's forward_euler with a variable gas density (1/N
    per face, E/N and gas species densities per cell)."""
    from afh.driver import Simulation as Sim
    from afh.users import Sprite3D
    sim = Sim(capi.oracle_library(), golden.load("case_s5"), user=Sprite3D)
    sim.start()
    for _ in range(3):
        sim.step()
    args = ["sprite_3d.cfg", "--user-gas=sprite"]
    cwd = "/root/reference/programs/3d_sprite"
    _replay_state(sim, "s5", 0, [0], [1.0], 1, 1e-12, tmp_path, cwd=cwd, cfg_args=args)
    _replay_state(sim, "s5", 1, [0, 1], [0.5, 0.5], 0, 5e-13, tmp_path, cwd=cwd,
                  cfg_args=args)


ION_ARGS = ["test_3d_chem.cfg", "-input_data%mobile_ions=N2_plus O2_plus O2_min",
            "-input_data%ion_mobilities=1e-2 2e-2 1.5e-2"]


def test_species_step_replay_mobile_ions(tmp_path):
    """Mobile ions (input_data%mobile_ions / ion_mobilities; flux species 2..
    of m_streamer.f90:253-282, their fluxes in m_fluid.f90:207-214): test_3d_chem
    with N2+, O2+ and O2- mobile (tests/golden/case_ions.npz, oracle/
    make_cases.py). After the initial refinement and three time steps, Heun
    stages 1 and 2 bitwise equal to the reference's forward_euler: every
    density -- the ions' now with their flux divergence -- and dt_lim, whose
    dielectric relaxation term sums the ions' mu u with the electrons' per
    face."""
    sim = Simulation(capi.oracle_library(), golden.load("case_ions"))
    assert [q[1] for q in sim.ions] == [3, 4, 5]
    sim.start()
    for _ in range(3):
        sim.step()
    _replay_state(sim, "ions", 0, [0], [1.0], 1, 1e-12, tmp_path, cfg_args=ION_ARGS)
    _replay_state(sim, "ions", 1, [0, 1], [0.5, 0.5], 0, 5e-13, tmp_path,
                  cfg_args=ION_ARGS)


def test_species_step_replay_ion_se(tmp_path):
    """Secondary emission from ions at the walls (input_data%ion_se_yield;
    handle_ion_se_flux, src/m_fluid.f90:584-663, called by forward_euler
    between the flux and the update, 63-67): the mobile-ion case with a yield
    of 0.5 (the two positive ions' wall fluxes feed the electrons'). Heun
    stages 1 and 2 bitwise the reference's forward_euler; the yield changes
    the densities (the emission is not vacuous here)."""
    g = dict(golden.load("case_ions"))
    g["ion_se_yield"] = np.array([0.5])
    args = ION_ARGS + ["-input_data%ion_se_yield=0.5"]
    sims = []
    for case in (g, golden.load("case_ions")):
        sim = Simulation(capi.oracle_library(), case)
        sim.start()
        for _ in range(3):
            sim.step()
        sims.append(sim)
    e = sims[0].species_itree[sims[0].plasma[0]]
    assert not np.array_equal(sims[0].tree.get_cc(e), sims[1].tree.get_cc(e))
    _replay_state(sims[0], "ions", 0, [0], [1.0], 1, 1e-12, tmp_path, cfg_args=args)
    _replay_state(sims[0], "ions", 1, [0, 1], [0.5, 0.5], 0, 5e-13, tmp_path, cfg_args=args)


S4_ARGS = ["streamer_3d.cfg", "-input_data%file=../../transport_data/air_chemistry_v2.txt",
           "-input_data%old_style=f", "-use_electrode=T", "-field_electrode_grounded=T",
           "-field_rod_r0=0.5 0.5 0.0", "-field_rod_r1=0.5 0.5 0.15",
           "-field_rod_radius=1e-3", "-refine_electrode_dx=2e-4", "-refine_min_dx=1e-4"]


def test_species_step_replay_s4(tmp_path):
    """BASELINE config 4 (streamer_3d.cfg + air_chemistry_v2 + the grounded
    rod electrode): after the initial refinement and two time steps, Heun
    stages 1 and 2 bitwise equal to the reference's forward_euler -- whose
    flux_update_densities masks the cells inside the electrode (set_box_mask,
    src/m_fluid.f90:469-483: no sources, no flux divergence where lsf <= 0,
    and no chemistry time-step limit from boxes wholly inside)."""
    from afh.driver import Simulation as Sim
    sim = Sim(capi.oracle_library(), golden.load("case_s4"))
    sim.start()
    for _ in range(2):
        sim.step()
    cwd = "/root/reference/programs/standard_3d"
    _replay_state(sim, "s4", 0, [0], [1.0], 1, 1e-12, tmp_path, cwd=cwd, cfg_args=S4_ARGS)
    _replay_state(sim, "s4", 1, [0, 1], [0.5, 0.5], 0, 5e-13, tmp_path, cwd=cwd,
                  cfg_args=S4_ARGS)
