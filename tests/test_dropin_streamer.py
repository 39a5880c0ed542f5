"""The reference's streamer program itself through the shim (VERDICT r4
item 7).

oracle/_ref/dropin_streamer is src/streamer.f90 compiled from the reference
sources with four kinds of call rewritten by oracle/dropin_subst.py -- mg_init
(its HYPRE set-up skipped), field_compute, field_from_potential and the
forward_euler handed to af_advance -- to oracle/harness/m_dropin.f90, which
does their work through the ISO_C_BINDING shim (afivo-streamer_amd/fortran)
on the C oracle (libafo.so, the afo_ twin of libafivo_hip's entry points;
the level-1 solve is the PFMG restatement). Everything else is the
reference's own code on its own af_t tree: the set-up, the time loop with
its step control and rejected steps, af_adjust_refinement, the output and
output_regression_log.

Run on programs/standard_3d/tests/test_3d.cfg (3 ns, regrids every 2 steps),
its regression log is the committed test_3d_rtest.log row for row at the
log's print precision (compare_logs.py would allow rtol 1e-5), and within
1e-7 of afh.driver's rows on the oracle with the same level-1 solve
(tests/test_rtest.py: afh.driver restates the time loop in Python).
Build container only: the reference and the binary built from it are not on
the GPU box.
"""
import os
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(REPO, "oracle", "_ref", "dropin_streamer")
TESTS = "/root/reference/programs/standard_3d/tests"

pytestmark = pytest.mark.skipif(not (os.path.exists(EXE) and os.path.isdir(TESTS)),
                                reason="build container only (oracle/_ref/dropin_streamer)")


def test_streamer_program_through_shim_test_3d(tmp_path):
    env = dict(os.environ, OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "8"),
               OMP_STACKSIZE="512M")
    out = subprocess.run([EXE, os.path.join(TESTS, "test_3d.cfg"),
                          "-output%name=" + str(tmp_path / "test_3d"),
                          "-input_data%file=" + os.path.join(TESTS, "td_air_siglo_swarm.txt")],
                         cwd=tmp_path, env=env, capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    rows = np.loadtxt(tmp_path / "test_3d_rtest.log", skiprows=1)
    ref = np.loadtxt(os.path.join(TESTS, "test_3d_rtest.log"), skiprows=1)
    assert rows.shape == ref.shape
    rel = np.abs(rows - ref) / np.maximum(np.abs(ref), 1e-300)
    print("drop-in streamer vs test_3d_rtest.log, max rel per row", rel.max(axis=1))
    # the log's own print precision (E20.8: 5e-9 relative)
    assert rel.max() <= 1e-8, rel.max(axis=1)
    # and afh.driver's rows on the same library with the same level-1 solve
    import golden
    from afh import capi
    from afh.driver import Simulation
    sim = Simulation(capi.oracle_library(), golden.load("rtest_test_3d"), coarse_cycles=50,
                     coarse_tol=1e-6, coarse_mode=capi.COARSE_PFMG)
    drv = sim.run()
    assert drv.shape == rows.shape
    assert np.allclose(drv, rows, rtol=1e-7, atol=1e-8)


S4_CFG = ["streamer_3d.cfg", "-input_data%file=../../transport_data/air_chemistry_v2.txt",
          "-input_data%old_style=f", "-use_electrode=T", "-field_electrode_grounded=T",
          "-field_rod_r0=0.5 0.5 0.0", "-field_rod_r1=0.5 0.5 0.15",
          "-field_rod_radius=1e-3", "-refine_electrode_dx=2e-4", "-refine_min_dx=1e-4"]


def run_dropin_s4(tmp_path, end_time, output_dt):
    """The reference's streamer program on BASELINE config 4 (streamer_3d.cfg
    with the grounded rod electrode) through the shim on the C oracle:
    mg_use's level-set stencils handed over per solve, set_box_mask in the
    update, the reference's own set_electrode_densities. Returns its
    regression-log rows."""
    env = dict(os.environ, OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "8"),
               OMP_STACKSIZE="512M")
    cwd = os.path.dirname(TESTS)  # programs/standard_3d
    out = subprocess.run([EXE] + S4_CFG + ["-output%name=" + str(tmp_path / "s4"),
                                           "-output%regression_test=T", "-silo_write=f",
                                           "-end_time=" + repr(end_time),
                                           "-output%dt=" + repr(output_dt)],
                         cwd=cwd, env=env, capture_output=True, text=True, timeout=1800)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    return np.loadtxt(tmp_path / "s4_rtest.log", skiprows=1, ndmin=2)


def test_streamer_program_through_shim_s4(tmp_path):
    """Config 4's time loop driven by the reference's own streamer.f90
    (round 6) against afh.driver's restatement of it on the
    same library: every regression-log row (it, time, dt, the species' sums
    and maxima) within 1e-7 over the first 40 ps (~80 steps, with regrids),
    as for test_3d above."""
    end_time, output_dt = 4e-11, 1e-11
    rows = run_dropin_s4(tmp_path, end_time, output_dt)
    import golden
    from afh import capi
    from afh.driver import Simulation
    g = dict(golden.load("case_s4"))
    g["end_time"] = np.array([end_time])
    g["output%dt"] = np.array([output_dt])
    sim = Simulation(capi.oracle_library(), g, coarse_cycles=50, coarse_tol=1e-6,
                     coarse_mode=capi.COARSE_PFMG)
    drv = sim.run()
    assert drv.shape == rows.shape, (drv.shape, rows.shape)
    rel = np.abs(drv - rows) / np.maximum(np.abs(rows), 1e-300)
    print("afh.driver vs the reference's streamer (s4), max rel per row", rel.max(axis=1))
    assert np.allclose(drv, rows, rtol=1e-7, atol=1e-8)
