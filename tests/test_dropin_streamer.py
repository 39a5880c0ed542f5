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
