"""Deferred reductions (afh_mg_fas_vcycle_fold, afh_fluid_forward_euler_fold,
afh_fluid_fetch_step, afh_tree_fetch_reduced): the maxima and limits a step
folds on the device are read in one transfer at the end instead of one
transfer per reduction. The results -- residuals, time-step limits, every
variable -- are bitwise those of the immediate reads (AFH_DEFER=0):

* the bench's unit step (bench.unit_step: field_compute with one V-cycle,
  whose residual comes back with the species step's limits);
* the driver's field_compute (src/m_field.f90:405-485), which reads max|rhs|
  of the fused rhs output together with the first V-cycle's residual;
* sharded (thread ranks), where the fetch reduces over the ranks.

The C oracle's twin of the entry points on the CPU; libafivo_hip on the GPU
(config 2 / S1 and config 3 / S3 at full size); libafivo_hip_2d's on config
1's bench tree.
"""
import numpy as np
import pytest

import golden
from afh import capi


def _unit_steps(lib, monkeypatch, defer, config, device, n=4):
    import bench
    monkeypatch.setenv("AFH_DEFER", "1" if defer else "0")
    c = bench.build_case(lib, config, device, 0)
    if c.ndim == 3:
        c.fuse_rhs(True, ghosts=False)
    out = [c.field_compute(0, n_vcycles=2)]
    for k in range(n):
        res, lim = bench.unit_step(c, 1e-13, k)
        # a Heun step's first sub-step fetches nothing (its limits are never
        # read, m_af_advance.f90:160-164): its V-cycle residual stays on the
        # device when deferred
        out.append((res if k % 2 else None, lim))
    state = [c.tree.get_cc(iv) for iv in range(1, c.tree.n_var_cell + 1)]
    c.tree.close()
    return out, state


def _driver_steps(lib, monkeypatch, defer, case, device, user=None, n=2):
    from afh.driver import Simulation
    from afh.users import USERS
    monkeypatch.setenv("AFH_DEFER", "1" if defer else "0")
    sim = Simulation(lib, golden.load(case), device=device, user=USERS.get(user))
    sim.start()
    lims = []
    for _ in range(n):
        if sim.photoi:
            sim.photoi_set_src()
        lims.append(sim.advance(2e-12))
        lims.append(tuple(sim.field_compute(0, True)))
    state = [sim.tree.get_cc(iv) for iv in range(1, sim.n_var_cell + 1)]
    return lims, state


def _same(a, b):
    assert a[0] == b[0], (a[0], b[0])
    for x, y in zip(a[1], b[1]):
        assert np.array_equal(x, y, equal_nan=True)


@pytest.fixture
def tiny(monkeypatch):
    import bench
    # 3 levels of 8^3 boxes, 512 leaves (S1's shape, a quarter of its cells)
    monkeypatch.setitem(bench.CONFIGS, "tiny", (8, (16, 16, 16), 3, (16e-3, 16e-3, 16e-3)))
    return "tiny"


def test_unit_step_deferred_oracle(monkeypatch, tiny):
    lib = capi.oracle_library()
    a = _unit_steps(lib, monkeypatch, True, tiny, -1)
    b = _unit_steps(lib, monkeypatch, False, tiny, -1)
    _same(a, b)
    # the deferred residual list was filled by the species step
    assert all(len(res) == 1 for res, _ in a[0][2::2])


def test_driver_deferred_oracle(monkeypatch):
    lib = capi.oracle_library()
    _same(_driver_steps(lib, monkeypatch, True, "rtest_test_3d_photoi_chem", -1),
          _driver_steps(lib, monkeypatch, False, "rtest_test_3d_photoi_chem", -1))


def test_fetch_slot_checks():
    """Only the |x| maxima are public slots; the limits go through
    fetch_step."""
    from afh.tree import uniform_tree
    from afh.model import Tree
    lib = capi.oracle_library()
    t = Tree(lib, uniform_tree(8, (8, 8, 8), (1.0, 1.0, 1.0), 1), 3, 0)
    with pytest.raises(capi.AfhError):
        t.fetch_reduced(capi.SLOT_MAXRES, 0)
    with pytest.raises(capi.AfhError):
        t.fetch_reduced(7)
    t.close()


@pytest.mark.gpu
def test_unit_step_deferred_s1(monkeypatch):
    lib = capi.hip_library()
    _same(_unit_steps(lib, monkeypatch, True, "s1", 0),
          _unit_steps(lib, monkeypatch, False, "s1", 0))


@pytest.mark.gpu
def test_driver_deferred_s3(monkeypatch):
    lib = capi.hip_library()
    _same(_driver_steps(lib, monkeypatch, True, "case_s3", 0),
          _driver_steps(lib, monkeypatch, False, "case_s3", 0))


@pytest.mark.gpu
def test_unit_step_deferred_2d(monkeypatch):
    """The 2-D build's deferred entry points (round 4) on config 1's bench
    tree: residuals, limits and every variable bitwise the immediate reads."""
    lib = capi.hip_library_2d()
    a = _unit_steps(lib, monkeypatch, True, "2d-uniform", 0)
    _same(a, _unit_steps(lib, monkeypatch, False, "2d-uniform", 0))
    assert all(len(res) == 1 for res, _ in a[0][2::2])
