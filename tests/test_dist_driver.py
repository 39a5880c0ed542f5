"""The device driver's AMR configurations sharded over ranks
(Simulation.shard_over, afh_dist_*): after the single-rank set-up (the
initial refinement of the reference's set_initial_conditions), the state is
split over 2 or 3 ranks -- threads of one process, AFH_DIST_LOCAL -- and
time steps run sharded: photoionization source (Helmholtz FMGs), electrode
species boundary condition, two Heun sub-steps with their field solves, the
final field solve. The boxes every rank computes, gathered, equal the
single-rank run bitwise, and so do the time-step limits.

Cases: the regression test with Helmholtz photoionization and chemistry
(test_3d_photoi_chem), BASELINE config 4's rod electrode (level-set
stencils, electrode coarse solve) and config 5's sprite (variable gas
density, photoionization; level-1 leaves next to refined level-1 boxes, so
the consistent fluxes of replicated coarse leaves come from the ranks that
own the fine children). The C oracle's CPU twin here; libafivo_hip on
the GPU.
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import golden
from afh import capi
from afh.dist import NativeGroup, NativeShard
from afh.driver import Simulation

CASES = {"photoi_chem": ("rtest_test_3d_photoi_chem", None),
         "s4_rod": ("case_s4", None), "s5_sprite": ("case_s5", "s5")}


def _steps(sim, n=2):
    lims = []
    for k in range(n):
        if sim.photoi:
            sim.photoi_set_src()
        if sim.lsf is not None:
            sim.fluid.electrode_species_bc(sim.i_lsf, sim.i_1pos_ion, sim.electrode_ids,
                                           sim.c.s("species_boundary_condition") ==
                                           "neumann_zero")
        lims.append(sim.advance(2e-12))
        lims.append(tuple(sim.field_compute(0, True)))
    return lims


def _run(lib, name, world, device=-1):
    from afh.users import USERS
    case, user = CASES[name]
    base = Simulation(lib, golden.load(case), device=device, user=USERS.get(user))
    base.start()
    clones = [base.clone(lib, device=device) for _ in range(world)]
    ref = _steps(base)
    topo = base.af.topology()
    group = NativeGroup(lib, world)
    shards = [NativeShard(lib, topo, world, r, group=group) for r in range(world)]
    for sim, sh in zip(clones, shards):
        sim.shard_over(sh)
    assert shards[0].lp is not None
    if world == 8:  # a mixed frontier: some level holds replicated and owned boxes
        o = shards[0].owner
        lv = base.af.topology()["meta_lvl"]
        assert any((o[lv == l] < 0).any() and (o[lv == l] >= 0).any()
                   for l in range(2, base.af.highest_lvl + 1))
    owned = [int(np.sum(sh.owner == r)) for r, sh in enumerate(shards)]
    assert min(owned) > 0, owned
    try:
        with ThreadPoolExecutor(world) as ex:
            outs = list(ex.map(_steps, clones))
        assert all(sh.n_exchanges > 0 for sh in shards)
    finally:
        for sim, sh in zip(clones, shards):
            sh.detach()
        group.close()
    for o in outs:
        assert o == ref, (o, ref)
    for iv in range(1, base.n_var_cell + 1):
        want = base.tree.get_cc(iv)
        got = np.full_like(want, np.nan)
        for sim, sh in zip(clones, shards):
            mine = sh.owned_mask()
            got[mine] = sim.tree.get_cc(iv)[mine]
        used = np.array([base.af.in_use[b] for b in range(1, len(want) + 1)], bool)
        assert np.array_equal(got[used], want[used]), (base.cc_names[iv - 1],
                                                       np.nanmax(np.abs(got[used] - want[used])))


@pytest.mark.parametrize("name,world", [("photoi_chem", 2), ("s4_rod", 2), ("s5_sprite", 2),
                                        ("s5_sprite", 8), ("s4_rod", 8)])
def test_sharded_driver_oracle_threads_bitwise(name, world):
    # 8 ranks: the partition frontier spans several levels (replicated
    # parents next to owned boxes of the same level, owned boxes restricted
    # into replicated parents on several levels)
    _run(capi.oracle_library(), name, world)


@pytest.mark.gpu
@pytest.mark.parametrize("name,world", [("photoi_chem", 2), ("photoi_chem", 3),
                                        ("s4_rod", 2), ("s5_sprite", 2), ("s5_sprite", 8)])
def test_sharded_driver_hip_threads_bitwise(name, world):
    _run(capi.hip_library(), name, world, device=0)


@pytest.mark.gpu
def test_rccl_single_rank_photoi_sum_destroy():
    """the first device SUM of a tree sharded over RCCL (which
    builds the fold weights) must not touch the side streams the concurrent
    Helmholtz modes created before it. Photoionization, then the sum, then
    photoionization again on the same tree, then destroy: bitwise the
    unsharded run."""
    from afh.dist import rccl_comm
    lib = capi.hip_library()
    base = Simulation(lib, golden.load("rtest_test_3d_photoi_chem"), device=0)
    base.start()
    sim = base.clone(lib, device=0)
    iv = base.cc_names.index("e") + 1

    def run(s):
        a = _steps(s, 1)
        total = s.tree.sum_cc(iv)
        return a + _steps(s, 1) + [total]

    ref = run(base)
    comm = rccl_comm(lib, 0, 1, 0)
    try:
        sh = NativeShard(lib, sim.af.topology(), 1, 0, transport=capi.DIST_RCCL, comm=comm)
        sim.shard_over(sh)
        got = run(sim)
        phi = sim.tree.get_cc(base.cc_names.index("phi") + 1)
        sh.detach()
        sim.tree.close()
    finally:
        lib.call("dist_rccl_comm_destroy", comm)
    assert got == ref
    assert np.array_equal(phi, base.tree.get_cc(base.cc_names.index("phi") + 1))


def _run_loop(lib, world, n_steps, device=-1, gather=False, monkeypatch=None):
    """The regression run test_3d sharded from its first step: the whole
    time loop -- step control, output rows, refinement every 2 steps (the
    first regrid that adds boxes is at step 46) -- with the refinement of a
    sharded run: rank-local (each rank regrids its part of the new partition
    from the boxes it needs, received point to point) or, with gather, the
    whole tree gathered and regridded on every rank."""
    if monkeypatch is not None:
        monkeypatch.setenv("AFH_REGRID_GATHER", "1" if gather else "0")
    base = Simulation(lib, golden.load("rtest_test_3d"), device=device)
    base.start()
    clones = [base.clone(lib, device=device) for _ in range(world)]
    for c in clones:
        c.time_last_output = base.time_last_output
        c.log = list(base.log)
    topo = base.af.topology()
    group = NativeGroup(lib, world)
    shards = [NativeShard(lib, topo, world, r, group=group) for r in range(world)]
    for sim, sh in zip(clones, shards):
        sim.shard_over(sh)

    def loop(sim):
        for _ in range(n_steps):
            sim.step()
        return np.array(sim.log), sim.af.highest_id

    with ThreadPoolExecutor(world) as ex:
        outs = list(ex.map(loop, clones))
    if not gather:
        # the regrid moved single boxes, not the tree: each rank received
        # fewer boxes than the new tree holds
        nb = int(clones[0].af.topology()["n_boxes"])
        got = [sim.regrid_rows_received for sim in clones]
        assert all(g < nb for g in got), (got, nb)
        # on the GPU the boxes moved device to device (Tree.pack_boxes,
        # NativeShard.exchange_rows_dev), never through host arrays
        assert all(sim.regrid_device_rows == (device >= 0) for sim in clones)
    if device >= 0:
        # the sharded V-cycles ran as segment graphs between their exchanges
        # (afh_mg.hip vcycle_segments), all ranks alike
        segs = [sim.graph_stats()[1] for sim in clones]
        assert segs[0] > 0 and len(set(segs)) == 1, segs
    for _ in range(n_steps):
        base.step()
    ref = np.array(base.log)
    ns = (ref.shape[1] - 3) // 3
    for log, hid in outs:
        assert hid == base.af.highest_id
        # it, time, dt and the maxima bitwise; the volume sums are summed
        # per rank, then over the ranks (another association: to rounding)
        assert np.array_equal(log[:, :3], ref[:, :3])
        assert np.array_equal(log[:, 3 + 2 * ns:], ref[:, 3 + 2 * ns:])
        np.testing.assert_allclose(log[:, 3:3 + 2 * ns], ref[:, 3:3 + 2 * ns], rtol=1e-13)
    # the state itself bitwise: every rank's computed boxes
    for iv in range(1, base.n_var_cell + 1):
        want = base.tree.get_cc(iv)
        got = np.full_like(want, np.nan)
        for sim in clones:
            owner = np.asarray(sim.shard.owner)
            mine = (owner == sim.shard.rank) | (owner < 0)
            got[mine] = sim.tree.get_cc(iv)[mine]
        used = np.array([base.af.in_use[b] for b in range(1, len(want) + 1)], bool)
        assert np.array_equal(got[used], want[used]), base.cc_names[iv - 1]
    for sim in clones:
        sim.shard.detach()
    group.close()
    return base


@pytest.mark.parametrize("world,gather", [(2, False), (3, False), (2, True)])
def test_sharded_time_loop_with_regrids_oracle(world, gather, monkeypatch):
    # 3 ranks: after the regrid some rank computes no box of a level
    base = _run_loop(capi.oracle_library(), world, 50, gather=gather,
                     monkeypatch=monkeypatch)
    assert base.af.highest_lvl == 6  # the step-46 regrid added level 6


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_sharded_time_loop_with_regrids_hip(world, monkeypatch):
    base = _run_loop(capi.hip_library(), world, 50, device=0, monkeypatch=monkeypatch)
    assert base.af.highest_lvl == 6
