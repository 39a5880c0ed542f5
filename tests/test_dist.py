"""Sharded tree over ranks (afh.dist).

world_size 2 (and 3) gloo processes each run their part of a sharded tree
-- on the CPU with the C oracle as the compute engine, on the GPU with
libafivo_hip (2 ranks sharing the test box's GPU) -- through the exchange
hooks the libraries call; the owned boxes of all ranks, gathered, must be
bitwise equal to a single-rank run of the same case (FMG start-up solve,
field solve with residual checks, a Heun step), and so must the time-step
limits.
"""
import os
import socket
import sys

import numpy as np
import pytest

import golden
from afh import capi
from afh.dist import Partition, Shard, morton3
from afh.streamer import IV, FV, StreamerCase, seed_state, tables_from
from afh.tree import build_tree, uniform_tree

TOPOS = {
    "uni8_l3": lambda: uniform_tree(8, (16, 16, 16), (2e-3, 2e-3, 2e-3), 3),
    "amr8": lambda: build_tree(
        8, (16, 16, 16), (2e-3, 2e-3, 2e-3), 2,
        refine=lambda lvl, r0, r1: lvl < 4 and np.all(r0 < 1.2e-3) and np.all(r1 > 0.7e-3)),
}
CC_VARS = [IV["e"], IV["e"] + 1, IV["pos"], IV["neg"], IV["phi"], IV["efld"], IV["rhs"]]


def _run(lib, topo, shard=None):
    g = golden.load("uni8")
    td, chem = tables_from(g)
    c = StreamerCase(lib, topo, td, chem, float(g["current_voltage"]),
                     coarse_cycles=12, shard=shard)
    seed_state(c)
    c.fluid.field_set_rhs(IV["rhs"], 0)
    c.mg.fas_fmg(True, have_guess=False)  # start-up solve
    res = c.field_compute(0)
    lim = c.heun_step(1e-12)
    out = {"res": np.asarray(res), "lim": np.asarray(lim)}
    for iv in CC_VARS:
        out["cc%d" % iv] = c.tree.get_cc(iv)
    out["fc_flux"] = c.tree.get_fc(FV["flux"])
    if shard is not None:
        shard.detach()
    return out


def _worker(rank, world, port, name, outdir, use_hip=False):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        topo = TOPOS[name]()
        part = Partition(topo, world)
        if use_hip:
            # several ranks share the one GPU of the test box: gloo transport
            # staged through the host
            lib, shard = capi.hip_library(), Shard(part, rank, "gloo", device="cuda:0")
        else:
            lib, shard = capi.oracle_library(), Shard(part, rank, "gloo")
        out = _run(lib, topo, shard)
        out["owner"] = part.owner
        np.savez(os.path.join(outdir, "rank%d.npz" % rank), **out)
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_partition_covers_every_box_once():
    topo = TOPOS["amr8"]()
    part = Partition(topo, 3)
    lp = part.lp
    for l in range(1, part.nlvl + 1):
        ids = part.ids[l]
        owners = part.owner[ids - 1]
        if l < lp:
            assert np.all(owners == -1)
        else:
            assert np.all((owners >= 0) & (owners < 3))
            # children live with their parent
            if l > lp:
                assert np.all(owners == part.owner[part.parent[ids - 1] - 1])
    assert set(part.owner[part.ids[lp] - 1]) == {0, 1, 2}
    assert list(morton3(np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [1, 1, 1]]))) == [0, 1, 2, 7]


def test_halo_plans_are_symmetric():
    topo = TOPOS["uni8_l3"]()
    part = Partition(topo, 2)
    for lvl in range(part.lp, part.nlvl + 1):
        for rims in (False, True):
            a = part.halo_regions(0, 1, lvl, rims)
            b = part.halo_regions(1, 0, lvl, rims)
            assert a and b
            assert all(part.owner[r[0] - 1] == 1 for r in a)
            assert all(part.owner[r[0] - 1] == 0 for r in b)


def _compare_sharded(name, world, tmp_path, use_hip):
    import torch.multiprocessing as mp
    lib = capi.hip_library() if use_hip else capi.oracle_library()
    ref = _run(lib, TOPOS[name]())
    mp.start_processes(_worker, args=(world, _free_port(), name, str(tmp_path), use_hip),
                       nprocs=world, start_method="spawn", join=True)
    parts = [np.load(tmp_path / ("rank%d.npz" % r)) for r in range(world)]
    owner = parts[0]["owner"]
    for p in parts:
        np.testing.assert_array_equal(p["lim"], ref["lim"])
        np.testing.assert_array_equal(p["res"], ref["res"])
    for key in ref:
        if key in ("res", "lim"):
            continue
        merged = np.array(ref[key], copy=True)
        merged[:] = np.nan
        for r, p in enumerate(parts):
            mine = (owner == r) | (owner < 0)
            merged[mine] = p[key][mine]
        assert not np.isnan(merged).any(), key
        bad = np.argwhere(merged != ref[key])
        assert len(bad) == 0, (key, bad[:5], np.max(np.abs(merged - ref[key])))


@pytest.mark.parametrize("name,world", [("uni8_l3", 2), ("amr8", 2), ("uni8_l3", 3)])
def test_sharded_run_bitwise_equals_single_rank(name, world, tmp_path):
    _compare_sharded(name, world, tmp_path, use_hip=False)


@pytest.mark.gpu
@pytest.mark.parametrize("fused", ["0", "1", "default"])
@pytest.mark.parametrize("name", ["uni8_l3", "amr8"])
def test_sharded_hip_bitwise_equals_single_rank(name, fused, tmp_path, monkeypatch):
    """The HIP library with 2 ranks on one GPU; split smoother, fused
    smoother on every level, and the default choice."""
    if fused != "default":
        monkeypatch.setenv("AFH_GSRB_FUSED_MIN_BOXES", fused)
    _compare_sharded(name, 2, tmp_path, use_hip=True)
