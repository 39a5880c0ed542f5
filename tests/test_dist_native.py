"""Native box sharding (afh_dist_*): the library partitions
the tree, builds the exchange plans and runs the exchange hook itself.

* The native partition and plans (afivo-streamer_amd/csrc/afh_dist_core.h,
  compiled into both libafivo_hip and the oracle) equal the Python statement
  of them (afh.dist.Partition) -- host code, checked on the CPU for both
  libraries.
* Ranks as threads of one process (AFH_DIST_LOCAL): the owned boxes of all
  ranks, gathered, are bitwise equal to a single-rank run (FMG start-up
  solve, field solve, a Heun step, time-step limits; on the rod-electrode
  AMR tree also the level-set operators and a Helmholtz FMG) -- the oracle's
  CPU twin here, libafivo_hip with 2 and 3 ranks on the test box's GPU. Each
  rank stores only the boxes it reads (afh_tree_create_sharded); the unused
  id that stands for the others reads as NaN, so a stray read would show.
* AFH_DIST_RCCL with one rank on the GPU (two ranks cannot share one GPU in
  an RCCL communicator): the reductions go through ncclAllReduce and the
  result is bitwise the unsharded run. Multi-rank RCCL is unmeasured here.
"""
import ctypes as C
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from afh import capi
import golden
from afh.dist import NativeGroup, NativeShard, Partition, rccl_comm
from afh.model import Tree
from afh.streamer import FV, IV
from test_dist import CC_VARS, FV, TOPOS, _run

KINDS = [capi.HOOK_HALO, capi.HOOK_RIMS, capi.HOOK_CFLUX, capi.HOOK_RESTRICT]


def _python_regions(part, kind, level, recv, send):
    if kind == capi.HOOK_HALO:
        r = part.halo_regions(recv, send, level, False)
    elif kind == capi.HOOK_RIMS:
        r = part.halo_regions(recv, send, level, True)
    elif kind == capi.HOOK_CFLUX:
        r = part.cflux_regions(recv, send)
    else:
        r = part.octant_regions(send, level) if level in part.restrict_levels() else []
    w = 8 if kind == capi.HOOK_CFLUX else 7
    return np.asarray(r, np.int32).reshape(-1, w)


@pytest.mark.parametrize("libname", ["oracle", "hip"])
@pytest.mark.parametrize("name,world", [("uni8_l3", 2), ("amr8", 2), ("amr8", 3),
                                        ("uni8_l3", 5)])
def test_native_partition_and_plans_equal_python(libname, name, world):
    lib = capi.oracle_library() if libname == "oracle" else capi.hip_library()
    topo = TOPOS[name]()
    part = Partition(topo, world)
    sh = NativeShard(lib, topo, world, 0, transport=capi.DIST_LOCAL,
                     group=type("G", (), {"h": None})())
    np.testing.assert_array_equal(sh.owner, part.owner)
    assert sh.lp == part.lp
    n_regions = 0
    for kind in KINDS:
        levels = [0] if kind == capi.HOOK_CFLUX else range(1, part.nlvl + 1)
        for level in levels:
            for recv in range(world):
                for send in range(world):
                    if recv == send:
                        continue
                    got = sh.plan(kind, level, recv, send)
                    want = _python_regions(part, kind, level, recv, send)
                    np.testing.assert_array_equal(got, want, err_msg=str((kind, level, recv, send)))
                    n_regions += len(got)
    assert n_regions > 0


def test_native_partition_refuses_too_many_ranks():
    lib = capi.oracle_library()
    topo = TOPOS["uni8_l3"]()
    with pytest.raises(capi.AfhError, match="no level"):
        NativeShard(lib, topo, 10 ** 4, 0, group=type("G", (), {"h": None})())


def test_native_tree_create_sharded_matches_local_topology():
    """afh_tree_create_sharded == tree_create on the Python local view: the
    sharded trees' reductions see only their own leaves."""
    from afh.model import Tree
    lib = capi.oracle_library()
    topo = TOPOS["amr8"]()
    part = Partition(topo, 2)
    sh = NativeShard(lib, topo, 2, 1, group=type("G", (), {"h": None})())
    a = sh.make_tree(lib, topo, 4, 1)
    b = Tree(lib, part.local_topology(1), 4, 1)
    rng = np.random.default_rng(0)
    x = rng.random(b.cc_shape)  # whole-tree array; a stores only its boxes
    a.put_cc(2, x)
    b.put_cc(2, x)
    assert a.sum_cc(2) == b.sum_cc(2)
    assert a.maxabs_cc(2) == b.maxabs_cc(2)
    # owned-box allocation: fewer stored boxes than the tree has, every
    # owned and replicated box among them, and the rest read back as NaN
    assert a.n_boxes - 1 < a.n_global
    mine = sh.owned_mask()
    assert np.all(np.isin(np.nonzero(mine)[0] + 1, a.global_ids))
    y = a.get_cc(2)
    np.testing.assert_array_equal(y[mine], x[mine])
    absent = np.setdiff1d(np.arange(1, a.n_global + 1), a.global_ids)
    assert len(absent) and np.isnan(y[absent - 1]).all()
    a.close()
    b.close()


def _sum_topo():
    """Leaves below the partition level: one of the eight level-1 boxes is
    refined, so with two ranks level 2 is the partition level and the seven
    level-1 leaves are replicated on both ranks."""
    from afh.tree import build_tree
    return build_tree(8, (16, 16, 16), (2e-3, 2e-3, 2e-3), 1,
                      refine=lambda lvl, r0, r1: lvl < 2 and np.all(r1 <= 1e-3 + 1e-12))


def _sharded_sums(lib, device=-1):
    topo = _sum_topo()
    world = 2
    rng = np.random.default_rng(3)
    from afh.model import Tree
    ref_tree = Tree(lib, topo, 2, 1, device=device)
    x = rng.random(ref_tree.cc_shape)
    ref_tree.put_cc(1, x)
    ref = [ref_tree.sum_cc(1), ref_tree.sum_cc(1, 2), ref_tree.maxabs_cc(1)]
    ref_tree.close()
    group = NativeGroup(lib, world)
    shards = [NativeShard(lib, topo, world, r, group=group) for r in range(world)]
    assert shards[0].lp == 2 and int(np.sum(shards[0].owner < 0)) == 8
    repl_leaves = [b for b in topo["lvl_leaves_1"]]
    assert len(repl_leaves) == 7

    def rank(r):
        t = shards[r].make_tree(lib, topo, 2, 1, device=device)
        shards[r].attach(t)
        t.put_cc(1, x)
        out = [t.sum_cc(1), t.sum_cc(1, 2), t.maxabs_cc(1)]
        shards[r].detach()
        t.close()
        return out

    try:
        with ThreadPoolExecutor(world) as ex:
            parts = list(ex.map(rank, range(world)))
    finally:
        group.close()
    return ref, parts


def _check_sums(ref, parts):
    for p in parts:
        assert p == parts[0]  # every rank holds the same all-reduced value
        # the sum over ranks regroups the additions: equal to rounding; a
        # replicated leaf counted twice would be off by ~7/36 of the total
        np.testing.assert_allclose(p[:2], ref[:2], rtol=1e-13)
        assert p[2] == ref[2]


def test_sharded_sum_counts_replicated_leaves_once_oracle():
    """af_tree_sum_cc on a sharded tree (the SUM all-reduce): the leaves of
    the replicated levels below the partition level count once, as on a
    single rank -- the oracle's twin, thread ranks."""
    _check_sums(*_sharded_sums(capi.oracle_library()))


@pytest.mark.gpu
def test_sharded_sum_counts_replicated_leaves_once_hip():
    _check_sums(*_sharded_sums(capi.hip_library(), device=0))


def _run_rod(lib, topo, shard=None):
    """Config 4's shape: the reference's rod-electrode AMR tree
    (tests/golden/rod8.npz, level-set stencils) -- two V-cycles, the
    gradient, FMG without and with guess, a Heun step, then a
    photoionization Helmholtz mode's FMG (m_photoi_helmh.f90:149-204)."""
    g = golden.load("rod8")
    c = golden.make_case(lib, g, coarse_cycles=12, shard=shard)
    golden.upload(c, {**golden.stage_outputs(g, "init"), **golden.stage_outputs(g, "rhs")})
    c.mg.fas_vcycle(True)
    c.mg.fas_vcycle(True)
    c.field_from_potential()
    c.mg.fas_fmg(True, have_guess=False)
    c.mg.fas_fmg(True, have_guess=True)
    out = {"lim": np.asarray(c.heun_step(1e-12)), "res": np.zeros(0)}
    for iv in CC_VARS:
        out["cc%d" % iv] = c.tree.get_cc(iv)
    c.set_voltage(0.0)
    c.fluid.field_set_rhs(IV["rhs"], 0)
    c.helmholtz_mg(44081.25 ** 2).fas_fmg(True, have_guess=False)
    out["helm_phi"] = c.tree.get_cc(IV["phi"])
    out["fc_field"] = c.tree.get_fc(FV["field"])
    if shard is not None:
        shard.detach()
    return out


RUNS = {"uni8_l3": _run, "amr8": _run, "rod8": _run_rod}


def _topo(name):
    return golden.load("rod8") if name == "rod8" else TOPOS[name]()


def _run_threads(lib, name, world, device=-1):
    topo = _topo(name)
    group = NativeGroup(lib, world)
    shards = [NativeShard(lib, topo, world, r, group=group) for r in range(world)]
    try:
        with ThreadPoolExecutor(world) as ex:
            futs = [ex.submit(RUNS[name], lib, topo, shards[r]) for r in range(world)]
            parts = [f.result() for f in futs]
    finally:
        group.close()
    return shards, parts


def _compare(ref, shards, parts):
    for p in parts:
        np.testing.assert_array_equal(p["lim"], ref["lim"])
        np.testing.assert_array_equal(p["res"], ref["res"])
    for key in ref:
        if key in ("res", "lim"):
            continue
        merged = np.array(ref[key], copy=True)
        merged[:] = np.nan
        for sh, p in zip(shards, parts):
            mine = sh.owned_mask()
            merged[mine] = p[key][mine]
        assert not np.isnan(merged).any(), key
        bad = np.argwhere(merged != ref[key])
        assert len(bad) == 0, (key, bad[:5], np.max(np.abs(merged - ref[key])))


@pytest.mark.parametrize("name,world", [("uni8_l3", 2), ("amr8", 3), ("rod8", 2)])
def test_native_sharded_oracle_threads_bitwise(name, world):
    lib = capi.oracle_library()
    ref = RUNS[name](lib, _topo(name))
    shards, parts = _run_threads(lib, name, world)
    _compare(ref, shards, parts)


@pytest.mark.gpu
@pytest.mark.parametrize("name,world", [("uni8_l3", 2), ("amr8", 2), ("amr8", 3),
                                        ("rod8", 2), ("rod8", 3)])
def test_native_sharded_hip_local_bitwise(name, world):
    lib = capi.hip_library()
    ref = RUNS[name](lib, _topo(name))
    shards, parts = _run_threads(lib, name, world)
    _compare(ref, shards, parts)


def _bcast_worker(rank, world, port, outdir):
    import os
    import torch.distributed as dist
    from afh.dist import broadcast_bytes
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        data = bytes(range(128)) if rank == 0 else bytes(128)
        got = broadcast_bytes(data)
        with open(os.path.join(outdir, "r%d" % rank), "wb") as f:
            f.write(got)
    finally:
        dist.destroy_process_group()


def test_unique_id_broadcast_gloo(tmp_path):
    """The RCCL unique id (128 bytes) reaches every rank over the process
    group (rccl_comm; gloo here, device tensors under nccl)."""
    import torch.multiprocessing as mp
    from test_dist import _free_port
    mp.start_processes(_bcast_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2,
                       start_method="spawn", join=True)
    for r in range(2):
        assert (tmp_path / ("r%d" % r)).read_bytes() == bytes(range(128))


@pytest.mark.gpu
def test_native_rccl_single_rank_bitwise():
    lib = capi.hip_library()
    topo = TOPOS["amr8"]()
    ref = _run(lib, topo)
    comm = rccl_comm(lib, 0, 1, 0)
    try:
        sh = NativeShard(lib, topo, 1, 0, transport=capi.DIST_RCCL, comm=comm)
        out = _run(lib, topo, sh)
    finally:
        lib.call("dist_rccl_comm_destroy", comm)
    _compare(ref, [sh], [out])


def _rows_worker(rank, world, port, outdir):
    import os
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # the RCCL transport's path of NativeShard.allgather_rows (torch
        # collectives; gloo here, device tensors under nccl)
        sh = type("S", (), {"transport": capi.DIST_RCCL, "n": world, "rank": rank})()
        ids = np.arange(rank + 1) * 10 + rank
        rows = np.arange((rank + 1) * 3, dtype=np.float64).reshape(rank + 1, 3) + 0.5 * rank
        got = NativeShard.allgather_rows(sh, ids, rows)
        np.savez(os.path.join(outdir, "r%d.npz" % rank),
                 **{"ids%d" % q: g[0] for q, g in enumerate(got)},
                 **{"rows%d" % q: g[1] for q, g in enumerate(got)})
    finally:
        dist.destroy_process_group()


def test_allgather_rows_gloo(tmp_path):
    """The numeric all-gather a sharded regrid gathers boxes with (ragged
    counts, padded rows): every rank receives every rank's ids and rows
    exactly."""
    import torch.multiprocessing as mp
    from test_dist import _free_port
    world = 3
    mp.start_processes(_rows_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       start_method="spawn", join=True)
    for r in range(world):
        d = np.load(tmp_path / ("r%d.npz" % r))
        for q in range(world):
            np.testing.assert_array_equal(d["ids%d" % q], np.arange(q + 1) * 10 + q)
            np.testing.assert_array_equal(
                d["rows%d" % q],
                np.arange((q + 1) * 3, dtype=np.float64).reshape(q + 1, 3) + 0.5 * q)


def _p2p_worker(rank, world, port, outdir):
    import os
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # the RCCL transport's path of NativeShard.exchange_rows (the counts
        # all-gathered, then batched send/recv; gloo here, device tensors
        # under nccl): rank r sends q + r rows of width 4 to every rank q > r
        sh = type("S", (), {"transport": capi.DIST_RCCL, "n": world, "rank": rank})()
        sends = {}
        for q in range(rank + 1, world):
            m = q + rank
            sends[q] = (np.arange(m) + 100 * rank,
                        np.arange(4 * m, dtype=np.float64).reshape(m, 4) + 1000 * rank + q)
        got = NativeShard.exchange_rows(sh, sends)
        np.savez(os.path.join(outdir, "p%d.npz" % rank),
                 **{"ids%d" % q: g[0] for q, g in got.items()},
                 **{"rows%d" % q: g[1] for q, g in got.items()})
    finally:
        dist.destroy_process_group()


def test_exchange_rows_gloo(tmp_path):
    """The point-to-point exchange of the rank-local regrid (only the boxes a
    rank needs from another): every rank receives exactly what each sender
    addressed to it, nothing from ranks that sent it nothing."""
    import torch.multiprocessing as mp
    from test_dist import _free_port
    world = 3
    mp.start_processes(_p2p_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       start_method="spawn", join=True)
    for r in range(world):
        d = np.load(tmp_path / ("p%d.npz" % r))
        assert sorted(k for k in d.files if k.startswith("ids")) == \
            ["ids%d" % q for q in range(r) if q + r > 0]
        for q in range(r):
            m = r + q
            if not m:
                continue
            np.testing.assert_array_equal(d["ids%d" % q], np.arange(m) + 100 * q)
            np.testing.assert_array_equal(
                d["rows%d" % q], np.arange(4 * m, dtype=np.float64).reshape(m, 4) + 1000 * q + r)



def _p2p_dev_worker(rank, world, port, outdir):
    import os
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # NativeShard.exchange_rows_dev's RCCL path with the rows as tensors
        # (CPU tensors under gloo; the tree's device tensors under nccl)
        sh = type("S", (), {"transport": capi.DIST_RCCL, "n": world, "rank": rank})()
        sends = {}
        for q in range(rank + 1, world):
            m = q + rank
            sends[q] = (np.arange(m) + 100 * rank,
                        torch.arange(4 * m, dtype=torch.float64).reshape(m, 4) + 1000 * rank + q)
        got = NativeShard.exchange_rows_dev(sh, sends, torch.device("cpu"))
        np.savez(os.path.join(outdir, "p%d.npz" % rank),
                 **{"ids%d" % q: g[0] for q, g in got.items()},
                 **{"rows%d" % q: g[1].numpy() for q, g in got.items()})
    finally:
        dist.destroy_process_group()


def test_exchange_rows_dev_gloo(tmp_path):
    """The device-tensor form of the rank-local regrid's exchange: the same
    deliveries as exchange_rows, the rows staying tensors."""
    import torch.multiprocessing as mp
    from test_dist import _free_port
    world = 3
    mp.start_processes(_p2p_dev_worker, args=(world, _free_port(), str(tmp_path)),
                       nprocs=world, start_method="spawn", join=True)
    for r in range(world):
        d = np.load(tmp_path / ("p%d.npz" % r))
        assert sorted(k for k in d.files if k.startswith("ids")) == \
            ["ids%d" % q for q in range(r) if q + r > 0]
        for q in range(r):
            m = r + q
            if not m:
                continue
            np.testing.assert_array_equal(d["ids%d" % q], np.arange(m) + 100 * q)
            np.testing.assert_array_equal(
                d["rows%d" % q], np.arange(4 * m, dtype=np.float64).reshape(m, 4) + 1000 * q + r)


class _HostRows:
    """A numpy array as Tree.pack_boxes' buffer (the oracle's "device" is
    the host)."""

    def __init__(self, n, w):
        self.a = np.zeros((n, w))
        self.shape = self.a.shape

    def data_ptr(self):
        return self.a.ctypes.data

    def is_contiguous(self):
        return True


def _pack_roundtrip(lib, rows):
    topo = TOPOS["amr8"]()
    rng = np.random.default_rng(5)
    dev = 0 if rows is not _HostRows else -1
    ta, tb = Tree(lib, topo, 3, 2, device=dev), Tree(lib, topo, 3, 2, device=dev)
    try:
        cc = [rng.standard_normal(ta.cc_shape) for _ in range(3)]
        fc = [rng.standard_normal(ta.fc_shape) for _ in range(2)]
        for iv in range(3):
            ta.put_cc(iv + 1, cc[iv])
        for iv in range(2):
            ta.put_fc(iv + 1, fc[iv])
        src = np.array([3, 1, 7, 2], np.int32)
        dst = np.array([5, 4, 1, 8], np.int32)
        buf = rows(len(src), ta.row_width(2, 1))
        ta.pack_boxes(src, 2, 1, buf)
        if rows is _HostRows:  # the row layout: cc 1, cc 2, fc 1 of each box
            w = int(np.prod(ta.cc_shape[1:]))
            for r, b in enumerate(src):
                assert np.array_equal(buf.a[r, :w], cc[0][b - 1].ravel())
                assert np.array_equal(buf.a[r, w:2 * w], cc[1][b - 1].ravel())
                assert np.array_equal(buf.a[r, 2 * w:], fc[0][b - 1].ravel())
        tb.unpack_boxes(dst, 2, 1, buf)
        got0, got1, gotf = tb.get_cc(1), tb.get_cc(2), tb.get_fc(1)
        for b, d in zip(src, dst):
            assert np.array_equal(got0[d - 1], cc[0][b - 1])
            assert np.array_equal(got1[d - 1], cc[1][b - 1])
            assert np.array_equal(gotf[d - 1], fc[0][b - 1])
        rest = np.setdiff1d(np.arange(1, tb.n_boxes + 1), dst) - 1
        assert not got0[rest].any() and not gotf[rest].any() and not tb.get_cc(3).any()
    finally:
        ta.close()
        tb.close()


def test_tree_pack_unpack_boxes_oracle():
    """afo_tree_pack_boxes / afo_tree_unpack_boxes: the row layout (each
    box's cell variables, then its face variables, ghost cells included) and
    the round trip into other boxes of another tree, the rest untouched."""
    _pack_roundtrip(capi.oracle_library(), _HostRows)


@pytest.mark.gpu
def test_tree_pack_unpack_boxes_roundtrip():
    """The same through device rows of the library's own allocation
    (afh_device_alloc, model.DeviceRows): boxes of one tree into other boxes
    of another without a host copy, every variable bitwise."""
    from afh.model import DeviceRows
    lib = capi.hip_library()
    _pack_roundtrip(lib, lambda n, w: DeviceRows(lib, 0, n, w))


@pytest.mark.gpu
def test_rccl_single_rank_device_sum():
    """af_tree_sum_cc on a tree sharded over RCCL (round 5): the box sums,
    their fold (k_sum_fold, the host loop's order) and the ncclAllReduce stay
    on the device, one transfer at the end -- bitwise the unsharded tree's
    host fold with one rank."""
    lib = capi.hip_library()
    topo = _sum_topo()
    rng = np.random.default_rng(3)
    from afh.model import Tree
    ref_tree = Tree(lib, topo, 2, 1, device=0)
    x = rng.random(ref_tree.cc_shape)
    ref_tree.put_cc(1, x)
    ref = [ref_tree.sum_cc(1), ref_tree.sum_cc(1, 2)]
    ref_tree.close()
    comm = rccl_comm(lib, 0, 1, 0)
    try:
        sh = NativeShard(lib, topo, 1, 0, transport=capi.DIST_RCCL, comm=comm)
        t = sh.make_tree(lib, topo, 2, 1, device=0)
        sh.attach(t)
        t.put_cc(1, x)
        got = [t.sum_cc(1), t.sum_cc(1, 2)]
        sh.detach()
        t.close()
    finally:
        lib.call("dist_rccl_comm_destroy", comm)
    assert got == ref


@pytest.mark.gpu
def test_rccl_capture_single_rank_bitwise(monkeypatch):
    """AFH_RCCL_CAPTURE=1: the V-cycles of a tree sharded over RCCL are
    captured as whole graphs with their exchanges inside (one rank here: the
    exchange posts an empty group), bitwise the unsharded run."""
    monkeypatch.setenv("AFH_RCCL_CAPTURE", "1")
    import golden
    from afh.streamer import IV, StreamerCase, seed_state, tables_from
    lib = capi.hip_library()
    topo = TOPOS["amr8"]()
    ref = _run(lib, topo)
    comm = rccl_comm(lib, 0, 1, 0)
    try:
        sh = NativeShard(lib, topo, 1, 0, transport=capi.DIST_RCCL, comm=comm)
        g = golden.load("uni8")
        td, chem = tables_from(g)
        c = StreamerCase(lib, topo, td, chem, float(g["current_voltage"]), coarse_cycles=12,
                         shard=sh)
        seed_state(c)
        c.fluid.field_set_rhs(IV["rhs"], 0)
        c.mg.fas_fmg(True, have_guess=False)
        res = c.field_compute(0)
        lim = c.heun_step(1e-12)
        replays, segmented = c.mg.graph_stats()
        out = {"res": np.asarray(res), "lim": np.asarray(lim)}
        for k in ref:
            if k.startswith("cc"):
                out[k] = c.tree.get_cc(int(k[2:]))
        out["fc_flux"] = c.tree.get_fc(FV["flux"])
        sh.detach()
    finally:
        lib.call("dist_rccl_comm_destroy", comm)
    _compare(ref, [sh], [out])
    # whole-graph replays (a segment replay would count as segmented)
    assert replays > 0 and segmented == 0, (replays, segmented)


def _peer_bytes_consistent(lib, name, world, monkeypatch):
    """afh_dist_peer_bytes (round 6): what rank r sent to q is what q
    received from r, and nothing goes to a rank itself (read as each rank
    detaches)."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    pb = {}
    detach = NativeShard.detach

    def record(self):
        pb[self.rank] = bench.dist_peer_bytes(self.lib, self)
        detach(self)
    monkeypatch.setattr(NativeShard, "detach", record)
    _run_threads(lib, name, world)
    assert sorted(pb) == list(range(world))
    for r in range(world):
        assert pb[r][0][r] == 0 and pb[r][1][r] == 0
        for q in range(world):
            assert pb[r][0][q] == pb[q][1][r], (r, q)
    assert sum(int(pb[r][0].sum()) for r in range(world)) > 0


def test_peer_bytes_consistent_oracle(monkeypatch):
    _peer_bytes_consistent(capi.oracle_library(), "amr8", 3, monkeypatch)


@pytest.mark.gpu
def test_peer_bytes_consistent_hip(monkeypatch):
    _peer_bytes_consistent(capi.hip_library(), "amr8", 3, monkeypatch)
