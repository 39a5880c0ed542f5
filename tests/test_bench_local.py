"""bench.py's sharded step on thread ranks (--transport local, round 5).

The driver's multi-GPU bench (`bench.py --gpus N` under torchrun, one rank
per GPU over RCCL) has never run on more than one GPU: our box has one. The
local transport runs every line of that path -- the partition, the plans,
the exchange hooks, the sharded unit step (field_compute + forward_euler's
species part, Heun stages alternating), the driver configurations'
shard_over -- with the ranks as threads of one process (AFH_DIST_LOCAL: pack,
host barrier, peer copies, unpack) instead of processes over RCCL. Here, on
the C oracle (CPU): N = 2 and 8 ranks for the uniform config 2 tree (s1) and
the driver configs 4 (s4, rod electrode) and 5 (s5, sprite), each rank's
owned boxes after the steps bitwise the single-rank run's, and the time-step
limits equal.
"""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from afh import capi  # noqa: E402

STEPS = 3


def _steps(case, steps=STEPS):
    out = []
    if case.__class__.__name__ != "DriverCase":
        case.fuse_rhs(True, ghosts=False)
        case.faces_from_phi(True)
    else:
        case.fuse_rhs(True, ghosts=False)
    case.field_compute(0, n_vcycles=2)
    for k in range(steps):
        res, d = bench.unit_step(case, 1e-13, k)
        out.append((tuple(res), None if d is None else tuple(np.ravel(d))))
    case.tree.sync()
    return out


def _single(lib, config, coarse, device):
    if config in bench.DRIVER_CONFIGS:
        return bench.DriverCase(bench.build_driver_case(lib, device, config, coarse))
    return bench.build_case(lib, config, device, coarse)


def _bitwise(lib, config, world, device=-1, floor=0):
    """floor: bench's min_level_cells (0: every level from 2 sharded)."""
    coarse = bench.coarse_choice("auto", config)
    one = _single(lib, config, coarse, device)
    ref = _steps(one)
    cases, shards, group, base = bench.local_ranks(lib, config, world, device, coarse,
                                                   min_level_cells=floor)
    try:
        outs = bench.run_ranks(cases, lambda r, c: _steps(c))
        stats = [bench.dist_stats(lib, sh) for sh in shards]
    finally:
        for sh in shards:
            sh.detach()
        group.close()
    if shards[0].lp is not None:
        assert all(n > 0 for n, _ in stats)
    else:  # the whole tree replicated: no exchange at all
        assert all(n == 0 for n, _ in stats)
    for o in outs:
        assert o == ref, (o, ref)
    for iv in range(1, one.tree.n_var_cell + 1):
        want = one.tree.get_cc(iv)
        got = np.full_like(want, np.nan)
        for c, sh in zip(cases, shards):
            mine = sh.owned_mask()
            got[mine] = c.tree.get_cc(iv)[mine]
        used = ~np.isnan(got).reshape(len(got), -1).all(axis=1)
        assert used.any()
        assert np.array_equal(got[used], want[used]), iv


@pytest.mark.parametrize("config,world", [("s1", 2), ("s1", 8), ("s4", 2), ("s5", 2),
                                          ("s5", 8)])
def test_local_transport_bitwise_single_rank(config, world):
    _bitwise(capi.oracle_library(), config, world)


@pytest.mark.parametrize("config,world", [("s1", 8), ("s5", 3)])
def test_local_transport_bitwise_level_floor(config, world):
    """bench's default partition (round 6): levels under MIN_LEVEL_CELLS
    replicated -- s1: levels 1-3 on every rank, level 4 sharded; s5's set-up
    tree: every level below the floor, the whole tree replicated."""
    _bitwise(capi.oracle_library(), config, world, floor=bench.MIN_LEVEL_CELLS)


@pytest.mark.gpu
@pytest.mark.parametrize("config,world", [("s1", 2), ("s1", 4), ("s5", 2), ("s5", 8)])
def test_local_transport_bitwise_single_rank_hip(config, world):
    """The same on libafivo_hip: the thread ranks share device 0, each on its
    own stream (peer copies within the device)."""
    _bitwise(capi.hip_library(), config, world, device=0)


@pytest.mark.gpu
@pytest.mark.parametrize("config,world", [("s1", 8), ("s1-64", 2)])
def test_local_transport_bitwise_level_floor_hip(config, world):
    """bench's default partition on the GPU: s1 with levels 1-3 replicated;
    s1-64 at N = 2 (the headline tree: fused 64^3 pairs with one- and
    two-layer halos, ghost-only rims)."""
    _bitwise(capi.hip_library(), config, world, device=0, floor=bench.MIN_LEVEL_CELLS)


@pytest.mark.gpu
def test_bench_local_json():
    """bench.py --transport local --gpus 4 --shared-stream, the line the
    scaling projection reads (scripts/project_scaling.py)."""
    import argparse
    args = argparse.Namespace(gpus=4, config="s5", steps=2, warmup=1, oracle=False,
                              shared_stream=True, no_fused_rhs=False,
                              stored_face_field=False, grow_cells=0, min_level_cells=0)
    out = bench.bench_local(args, bench.coarse_choice("auto", "s5"))
    assert out["n_ranks"] == 4 and out["value"] > 0
    assert len(out["owned_leaf_cells"]) == 4 and min(out["owned_leaf_cells"]) > 0
    assert sum(out["owned_leaf_cells"]) <= out["config"]["leaf_cells"]
    assert all(x > 0 for x in out["exchanges_per_step"])
