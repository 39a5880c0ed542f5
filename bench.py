#!/usr/bin/env python3
"""Benchmark: cell-updates/s of the afivo-streamer hot path on MI355X.

One step = one unit of SURVEY.md 8(d) on every leaf cell: field_set_rhs +
max|rhs| + one FAS V(2,2)-cycle with the residual + max|residual| (the
field_compute convergence test) + field_from_potential (gradient, |E|, |E|
ghost cells) + flux_upwind_tree + flux_update_densities with chemistry --
one sub-step of af_heuns_method, stages 1 and 2 alternating (unit_step) --
all through libafivo_hip.so.

Default workload: S1-64: a uniform 3-D tree of 512 leaf boxes
of 64^3 cells (134 M leaf cells, 585 boxes, 4 levels, 64^3 coarse grid),
16 mm cube, electrons + M+ + M- (td_air_siglo_swarm.txt old-style model),
Gaussian seed, -2.5 MV/m background field. Synthetic data, FP64.

Multi-GPU (torchrun, one rank per GPU): the SAME tree is sharded over the
ranks (afh.dist: Morton-ordered subtrees of the coarsest level with a box per
rank, coarser levels replicated; halo / restriction / consistent-flux
exchanges with RCCL on the tree's stream, all-reduced time-step limits), so
the per-GPU work shrinks as N grows ("scaling": "strong"). A barrier
brackets the timed region and the time is the max over ranks. `--replicas`
runs one independent copy of the workload per GPU instead ("weak").
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "afivo-streamer_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

CONFIGS = {
    # name: (n_cell, coarse grid, levels, domain [m])
    "s1-64": (64, (64, 64, 64), 4, (16e-3, 16e-3, 16e-3)),
    "s1": (16, (16, 16, 16), 4, (16e-3, 16e-3, 16e-3)),
    # BASELINE.json config 3: programs/standard_3d/streamer_3d.cfg with
    # air_chemistry_v2 (9 species, 25 reactions), the AMR tree the reference's
    # set_initial_conditions builds (afivo-streamer_amd/afh/decks/case_s3.npz, exported from
    # the reference's own initializers; afh.driver builds the tree on the
    # device)
    "s3": (8, None, None, (16e-3, 16e-3, 16e-3)),
    # BASELINE.json config 5: programs/3d_sprite/sprite_3d.cfg -- sprite
    # chemistry (10 species, 12 reactions), the exponential atmosphere of its
    # m_user.f90 as a variable gas density, Helmholtz photoionization every
    # photoi%per_steps time steps, the 8-level AMR tree of 8^3 boxes its
    # initial refinement builds (afivo-streamer_amd/afh/decks/case_s5.npz, afh.users.Sprite3D)
    "s5": (8, None, None, (5e3, 5e3, 20e3)),
    # BASELINE.json config 4 on one device: config 3 with the grounded rod
    # electrode of SURVEY 8(d) S4 (afivo-streamer_amd/afh/decks/case_s4.npz): level-set
    # stencils on the boxes the rod crosses (afh.electrode), the electrode's
    # species boundary condition every time step, 5 levels of 8^3 boxes
    "s4": (8, None, None, (16e-3, 16e-3, 16e-3)),
    # BASELINE.json config 1: programs/standard_2d/streamer_2d.cfg itself on
    # the 2-D build (libafivo_hip_2d.so) -- air_chemistry_v1 (8 species, 25
    # reactions), the AMR tree of 8^2 boxes its set_initial_conditions
    # builds (afivo-streamer_amd/afh/decks/case_s2d.npz, exported from the reference's own
    # initializers)
    "2d": (8, None, None, (32e-3, 32e-3)),
    # a uniform 2-D tree with config 1's box size and domain (8 levels of 8^2
    # boxes, 1024^2 cells, the old-style 3-species model): the 2-D tests'
    # synthetic workload
    "2d-uniform": (8, (8, 8), 8, (32e-3, 32e-3)),
}
DRIVER_CONFIGS = ("s3", "s4", "s5", "2d")
DRIVER_FIXTURE = {"s3": "case_s3", "s4": "case_s4", "s5": "case_s5", "2d": "case_s2d"}
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md, HBM3E peak (spec)


# level-1 solves (--coarse): the reference's HYPRE PFMG restated (50
# iterations at most, tolerance 1e-6: m_af_types.f90:560-565), or our exact
# separable solve
COARSE = {"pfmg": dict(coarse_cycles=50, coarse_tol=1e-6, coarse_mode=3),
          "direct": dict(coarse_cycles=0, coarse_tol=0.0, coarse_mode=None)}


def coarse_kw(coarse):
    """Level-1 solve keywords: "pfmg" / "direct", or an int (the tests'
    form): 0 = the exact solve, N > 0 = N of our MG cycles."""
    if isinstance(coarse, str):
        return COARSE[coarse]
    return dict(coarse_cycles=int(coarse)) if coarse else COARSE["direct"]


def coarse_choice(arg, config):
    """auto: the reference's PFMG on its own configurations (s3, s4, s5, 2d),
    the exact solve on the synthetic uniform trees (s1, s1-64: a 64^3 level 1
    is one workgroup's worth of PFMG too many)."""
    if arg != "auto":
        return arg
    return "pfmg" if config in DRIVER_CONFIGS or config == "2d" else "direct"


# levels smaller than this are replicated on every rank instead of sharded
# (afh_dist_partition_levels): such a level's kernels are launch-bound on one
# GPU already, so sharding it only adds its exchanges
MIN_LEVEL_CELLS = 1 << 21


def build_case(lib, config, device, coarse, shard_ranks=None, shard=None,
               min_level_cells=MIN_LEVEL_CELLS):
    """shard_ranks = (world, rank, "native" | "python"): this rank's part of
    the sharded tree; or shard: a prepared afh.dist shard (thread ranks)."""
    from afh.streamer import StreamerCase, seed_state, tables_from
    from afh.tree import uniform_tree
    from afh import decks
    nc, cgs, lvls, dom = CONFIGS[config]
    if len(dom) == 2:
        from afh.tree import uniform_tree_2d
        topo = uniform_tree_2d(nc, cgs, dom, lvls)
    else:
        topo = uniform_tree(nc, cgs, dom, lvls)
    # transport / chemistry tables exported from the reference (package data)
    td, chem = tables_from(decks.load("tables_air_siglo"))
    voltage = -dom[-1] * (-2.5e6)
    if shard_ranks is not None:
        world, rank, kind = shard_ranks
        if kind == "native":
            # the library's own sharding: owned-box storage, exchanges as
            # RCCL send/recv on the tree's stream, no Python in the step
            from afh import capi
            from afh.dist import NativeShard, rccl_comm
            shard = NativeShard(lib, topo, world, rank, transport=capi.DIST_RCCL,
                                comm=rccl_comm(lib, rank, world, device),
                                min_level_cells=min_level_cells)
        else:
            from afh.dist import Partition, Shard
            shard = Shard(Partition(topo, world), rank, "nccl", device="cuda:%d" % device)
    case = StreamerCase(lib, topo, td, chem, voltage, device=device, shard=shard,
                        **coarse_kw(coarse))
    seed_state(case, width=0.05 * dom[-1])
    return case


def unit_step(case, dt, k):
    """One sub-step of af_heuns_method (m_af_advance.f90:159-163), the
    reference's default integrator: field_compute (1 V-cycle) on the
    derivative state + forward_euler's species part (flux_upwind_tree +
    flux_update_densities). Even k: stage 1 (state 0 -> 1); odd k: stage 2
    (states 0, 1 -> 0, with the chemistry dt limit). Returns the residuals and
    dt limits."""
    if hasattr(case, "pre_step"):
        case.pre_step(k)
    # defer: the V-cycle's residual is read with the species step's limits,
    # one host synchronisation per sub-step (afh_mg_fas_vcycle_fold)
    # stage 1's dt limits are never read (af_advance keeps the last
    # sub-step's, m_af_advance.f90:160-164): they stay on the device and the
    # host synchronises once per time step, after stage 2. So is stage 1's
    # V-cycle residual: the returned list is empty for stage 1 (the JSON
    # line's last_residual is stage 2's)
    if k % 2 == 0:
        res = case.field_compute(0, n_vcycles=1, defer=True)
        d = case.species_step(dt, 0, [0], [1.0], 1, False, fetch=False)
    else:
        res = case.field_compute(1, n_vcycles=1, defer=True)
        d = case.species_step(0.5 * dt, 1, [0, 1], [0.5, 0.5], 0, True)
    return res, d


class DriverCase:
    """bench adapter for an afh.driver.Simulation (config s3): the same unit
    step -- field_compute of the derivative state (the reference's
    field_compute: field_set_rhs + up to multigrid_num_vcycles V-cycles with
    the residual test + field_from_potential) + forward_euler's species part,
    Heun stages alternating."""

    def __init__(self, sim):
        self.sim = sim
        self.topo = sim.af.topology()

    @property
    def tree(self):
        return self.sim.tree

    @property
    def shard(self):
        return self.sim.shard

    def field_compute(self, s, n_vcycles=2, defer=False):
        return self.sim.field_compute(s, True)

    def species_step(self, dt, s_deriv, s_prev, w_prev, s_out, last, fetch=True):
        if not fetch:
            self.sim.fluid.forward_euler_fold(dt, s_deriv, s_prev, w_prev, s_out, last)
            return None
        return self.sim.fluid.forward_euler(dt, s_deriv, s_prev, w_prev, s_out, last)

    def pre_step(self, k):
        """photoi_set_src every photoi%per_steps time steps (streamer.f90:
        230-234), i.e. every 2 * per_steps unit steps."""
        sim = self.sim
        if sim.photoi and k % (2 * sim.c.i("photoi%per_steps")) == 0:
            sim.photoi_set_src()
        if sim.lsf is not None and k % 2 == 0:  # set_electrode_densities
            sim.fluid.electrode_species_bc(
                sim.i_lsf, sim.i_1pos_ion, sim.electrode_ids,
                sim.c.s("species_boundary_condition") == "neumann_zero")

    def fuse_rhs(self, on=True, ghosts=False):
        self.sim.fluid.set_rhs_output(self.sim.i_rhs if on else 0, ghosts)
        self.sim.fused_rhs = on


def build_driver_case(lib, device, config="s3", coarse="pfmg", grow_cells=0,
                      grow_seconds=240.0):
    """The reference's set-up (set_initial_conditions) of a driver config;
    with grow_cells, then the time loop (streamer.f90's main loop: Heun
    steps with step control, refinement every refine_per_steps, output rows)
    until the tree holds at least grow_cells leaf cells, or grow_seconds
    pass, or the end time is reached."""
    from afh import decks
    from afh.driver import Simulation
    from afh.users import USERS
    sim = Simulation(lib, decks.load(DRIVER_FIXTURE[config]), device=device,
                     user=USERS.get(config), **coarse_kw(coarse))
    sim.set_initial_conditions()
    sim.grown = {"steps": 0, "time_s": 0.0, "leaf_cells_initial": sim.af.n_leaf_cells()}
    if grow_cells:
        sim.output_cnt = 0
        sim.output_write()
        sim.time_last_output = sim.time
        t0 = t_print = time.perf_counter()
        while (sim.af.n_leaf_cells() < grow_cells and
               time.perf_counter() - t0 < grow_seconds and sim.step()):
            sim.grown["steps"] += 1
            if time.perf_counter() - t_print > 20:  # progress (a long growth is not a hang)
                t_print = time.perf_counter()
                print("grow: %d steps, t = %.4g s, %d leaf cells, %.0f s" %
                      (sim.grown["steps"], sim.time, sim.af.n_leaf_cells(), t_print - t0),
                      file=sys.stderr, flush=True)
        sim.grown["time_s"] = sim.time
    return sim


def cpu_baseline_driver(sim, steps=2, config="s3"):
    """The C oracle on the same S3 / S5 state (the tree built on the device, every
    variable copied over), `steps` unit steps."""
    from afh import capi
    osim = sim.clone(capi.oracle_library())
    case = DriverCase(osim)
    unit_step(case, 1e-13, 0)
    t0 = time.perf_counter()
    for k in range(steps):
        unit_step(case, 1e-13, k + 1)
    dt = time.perf_counter() - t0
    ncell = osim.af.n_leaf_cells()
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    return {"value": ncell * steps / dt, "unit": "cell-updates/s", "cores": threads,
            "kind": "port",
            "sample": "%d steps of the full %s workload (%d leaf cells), C oracle "
                      "OpenMP" % (steps, config.upper(), ncell)}


def cpu_baseline(config, coarse, steps=2):
    """The C oracle (oracle/lib/libafo.so, OpenMP) on a bounded sample of the
    same workload: the same 64^3 boxes but a 3-level tree (64 leaf boxes)."""
    from afh import capi
    from afh.streamer import StreamerCase, seed_state, tables_from
    from afh.tree import uniform_tree
    from afh import decks
    nc, cgs, lvls, dom = CONFIGS[config]
    sample_lvls = 3 if config == "s1-64" else lvls
    topo = uniform_tree(nc, cgs, dom, sample_lvls)
    td, chem = tables_from(decks.load("tables_air_siglo"))
    lib = capi.oracle_library()
    case = StreamerCase(lib, topo, td, chem, -dom[2] * (-2.5e6), **coarse_kw(coarse))
    seed_state(case, width=0.05 * dom[2])
    unit_step(case, 1e-13, 0)
    unit_step(case, 1e-13, 1)
    t0 = time.perf_counter()
    for k in range(steps):
        unit_step(case, 1e-13, k)
    dt = time.perf_counter() - t0
    from afh.streamer import cells
    ncell = cells(topo)
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    return {"value": ncell * steps / dt, "unit": "cell-updates/s",
            "cores": threads, "kind": "port",
            "sample": "%d steps on a %d-level uniform tree of %d leaf boxes of "
                      "%d^3 (%d cells), C oracle OpenMP" %
                      (steps, sample_lvls, ncell // nc ** 3, nc, ncell)}


def pmc_traffic(config, kernel="k_gsrb_pair2"):
    """HBM bytes per launch of `kernel` from the PMC passes (scripts/pmc.sh ->
    scripts/pmc_summary.py -> profiles/*pmc*.json, newest round first), or
    None when no summary for this workload and kernel is committed."""
    import glob
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc_*%s.json" % config)),
                       reverse=True):
        if not path.endswith("_pmc_%s.json" % config) and \
                not path.endswith("_%s.json" % config):
            continue
        with open(path) as f:
            d = json.load(f)
        if kernel in d.get("kernel", "") and "hbm_bytes_per_launch" in d:
            return d["hbm_bytes_per_launch"]
    return None


def write_topology(case, config, path, faces_from_phi=False, fused_rhs=False):
    """Boxes, leaves and parents per level, the box size and the species
    counts of the benchmarked tree (scripts/prof_steady.py)."""
    topo = case.topo
    nl = int(topo["highest_lvl"])
    cnt = lambda kind: [len(topo["lvl_%s_%d" % (kind, l)]) for l in range(1, nl + 1)]  # noqa: E731
    if isinstance(case, DriverCase):
        charges = [case.sim.species_charge[n] for n in case.sim.plasma]
    else:
        charges = [-1, 1, -1]  # e, M+, M-
    with open(path, "w") as f:
        json.dump({"config": config, "nc": int(topo["nc"]), "ids": cnt("ids"),
                   "leaves": cnt("leaves"), "parents": cnt("parents"),
                   "n_species": len(charges),
                   "n_charged": sum(1 for q in charges if q != 0),
                   "faces_from_phi": bool(faces_from_phi),
                   "fused_rhs": bool(fused_rhs)}, f)


def _hip_stream():
    """A HIP stream shared by the thread ranks of --shared-stream."""
    import ctypes as C
    hip = C.CDLL("libamdhip64.so")
    st = C.c_void_p()
    if hip.hipStreamCreate(C.byref(st)) != 0:
        raise RuntimeError("hipStreamCreate")
    return st


def local_ranks(lib, config, world, device, coarse, shared_stream=False, grow_cells=0,
                min_level_cells=MIN_LEVEL_CELLS, base=None):
    """--transport local: the sharded workload on `world` thread ranks of this
    process (afh_dist AFH_DIST_LOCAL: pack, host barrier, peer copies,
    unpack), every rank on `device`. The same partition, plans and hooks the
    RCCL transport uses; only the transport differs. Returns (cases, shards,
    group, base): base is the unsharded set-up (driver configs) or None."""
    from afh import capi
    from afh.dist import NativeGroup, NativeShard
    group = NativeGroup(lib, world)
    if config in DRIVER_CONFIGS:
        # (base: a prepared set-up, e.g. one grown tree for several rank counts)
        if base is None:
            base = build_driver_case(lib, device, config, coarse, grow_cells)
        topo = base.af.topology()
        sims = [base.clone(lib, device=device) for _ in range(world)]
        shards = [NativeShard(lib, topo, world, r, transport=capi.DIST_LOCAL, group=group,
                              min_level_cells=min_level_cells) for r in range(world)]
        for sim, sh in zip(sims, shards):
            sim.shard_over(sh)
        cases = [DriverCase(sim) for sim in sims]
    else:
        from afh.tree import uniform_tree
        nc, cgs, lvls, dom = CONFIGS[config]
        topo = uniform_tree(nc, cgs, dom, lvls)
        shards = [NativeShard(lib, topo, world, r, transport=capi.DIST_LOCAL, group=group,
                              min_level_cells=min_level_cells) for r in range(world)]
        # (the set-up fills ghost cells: exchanges, so every rank on its thread)
        cases = run_ranks(shards, lambda r, sh: build_case(lib, config, device, coarse,
                                                           shard=sh))
    if shared_stream:
        st = _hip_stream()
        for c in cases:
            lib.call("tree_set_stream", c.tree.h, st)
    return cases, shards, group, base


def run_ranks(cases, fn):
    """fn(rank, case) on one thread per rank; the results in rank order."""
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(len(cases)) as ex:
        futs = [ex.submit(fn, r, c) for r, c in enumerate(cases)]
        return [f.result() for f in futs]


def dist_stats(lib, shard):
    import ctypes as C
    n, b = C.c_int64(), C.c_int64()
    lib.call("dist_stats", shard.h, C.byref(n), C.byref(b))
    return n.value, b.value


def dist_peer_bytes(lib, shard):
    """(sent, received) bytes per peer so far (afh_dist_peer_bytes)."""
    import ctypes as C
    s, r = (C.c_int64 * shard.n)(), (C.c_int64 * shard.n)()
    lib.call("dist_peer_bytes", shard.h, s, r)
    return np.array(s[:], np.int64), np.array(r[:], np.int64)


def bench_local(args, coarse, base=None):
    """--transport local --gpus N: N thread ranks on ONE device run the
    sharded unit step; not the metric (the ranks share one GPU), but every
    line of the sharded bench except the RCCL calls, plus what a scaling
    projection needs: per rank the leaf cells it owns, the exchanges and the
    bytes per step."""
    import threading
    from afh import capi
    from afh.streamer import cells
    lib = capi.hip_library() if not args.oracle else capi.oracle_library()
    device = -1 if args.oracle else 0
    world = args.gpus
    # one stream for all ranks: no V-cycle graphs (a capture on a stream
    # other threads launch into would take their work too)
    graphs_env = os.environ.get("AFH_GRAPHS")
    if args.shared_stream:
        os.environ["AFH_GRAPHS"] = "0"
    try:
        cases, shards, group, base = local_ranks(lib, args.config, world, device, coarse,
                                                 args.shared_stream, args.grow_cells,
                                                 args.min_level_cells, base)
    finally:
        if args.shared_stream:
            if graphs_env is None:
                os.environ.pop("AFH_GRAPHS", None)
            else:
                os.environ["AFH_GRAPHS"] = graphs_env
    dt = 1e-13
    bar = threading.Barrier(world)
    clock = {}
    peer = {}

    def work(r, case):
        if not args.no_fused_rhs:
            case.fuse_rhs(True, ghosts=False)
        if args.config not in DRIVER_CONFIGS and not args.stored_face_field:
            case.faces_from_phi(True)
        case.field_compute(0, n_vcycles=2)
        for k in range(args.warmup):
            unit_step(case, dt, k)
        case.tree.sync()
        s0 = dist_stats(lib, shards[r])
        p0 = dist_peer_bytes(lib, shards[r])
        bar.wait()
        if r == 0:
            clock["t0"] = time.perf_counter()
            clock["ns0"] = time.clock_gettime_ns(time.CLOCK_MONOTONIC)
        bar.wait()
        for k in range(args.steps):
            unit_step(case, dt, args.warmup + k)
        case.tree.sync()
        bar.wait()
        if r == 0:
            clock["t1"] = time.perf_counter()
            clock["ns1"] = time.clock_gettime_ns(time.CLOCK_MONOTONIC)
        s1 = dist_stats(lib, shards[r])
        p1 = dist_peer_bytes(lib, shards[r])
        peer[r] = ((p1[0] - p0[0]).tolist(), (p1[1] - p0[1]).tolist())
        return s1[0] - s0[0], s1[1] - s0[1]

    try:
        stats = run_ranks(cases, work)
    finally:
        for sh in shards:
            sh.detach()
        group.close()
    elapsed = clock["t1"] - clock["t0"]
    topo = base.af.topology() if base is not None else shards[0].topo
    ncell = cells(topo)
    nc = int(topo["nc"])
    leaves = set()
    for l in range(1, int(topo["highest_lvl"]) + 1):
        leaves.update(int(i) for i in topo["lvl_leaves_%d" % l])
    owned = []
    for sh in shards:
        own = [i for i in leaves if sh.owner[i - 1] == sh.rank]
        owned.append(len(own) * nc ** 3)
    steps = max(1, args.steps)
    return {
        "metric": "cell-updates/s (fluid+MG V-cycle), thread ranks sharing one GPU",
        "value": ncell * args.steps / elapsed, "unit": "cell-updates/s",
        "n_ranks": world, "transport": "local (AFH_DIST_LOCAL thread ranks, one device)",
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1e3 * elapsed / steps,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic", "shared_stream": bool(args.shared_stream),
        "config": {"workload": args.config, "leaf_cells": ncell, "boxes": int(topo["n_boxes"]),
                   "coarse_solve": coarse, "min_level_cells": args.min_level_cells,
                   "partition_level": shards[0].lp},
        "owned_leaf_cells": owned,
        "exchanges_per_step": [n / steps for n, _ in stats],
        "exchange_bytes_per_step": [b / steps for _, b in stats],
        # per rank r, per peer q: bytes sent to q / received from q per step
        "peer_bytes_per_step": [{"sent": [x / steps for x in peer[r][0]],
                                 "received": [x / steps for x in peer[r][1]]}
                                for r in range(world)],
        "note": "not the metric: the ranks share one device; see scripts/project_scaling.py",
        # the timed region on CLOCK_MONOTONIC (a kernel trace's clock)
        "window_ns": [clock["ns0"], clock["ns1"]],
    }


def _roctx():
    """--profile-steps: the ROCTx pause / resume of rocprofv3's
    --selected-regions (collection paused from the start, so that the kernel
    trace of a grown tree holds only the profile window, not the growth)."""
    import ctypes as C
    lib = C.CDLL("/opt/rocm/lib/librocprofiler-sdk-roctx.so")
    lib.roctxProfilerPause.argtypes = lib.roctxProfilerResume.argtypes = [C.c_uint64]
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="s1-64", choices=sorted(CONFIGS))
    ap.add_argument("--coarse", choices=("auto", "pfmg", "direct"), default="auto",
                    help="level-1 solve: the reference's HYPRE PFMG restated "
                         "(AFH_COARSE_PFMG) or our exact separable solve "
                         "(AFH_COARSE_DIRECT); auto: PFMG on s3/s4/s5/2d")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-fused-rhs", action="store_true",
                    help="separate field_set_rhs pass instead of the rhs folded "
                         "into the density update (afh_fluid_set_rhs_output)")
    ap.add_argument("--stored-face-field", action="store_true",
                    help="the gradient stores the face field and the flux reads it, as "
                         "the reference does, instead of the flux evaluating it from phi "
                         "(afh_fluid_set_field_source)")
    ap.add_argument("--replicas", action="store_true",
                    help="N>1: one independent replica per GPU instead of sharding")
    ap.add_argument("--shard", choices=("native", "python"), default="native",
                    help="N>1 sharding: the library's (afh_dist, RCCL transport, owned-box "
                         "storage) or the Python hook over torch.distributed (afh.dist.Shard)")
    ap.add_argument("--transport", choices=("rccl", "local"), default="rccl",
                    help="N>1: one process per GPU over RCCL (torchrun), or local: N thread "
                         "ranks of this process on one GPU (AFH_DIST_LOCAL; a rehearsal of "
                         "the sharded step and the input of the scaling projection)")
    ap.add_argument("--shared-stream", action="store_true",
                    help="--transport local: every rank on one HIP stream (kernels "
                         "serialised, so that a kernel trace gives each rank's own time)")
    ap.add_argument("--min-level-cells", type=int, default=MIN_LEVEL_CELLS,
                    help="N>1: levels holding fewer cells are replicated on every rank, "
                         "not sharded (0: shard from level 2, as before round 6)")
    ap.add_argument("--grow-cells", type=float, default=0,
                    help="driver configs: advance the time loop (untimed) until the tree "
                         "holds this many leaf cells (or --grow-seconds pass), then bench "
                         "on that tree")
    ap.add_argument("--grow-seconds", type=float, default=240.0)
    ap.add_argument("--profile-steps", type=int, default=0,
                    help="after the timed region, this many more unit steps inside a "
                         "ROCTx resume / pause (run under rocprofv3 --selected-regions: "
                         "the trace holds these steps only)")
    ap.add_argument("--oracle", action="store_true",
                    help="--transport local on the C oracle (CPU), for tests")
    ap.add_argument("--graphs", choices=("auto", "on", "off"), default="auto",
                    help="V-cycles replayed as captured hipGraphs (auto: on for the "
                         "small-box configs s1 / s3, whose steps are launch-bound)")
    args = ap.parse_args()
    # (rocprofv3 --selected-regions starts paused; --marker-trace routes the
    # ROCTx calls to it)
    roctx = _roctx() if args.profile_steps else None
    coarse = coarse_choice(args.coarse, args.config)
    if args.transport == "local":
        if args.graphs == "off":
            os.environ["AFH_GRAPHS"] = "0"
        print(json.dumps(bench_local(args, coarse)))
        return

    if args.graphs == "off":
        os.environ["AFH_GRAPHS"] = "0"  # read by afh_mg_create
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        dist.init_process_group("nccl" if torch.cuda.is_available() else "gloo")
        if torch.cuda.is_available():
            torch.cuda.set_device(local)

    from afh import capi
    two_d = len(CONFIGS[args.config][3]) == 2
    lib = capi.hip_library_2d() if two_d else capi.hip_library()
    sharded = world > 1 and not args.replicas
    if two_d and sharded:
        raise SystemExit("the 2-D build does not shard (--replicas runs one per GPU)")
    if args.config in DRIVER_CONFIGS:
        sim = build_driver_case(lib, local, args.config, coarse, int(args.grow_cells),
                                args.grow_seconds)
        if sharded:
            # every rank built the same AMR tree (the set-up is deterministic);
            # its part of it continues sharded, exchanges over RCCL
            from afh.dist import NativeShard, rccl_comm
            sim.shard_over(NativeShard(lib, sim.af.topology(), world, rank,
                                       transport=capi.DIST_RCCL,
                                       comm=rccl_comm(lib, rank, world, local),
                                       min_level_cells=args.min_level_cells))
        case = DriverCase(sim)
    else:
        case = build_case(lib, args.config, local, coarse,
                          (world, rank, args.shard) if sharded else None,
                          min_level_cells=args.min_level_cells)
    from afh.streamer import cells
    ncell = cells(case.topo)  # leaf cells of the whole tree
    dt = 1e-13

    if not args.no_fused_rhs and not two_d:
        case.fuse_rhs(True, ghosts=False)
    if args.config in DRIVER_CONFIGS:
        if args.stored_face_field and case.sim.faces_from_phi:
            raise SystemExit("--stored-face-field: set AFH_FACES_FROM_PHI=0 for the driver configs")
        faces_from_phi = case.sim.faces_from_phi
    else:
        faces_from_phi = (not args.stored_face_field and not two_d and
                          os.environ.get("AFH_FACES_FROM_PHI", "1") != "0")
        if faces_from_phi:
            case.faces_from_phi(True)
    case.field_compute(0, n_vcycles=2)  # initial potential (untimed)
    for k in range(args.warmup):
        unit_step(case, dt, k)
    case.tree.sync()

    def barrier():
        if dist is not None:
            dist.barrier()

    # timed region: K steps. The dominant kernel (the fused red+black
    # Gauss-Seidel pair on the leaf level) is timed with HIP events on the
    # tree's stream (afh_profile_*) over the same region -- unless V-cycles
    # are replayed as hipGraphs (kernel timing needs eager launches): then
    # over two eager unit steps right after the timed region
    import ctypes as C
    graphs = args.graphs == "on" or (args.graphs == "auto" and args.config != "s1-64")
    if two_d:
        # the 2-D library replays its V-cycles as hipGraphs by itself
        # (AFH2_GRAPHS, default on: nothing is profiled in the timed region);
        # its kernels are timed after the timed region (launches of a few us
        # each, the events around them would weigh on the step clock)
        graphs = os.environ.get("AFH2_GRAPHS", "1") != "0"
    elif not graphs:
        lib.call("profile_enable", case.tree.h, capi.PROF_GSRB_PAIR)
    barrier()
    case.tree.sync()
    t0 = time.perf_counter()
    ns0 = time.clock_gettime_ns(time.CLOCK_MONOTONIC)
    last_res = None
    for k in range(args.steps):
        last = unit_step(case, dt, args.warmup + k)
        if last[0]:
            last_res = last[0]  # (stage 1 returns no residual: deferred)
    case.tree.sync()
    barrier()
    elapsed = time.perf_counter() - t0
    ns1 = time.clock_gettime_ns(time.CLOCK_MONOTONIC)
    if graphs or two_d:
        lib.call("profile_enable", case.tree.h, capi.PROF_GSRB if two_d else capi.PROF_GSRB_PAIR)
        for k in range(2):
            unit_step(case, dt, args.warmup + args.steps + k)
        case.tree.sync()
    ms, nl, by = C.c_double(), C.c_int64(), C.c_double()
    lib.call("profile_read", case.tree.h, C.byref(ms), C.byref(nl), C.byref(by))
    kname = ("k_gsrb_pair2<%d,%d>" % (CONFIGS[args.config][0], CONFIGS[args.config][0])
             if CONFIGS[args.config][0] > 16 else "k_gsrb_pair_box<%d>" % CONFIGS[args.config][0])
    if two_d:
        kname = ("k2_pair_box (red+black pair, levels of >= 256 boxes, 24 B/cell)"
                 if os.environ.get("AFH_PAIR2D", "1") != "0" else
                 "k2_gsrb (half sweep, levels of >= 256 boxes, 16 B/cell)")
    if nl.value == 0 and two_d:
        # no level of >= 256 boxes runs the pair in the timed window: the
        # split half-sweep on every level
        kname = "k2_gsrb (half sweep, 16 B/cell)"
        lib.call("profile_enable", case.tree.h, capi.PROF_GSRB)
        for k in range(2):
            unit_step(case, dt, args.warmup + args.steps + 2 + k)
        case.tree.sync()
        lib.call("profile_read", case.tree.h, C.byref(ms), C.byref(nl), C.byref(by))
    if nl.value == 0 and two_d:
        # no level of >= 256 boxes at all (config 1's set-up tree): the flux
        # over every leaf (48 B/cell: the densities' two ghost layers read,
        # the face fluxes written) is the line
        kname = "k2_flux (all leaves, 48 B/cell)"
        lib.call("profile_enable", case.tree.h, capi.PROF_FLUX)
        for k in range(2):
            unit_step(case, dt, args.warmup + args.steps + 4 + k)
        case.tree.sync()
        lib.call("profile_read", case.tree.h, C.byref(ms), C.byref(nl), C.byref(by))
    if nl.value == 0 and not two_d:
        # no level runs the fused pair (too few boxes per level, or
        # electrode stencils): the split half-sweep k_gsrb is the smoother
        kname = "k_gsrb (half-sweep, 16 B/cell)"
        graphs = True
        lib.call("profile_enable", case.tree.h, capi.PROF_GSRB)
        for k in range(2):
            unit_step(case, dt, args.warmup + args.steps + 2 + k)
        case.tree.sync()
        lib.call("profile_read", case.tree.h, C.byref(ms), C.byref(nl), C.byref(by))
    # config 1: the level-1 solve (k2_cs_pfmg) per unit step over two eager
    # steps, so that the line can also be read without it -- the reference's
    # CPU timing cannot run it (HYPRE is absent)
    cs_ms_step = None
    if two_d:
        lib.call("profile_enable", case.tree.h, capi.PROF_CS)
        k0 = args.warmup + args.steps + 8
        for k in range(2):
            unit_step(case, dt, k0 + k)
        case.tree.sync()
        cms, cnl, cby = C.c_double(), C.c_int64(), C.c_double()
        lib.call("profile_read", case.tree.h, C.byref(cms), C.byref(cnl), C.byref(cby))
        lib.call("profile_enable", case.tree.h, 0)
        cs_ms_step = cms.value / 2
    # the fused species step (k_fe_lds, 64^3 boxes) over two eager unit steps
    # after the timed region -- one Heun stage of each kind: when it takes
    # more of a step than the smoother it is the dominant kernel of the line
    fe = None
    if not two_d and not sharded and CONFIGS[args.config][0] == 64:
        lib.call("profile_enable", case.tree.h, capi.PROF_FE)
        # the Heun sequence continued (after the smoother's two eager steps
        # when V-cycle graphs ran): the rhs folded by the previous update
        # stays valid, as in the timed region
        k0 = args.warmup + args.steps + (2 if graphs else 0)
        for k in range(2):
            unit_step(case, dt, k0 + k)
        case.tree.sync()
        fms, fnl, fby = C.c_double(), C.c_int64(), C.c_double()
        lib.call("profile_read", case.tree.h, C.byref(fms), C.byref(fnl), C.byref(fby))
        lib.call("profile_enable", case.tree.h, 0)
        if fnl.value:
            fe = (fms.value, fnl.value, fby.value)
    if roctx:
        lib.call("profile_enable", case.tree.h, 0)
        k0 = args.warmup + args.steps + 6  # even: the window starts on a Heun stage 1
        case.tree.sync()
        roctx.roctxProfilerResume(0)
        for k in range(args.profile_steps):
            unit_step(case, dt, k0 + k)
        case.tree.sync()
        roctx.roctxProfilerPause(0)

    if dist is not None:
        import torch
        tt = torch.tensor([elapsed], dtype=torch.float64,
                          device="cuda" if torch.cuda.is_available() else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    if rank == 0 and os.environ.get("AFH_BENCH_TOPO"):
        # the run's topology for scripts/prof_steady.py's byte model
        write_topology(case, args.config, os.environ["AFH_BENCH_TOPO"], faces_from_phi,
                       not args.no_fused_rhs and not two_d)

    if rank == 0:
        avg_s = ms.value / 1e3 / max(1, nl.value)
        bytes_per_launch = by.value / max(1, nl.value)
        achieved = bytes_per_launch / avg_s / 1e9 if avg_s > 0 else 0.0
        out = {
            "metric": "cell-updates/s (fluid+MG V-cycle)",
            "value": ncell * args.steps * (1 if sharded else world) / elapsed,
            "unit": "cell-updates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "strong" if sharded else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": args.config, "n_cell": CONFIGS[args.config][0],
                       "leaf_cells": ncell, "boxes": int(case.topo["n_boxes"]),
                       "levels": int(case.topo["highest_lvl"]),
                       "coarse_solve": {"pfmg": "HYPRE PFMG restated (tol 1e-6, <= 50 it.)",
                                        "direct": "exact separable"}[coarse],
                       "fused_rhs": "interior" if not args.no_fused_rhs else False,
                       "face_field": "from phi in the flux" if faces_from_phi else "stored",
                       "vcycle_graphs": graphs,
                       "parallelism": ("box-shard-%d-%s" % (world, args.shard)) if sharded else
                       ("replica-per-gpu" if world > 1 else "single-gpu")},
            "roofline": {"bound": "hbm",
                         "kernel": kname,
                         "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": pmc_traffic(args.config),
                         "avg_launch_us": avg_s * 1e6,
                         "algorithmic_bytes_per_launch": bytes_per_launch,
                         "launches": nl.value,
                         "timed_over": ("2 eager unit steps after the timed region"
                                        if graphs or two_d else "the timed region")},
            "last_residual": last_res[-1] if last_res else None,
            # one FAS V(2,2)-cycle per step (SURVEY.md 8(d) reports both)
            "vcycles_per_s": args.steps / elapsed,
            # the timed region on CLOCK_MONOTONIC (a kernel trace's clock;
            # scripts/project_scaling.py)
            "window_ns": [ns0, ns1],
        }
        if fe is not None:
            # the fused species step per unit step against the smoother's
            # (its launches over the timed region): the larger is the line
            fe_ms, fe_nl, fe_by = fe
            pair_ms_step = ms.value / (2 if graphs else max(1, args.steps))
            fe_ms_step = fe_ms / 2
            fe_s = fe_ms / 1e3 / fe_nl
            fe_ach = fe_by / fe_nl / fe_s / 1e9
            fe_line = {"bound": "hbm",
                       "kernel": "k_fe_lds<64> (flux + density update fused; 72 / 96 B/cell "
                                 "for one / two previous states)",
                       "achieved": fe_ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                       "frac": fe_ach / HBM_PEAK_GBS,
                       "traffic": pmc_traffic(args.config, "k_fe_lds"),
                       "avg_launch_us": fe_s * 1e6,
                       "algorithmic_bytes_per_launch": fe_by / fe_nl, "launches": fe_nl,
                       "ms_per_step": fe_ms_step,
                       "timed_over": "2 eager unit steps after the timed region (one per "
                                     "Heun stage)"}
            out["roofline"]["ms_per_step"] = pair_ms_step
            if fe_ms_step > pair_ms_step:
                out["roofline_smoother"] = out["roofline"]
                out["roofline"] = fe_line
            else:
                out["roofline_species"] = fe_line
        if two_d:
            # BASELINE's config 1 (streamer_2d.cfg), not the headline: its
            # roofline line is the 2-D fused pair on levels of >= 256 boxes
            out["config"]["ndim"] = 2
            out["config"]["fused_rhs"] = False
            out["config"]["chemistry"] = "air_chemistry_v1 (8 species, 25 reactions)"
            # the line without the level-1 solve, as the reference is timed
            ms_x = 1e3 * elapsed / args.steps - cs_ms_step
            out["level1_solve_ms_per_step"] = cs_ms_step
            out["ms_per_step_without_level1"] = ms_x
            out["value_without_level1"] = ncell / (ms_x * 1e-3)
            # a set-up tree of 17.5 K cells is launch-bound: no kernel's HBM
            # fraction says anything about it
            out["roofline"]["note"] = ("launch-bound configuration (a hundred-odd kernels "
                                       "per step, microseconds each): the fraction is not a "
                                       "measure of kernel quality here; see launch_bound")
            # what bounds it instead: launches per step and their mean time,
            # from the committed steady-step kernel trace of this config
            # (scripts/prof_cfg.sh -> scripts/prof_steady.py)
            sp = os.path.join(REPO, "profiles", "r06_steady_2d.json")
            if os.path.exists(sp):
                st = json.load(open(sp))
                out["launch_bound"] = {
                    "launches_per_step": st["launches_per_step"],
                    "us_per_launch": 1e3 * st["busy_ms_per_step"] / st["launches_per_step"],
                    "gap_share": st["gap_share"],
                    "source": "profiles/r06_steady_2d.json (rocprofv3 kernel trace of this "
                              "command, the timed window's unit steps)"}
            # the C oracle is 3-D: the reference's own 2-D code on the same
            # set-up tree (scripts/record_setup_state.py -> ref_timing's
            # record mode), timed in the build container -- its binary does
            # not travel to the GPU box
            ref = json.load(open(os.path.join(REPO, "profiles", "r06_ref_cpu_timing_2d.json")))
            best = max(ref["threads"].items(), key=lambda kv: kv[1]["cell_updates_per_s"])
            out["cpu_baseline"] = {
                "value": best[1]["cell_updates_per_s"], "unit": "cell-updates/s",
                "cores": int(best[0]), "kind": "reference",
                "compare_with": "value_without_level1",
                "sample": "the reference's 2-D forward_euler + one V(2,2)-cycle without the "
                          "level-1 solve on streamer_2d.cfg's own set-up tree (%d boxes, %d "
                          "leaf cells: the tree of this line), measured in the build "
                          "container (profiles/r06_ref_cpu_timing_2d.json), not on this host"
                          % (ref["boxes"], ref["cells"])}
            if ref["cells"] != ncell:
                out["cpu_baseline"]["warning"] = "timed on a %d-cell tree, this line %d" % (
                    ref["cells"], ncell)
        if args.config in DRIVER_CONFIGS:
            g = sim.grown
            out["config"]["tree"] = {"leaf_cells_setup": g["leaf_cells_initial"],
                                     "grown_steps": g["steps"],
                                     "grown_to_time_s": g["time_s"],
                                     "highest_lvl": int(sim.af.highest_lvl)}
        if sharded:
            out["exchanges_per_step"] = case.shard.n_exchanges / max(1, args.steps + args.warmup + 1)
        if args.config == "s3":
            out["config"]["chemistry"] = "air_chemistry_v2 (9 species, 25 reactions)"
        if args.config == "s4":
            out["config"]["chemistry"] = "air_chemistry_v2 (9 species, 25 reactions)"
            out["config"]["electrode"] = ("grounded rod (0.5,0.5,0)-(0.5,0.5,0.15) L, r = 1 mm, "
                                          "%d electrode boxes" % len(sim.electrode_ids))
            if coarse == "direct":
                out["config"]["coarse_solve"] = "electrode level 1: dense inverse product (one 8^3 box)"
        if args.config == "s5":
            out["config"]["chemistry"] = "sprite_chemistry_v0 (10 species, 12 reactions)"
            out["config"]["gas_density"] = "variable (3d_sprite m_user: 2.5e25 exp(-z/7.2 km))"
            out["config"]["photoionization"] = ("Helmholtz Bourdon-3, every %d time steps"
                                                % sim.c.i("photoi%per_steps"))
        if not args.no_cpu_baseline and world == 1 and not two_d:
            out["cpu_baseline"] = (cpu_baseline_driver(sim, config=args.config)
                                   if args.config in DRIVER_CONFIGS else
                                   cpu_baseline(args.config, coarse))
        print(json.dumps(out))
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
