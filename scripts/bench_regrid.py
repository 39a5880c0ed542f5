#!/usr/bin/env python3
"""Regrid on the S1-64 workload (512 leaf boxes of 64^3): the device
refinement criterion (afh_refine_flags: default_refinement + cell_to_ref_flags
summaries over 134 M cells) and the data movement of one regrid that refines
the 8 leaf boxes around the seed (64 new boxes of 64^3, afh_tree_regrid in
place: auto_prolong + ghost cells). Prints one JSON line."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "afivo-streamer_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import numpy as np  # noqa: E402

import bench  # noqa: E402
from afh import capi  # noqa: E402
from afh.streamer import IV, StreamerCase, seed_state, tables_from  # noqa: E402
from afh.tree import build_tree, uniform_tree  # noqa: E402
import golden  # noqa: E402


def main():
    lib = capi.hip_library()
    nc, cgs, lvls, dom = bench.CONFIGS["s1-64"]
    topo = uniform_tree(nc, cgs, dom, lvls)
    c = 0.5 * np.asarray(dom)
    # refine the 8 leaf boxes touching the centre (seed)
    new_topo = build_tree(nc, cgs, dom, lvls, refine=lambda lvl, r0, r1: (
        lvl == lvls and np.all(r0 <= c) and np.all(r1 >= c)))
    td, chem = tables_from(golden.load("uni8"))
    case = StreamerCase(lib, topo, td, chem, -dom[2] * (-2.5e6), coarse_cycles=0,
                        box_capacity=int(new_topo["n_boxes"]))
    seed_state(case, width=0.05 * dom[2])
    t = case.tree
    for sp in ("e", "pos", "neg"):
        t.set_cc_prolong(IV[sp], capi.PROLONG_LIMIT, capi.LIM_GMINMOD43)
    t.set_cc_prolong(IV["efld"], capi.PROLONG_LINEAR)
    t.set_cc_prolong(IV["phi"], capi.PROLONG_LINEAR)
    case.field_compute(0, n_vcycles=2)
    d = capi.RefineDesc()
    d.i_electron, d.i_efld, d.td_alpha_col, d.td_eta_col = IV["e"], IV["efld"], 3, 4
    d.buffer_width = 4
    d.adx, d.adx_fac, d.min_dens = 1.0, 1.0, -1e99
    d.derefine_dx, d.max_dx, d.min_dx, d.electrode_dx = 1e-4, 1e-3, 1e-7, 1e99
    case.fluid.refine_flags(d)  # warm-up
    t.sync()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        flags, masks = case.fluid.refine_flags(d)
    t_flags = (time.perf_counter() - t0) / reps
    t.sync()
    t0 = time.perf_counter()
    t2 = t.regrid(new_topo)
    t2.sync()
    t_regrid = time.perf_counter() - t0
    n_new = int(new_topo["n_boxes"]) - int(topo["n_boxes"])
    print(json.dumps({
        "workload": "s1-64", "leaf_cells": 512 * nc ** 3,
        "refine_flags_ms": 1e3 * t_flags,
        "refine_flags_cells_per_s": 585 * nc ** 3 / t_flags,
        "flag_counts": {str(k): int(v) for k, v in zip(*np.unique(flags, return_counts=True))},
        "regrid_in_place_ms": 1e3 * t_regrid, "new_boxes": n_new,
        "regrid_new_cells_per_s": n_new * nc ** 3 / t_regrid,
        "auto_vars": 5}))


if __name__ == "__main__":
    main()
