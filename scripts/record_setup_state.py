#!/usr/bin/env python3
"""The set-up state of a driver configuration (bench.py's build_driver_case:
the reference's set_initial_conditions on the device) as a record of
oracle/harness/replay_step.f90's format -- the topology and every cell and
face variable -- for oracle/_ref[/2d]/ref_timing's record mode, which times
the reference's own code on that very tree (config 1's
cpu_baseline on the tree its GPU line runs).

Usage: record_setup_state.py <config> <out.bin>   (on the GPU box)
"""
import os
import struct
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def write_record(path, sim):
    af, t = sim.af, sim.tree
    hid = af.highest_id
    used = [b for b in range(1, hid + 1) if af.in_use[b]]
    with open(path, "wb") as f:
        f.write(struct.pack("<4i", hid, sim.n_var_cell, sim.n_var_face, af.nc))
        for b in range(1, hid + 1):
            ix = (tuple(af.ix[b]) + (0, 0, 0))[:3] if af.in_use[b] else (0, 0, 0)
            f.write(struct.pack("<6i", af.parent[b], af.lvl[b], *ix, int(af.in_use[b])))
        # (the stage fields: ref_timing skips them)
        f.write(struct.pack("<ddii", 1e-13, sim.time, 0, 1))
        f.write(struct.pack("<i", 0))
        f.write(struct.pack("<d", 1.0))
        f.write(struct.pack("<i", 1))
        for iv in range(1, sim.n_var_cell + 1):
            a = t.get_cc(iv)
            for b in used:
                f.write(np.ascontiguousarray(a[b - 1]).tobytes())
        for iv in range(1, sim.n_var_face + 1):
            a = t.get_fc(iv)
            for b in used:
                f.write(np.ascontiguousarray(a[b - 1]).tobytes())
    return len(used), af.n_leaf_cells()


def main(config, out):
    from afh import capi
    two_d = len(bench.CONFIGS[config][3]) == 2
    lib = capi.hip_library_2d() if two_d else capi.hip_library()
    sim = bench.build_driver_case(lib, 0, config, bench.coarse_choice("auto", config))
    n_boxes, cells = write_record(out, sim)
    print({"config": config, "boxes": n_boxes, "leaf_cells": cells, "record": out})


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
