#!/usr/bin/env python3
"""Timing probe: S5's photoionization (photoi_set_src: the Zheleznyak source +
photoi_helmh_compute's three Bourdon-3 Helmholtz FMG solves) on its set-up
tree, against one unit step. Prints the FMG cycles per mode and ms per call.
Usage: photoi_probe.py [reps]
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "afivo-streamer_amd"))
import bench  # noqa: E402
from afh import capi  # noqa: E402


def main(reps=5):
    sim = bench.build_driver_case(capi.hip_library(), 0, "s5", "pfmg")
    case = bench.DriverCase(sim)
    case.fuse_rhs(True, ghosts=False)
    case.field_compute(0)
    for k in range(4):
        bench.unit_step(case, 1e-13, k)
    sim.tree.sync()
    out = {"photoi_ms": [], "n_fmg": [], "unit_step_ms": []}
    for r in range(reps):
        t0 = time.perf_counter()
        n = sim.photoi_set_src()
        sim.tree.sync()
        out["photoi_ms"].append(1e3 * (time.perf_counter() - t0))
        out["n_fmg"].append([int(x) for x in n])
        t0 = time.perf_counter()
        for k in range(2):
            bench.unit_step(case, 1e-13, k)
        sim.tree.sync()
        out["unit_step_ms"].append(1e3 * (time.perf_counter() - t0) / 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 5)
