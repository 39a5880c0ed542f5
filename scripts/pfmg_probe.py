"""The level-1 solve (k_cs_pfmg) of the driver configurations, timed alone.

usage: python scripts/pfmg_probe.py OUT.json [configs...] (default s3 s4 s5)

Builds each configuration's set-up tree (bench.build_driver_case), runs
field_compute a few times eagerly (AFH_GRAPHS=0) with the AFH_PROF_CS events
around every k_cs_pfmg launch, and writes the mean launch time, the PFMG
iteration count. With AFH_HIP_LIB naming a -DAFH_PFMG_TIMING build
of the library, the kernel also prints its per-operation clock sums
(PFTIME lines)."""
import ctypes as C
import json
import os
import sys
import time

os.environ.setdefault("AFH_GRAPHS", "0")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from afh import capi  # noqa: E402


def probe(lib, config, reps=6):
    sim = bench.build_driver_case(lib, 0, config)
    t = sim.tree
    sim.field_compute(0, True)  # the hierarchy's set-up outside the window
    t.sync()
    lib.call("profile_enable", t.h, capi.PROF_CS)
    t0 = time.perf_counter()
    for _ in range(reps):
        sim.field_compute(0, True)
    t.sync()
    wall = (time.perf_counter() - t0) / reps
    ms, nl, by = C.c_double(), C.c_int64(), C.c_double()
    lib.call("profile_read", t.h, C.byref(ms), C.byref(nl), C.byref(by))
    lib.call("profile_enable", t.h, 0)
    return {"config": config, "launches": nl.value,
            "us_per_launch": 1e3 * ms.value / max(nl.value, 1),
            "iterations": sim.mg.coarse_iterations(),
            "field_compute_wall_ms": 1e3 * wall}


def main():
    out = sys.argv[1]
    configs = sys.argv[2:] or ["s3", "s4", "s5"]
    lib = capi.hip_library()
    rows = [probe(lib, c) for c in configs]
    for r in rows:
        print(json.dumps(r), flush=True)
    json.dump(rows, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
