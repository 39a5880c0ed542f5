"""Does the S1-64 pair's speed mode change with the allocation inside one
process? Builds the S1-64 case N times in one process (freeing the previous
tree), times the leaf pair (HIP events, afh_profile_*) and the step clock over
a few unit steps each. Usage: python scripts/placement_probe.py [N]"""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from afh import capi  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
lib = capi.hip_library()
for r in range(n):
    case = bench.build_case(lib, "s1-64", 0, 0)
    case.fuse_rhs(True, ghosts=False)
    case.faces_from_phi(True)
    case.field_compute(0, n_vcycles=2)
    for k in range(2):
        bench.unit_step(case, 1e-13, k)
    case.tree.sync()
    lib.call("profile_enable", case.tree.h, capi.PROF_GSRB_PAIR)
    t0 = time.perf_counter()
    for k in range(4):
        bench.unit_step(case, 1e-13, 2 + k)
    case.tree.sync()
    ms = (time.perf_counter() - t0) * 1e3 / 4
    t_ms, nl, by = C.c_double(), C.c_int64(), C.c_double()
    lib.call("profile_read", case.tree.h, C.byref(t_ms), C.byref(nl), C.byref(by))
    print("allocation %d: %.3f ms/step, pair %.1f us (%d launches)"
          % (r, ms, t_ms.value * 1e3 / max(1, nl.value), nl.value), flush=True)
    case.tree.close()
