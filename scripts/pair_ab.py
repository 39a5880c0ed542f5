#!/usr/bin/env python3
"""Interleaved A/B timing of k_gsrb_pair2 variants on the S1-64 tree, in one
process: one afh_mg per variant (AFH_GSRB_PAIR_* read at afh_mg_create),
V-cycles alternating between them, the leaf-level pair timed with HIP
events (afh_profile_*). Usage: pair_ab.py VAR1 VAR2 ... ("default" = none),
each VAR a comma-separated list of NAME=VALUE."""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "afivo-streamer_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import bench  # noqa: E402
from afh import capi  # noqa: E402
from afh.model import Multigrid  # noqa: E402
from afh.streamer import IV  # noqa: E402


def main():
    variants = sys.argv[1:] or ["default"]
    lib = capi.hip_library()
    case = bench.build_case(lib, os.environ.get("CFG", "s1-64"), 0, 0)
    case.field_compute(0, n_vcycles=1)
    mgs = []
    keys = set()
    for v in variants:
        env = {} if v == "default" else dict(kv.split("=") for kv in v.split(","))
        keys |= set(env)
        for k in keys:
            os.environ.pop(k, None)
        os.environ.update(env)
        mgs.append(Multigrid(case.tree, IV["phi"], IV["rhs"], IV["tmp"], coarse_cycles=0))
    for k in keys:
        os.environ.pop(k, None)
    tot = [[0.0, 0] for _ in variants]
    for rnd in range(int(os.environ.get("ROUNDS", "6"))):
        for n, mg in enumerate(mgs):
            lib.call("profile_enable", case.tree.h, capi.PROF_GSRB_PAIR)
            for _ in range(2):
                lib.call("mg_fas_vcycle", mg.h, 0, 0)
            case.tree.sync()
            ms, nl, by = C.c_double(), C.c_int64(), C.c_double()
            lib.call("profile_read", case.tree.h, C.byref(ms), C.byref(nl), C.byref(by))
            if rnd > 0:
                tot[n][0] += ms.value
                tot[n][1] += nl.value
        print("round", rnd, flush=True)
    for v, (ms, nl) in zip(variants, tot):
        us = 1e3 * ms / max(1, nl)
        print("%-40s %8.1f us per pair launch (avg of %d; all levels)" % (v, us, nl))


if __name__ == "__main__":
    main()
