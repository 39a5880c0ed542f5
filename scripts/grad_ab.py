#!/usr/bin/env python3
"""Interleaved A/B of field_from_potential's gradient kernel variants on the
S1-64 tree, in one process: one afh_mg per variant (AFH_GRAD_NT read at
afh_mg_create), compute_phi_gradient calls alternating between them, timed
on the host around a synchronised batch. The outputs (face fields and |E|)
must be bitwise equal across variants. Usage: grad_ab.py 1 0."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "afivo-streamer_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import bench  # noqa: E402
from afh import capi  # noqa: E402
from afh.model import Multigrid  # noqa: E402
from afh.streamer import FV, IV  # noqa: E402


def main():
    variants = sys.argv[1:] or ["0"]
    lib = capi.hip_library()
    case = bench.build_case(lib, os.environ.get("CFG", "s1-64"), 0, 0)
    case.field_compute(0, n_vcycles=1)
    mgs = []
    for v in variants:
        os.environ["AFH_GRAD_NT"] = v
        mgs.append(Multigrid(case.tree, IV["phi"], IV["rhs"], IV["tmp"], coarse_cycles=0))
    os.environ.pop("AFH_GRAD_NT")
    ref = None
    for v, mg in zip(variants, mgs):
        case.tree.put_fc(FV["field"], np.zeros(case.tree.fc_shape))
        mg.compute_phi_gradient(FV["field"], -1.0, IV["efld"])
        out = (case.tree.get_fc(FV["field"]), case.tree.get_cc(IV["efld"]))
        if ref is None:
            ref = out
        else:
            same = all(np.array_equal(a, b) for a, b in zip(out, ref))
            print("variant %s bitwise equal to %s: %s" % (v, variants[0], same), flush=True)
    tot = [0.0] * len(variants)
    reps = int(os.environ.get("REPS", "10"))
    for rnd in range(int(os.environ.get("ROUNDS", "5"))):
        for n, mg in enumerate(mgs):
            case.tree.sync()
            t0 = time.perf_counter()
            for _ in range(reps):
                mg.compute_phi_gradient(FV["field"], -1.0, IV["efld"])
            case.tree.sync()
            tot[n] += time.perf_counter() - t0
    for v, t in zip(variants, tot):
        print("AFH_GRAD_NT=%-3s %.1f us per gradient" %
              (v, 1e6 * t / (reps * int(os.environ.get("ROUNDS", "5")))), flush=True)


if __name__ == "__main__":
    main()
