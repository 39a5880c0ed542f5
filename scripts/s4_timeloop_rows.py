#!/usr/bin/env python3
"""Config 4's time loop (afh.driver, from the reference's set-up) writing
output_regression_log rows every OUT_DT seconds to END (default 2.5 ns,
every 0.05 ns), for comparison with the reference's own streamer.f90 run
through the shim on the C oracle (oracle/_ref/dropin_streamer with the same
end_time / output%dt, build container). Usage:
  s4_timeloop_rows.py <out.json> [end_time] [output_dt] [max_seconds]
On the GPU box (libafivo_hip); ORACLE=1: the C oracle on the CPU."""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "afivo-streamer_amd"))
from afh import capi, decks  # noqa: E402
from afh.driver import Simulation  # noqa: E402


def main(out, end_time=2.5e-9, output_dt=0.05e-9, max_s=900.0):
    oracle = os.environ.get("ORACLE") == "1"
    g = dict(decks.load("case_s4"))
    g["end_time"] = np.array([float(end_time)])
    g["output%dt"] = np.array([float(output_dt)])
    lib = capi.oracle_library() if oracle else capi.hip_library()
    sim = Simulation(lib, g, device=-1 if oracle else 0, coarse_cycles=50, coarse_tol=1e-6,
                     coarse_mode=capi.COARSE_PFMG)
    sim.start()
    t0, err, n = time.perf_counter(), None, 0
    t_print = t0
    try:
        while time.perf_counter() - t0 < float(max_s) and sim.step():
            n += 1
            if time.perf_counter() - t_print > 20:
                t_print = time.perf_counter()
                print("step %d t %.4e dt %.3e rows %d" % (sim.it, sim.time, sim.global_dt,
                                                        len(sim.log)), flush=True)
    except RuntimeError as ex:
        err = str(ex)
    res = {"steps": n, "it": sim.it, "time": sim.time, "dt": sim.global_dt, "error": err,
           "end_time": float(end_time), "output_dt": float(output_dt),
           "leaf_cells": sim.af.n_leaf_cells(), "seconds": time.perf_counter() - t0,
           "rows": np.array(sim.log).tolist()}
    json.dump(res, open(out, "w"))
    print({k: v for k, v in res.items() if k != "rows"}, flush=True)


if __name__ == "__main__":
    main(*sys.argv[1:])
