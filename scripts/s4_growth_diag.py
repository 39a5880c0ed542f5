#!/usr/bin/env python3
"""Diagnostic: the S4 (rod electrode) time loop on the device from its
set-up, logging every N steps the time, dt, the four dt limits of the last
forward_euler (CFL, diffusion, dielectric relaxation, chemistry), the leaf
cells, max |E| and max n_e; stops at the end time, at MAX_S seconds or at the
driver's "dt too small". Usage: s4_growth_diag.py [config] [coarse] [max_s]
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


def main(config="s4", coarse="pfmg", max_s=60.0, every=250):
    oracle = os.environ.get("ORACLE") == "1"  # the C oracle on the CPU (a checker run)
    sim = bench.build_driver_case(capi.oracle_library() if oracle else capi.hip_library(),
                                  -1 if oracle else 0, config, coarse)
    last = {}
    fe = sim.forward_euler

    def rec(dt, s_deriv, s_prev, w_prev, s_out, i_step, n_steps):
        if i_step > 1:
            sim.field_compute(s_deriv, True)
        lim = sim.fluid.forward_euler(dt, s_deriv, s_prev, w_prev, s_out, i_step == n_steps)
        last["lim"] = [lim[0] * sim.cfl, lim[1], lim[2], lim[3]]
        return min(sim.dt_max, min(last["lim"]))
    sim.forward_euler = rec
    assert fe is not None
    sim.output_cnt = 0
    sim.output_write()
    sim.time_last_output = sim.time
    i_e = sim.densities[0]
    rows, t0, n, err = [], time.perf_counter(), 0, None

    def row():
        e = sim.tree.get_cc(sim.i_efld)
        ne = sim.tree.get_cc(i_e)
        return {"it": sim.it, "time": sim.time, "dt": sim.global_dt,
                "lim": last.get("lim"), "leaf_cells": sim.af.n_leaf_cells(),
                "max_E": float(abs(e).max()), "max_ne": float(ne.max()),
                "rejected": sim.n_steps_rejected, "lvl": int(sim.af.highest_lvl)}
    hist = []
    try:
        while time.perf_counter() - t0 < max_s:
            if not sim.step():
                break
            n += 1
            hist.append((sim.it, sim.time, sim.global_dt, last.get("lim")))
            hist = hist[-40:]
            if n % every == 0:
                rows.append(row())
                print(json.dumps(rows[-1]), flush=True)
    except RuntimeError as ex:
        err = str(ex)
    rows.append(row())
    out = {"config": config, "coarse": coarse, "steps": n, "error": err,
           "rows": rows, "last_steps": hist}
    print(json.dumps(rows[-1]), flush=True)
    print("ERROR", err, flush=True)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "diag_%s_%s_%s%s.json" %
                           (config, coarse, os.environ.get("TAG", "a"),
                            "_oracle" if oracle else "")), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0] if a else "s4", a[1] if len(a) > 1 else "pfmg",
         float(a[2]) if len(a) > 2 else 60.0)
