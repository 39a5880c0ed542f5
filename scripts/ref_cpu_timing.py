#!/usr/bin/env python3
"""Reference CPU timings for BASELINE.md (build container only).

Times, on the host cores with OMP_NUM_THREADS = 1 and 8:
* the reference's own code (oracle/_ref/ref_timing, compiled from
  /root/reference): forward_euler (flux + update with chemistry) per Heun
  sub-step and one FAS V(2,2)-cycle without the level-1 solve, on
  - S1: 512 leaf boxes of 16^3 (4 levels, 16^3 coarse grid),
  - the S1-64 sample: 64 leaf boxes of 64^3 (3 levels, 64^3 coarse grid),
  both 16 mm cubes with the regression test's old-style air model and seed
  (programs/standard_3d/tests/test_3d.cfg);
* the C oracle (oracle/lib/libafo.so, OpenMP) on the bench's unit step of
  the same trees (bench.cpu_baseline).
Writes profiles/<tag>_ref_cpu_timing.json.

    python3 scripts/ref_cpu_timing.py r02
"""
import json
import os
import platform
import resource
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTS = "/root/reference/programs/standard_3d/tests"
EXE = os.path.join(REPO, "oracle", "_ref", "ref_timing")
CASES = {"s1": (4, 16, 3), "s1-64-sample": (3, 64, 2)}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def run_ref(levels, nc, reps, threads):
    def lim():
        resource.setrlimit(resource.RLIMIT_STACK, (resource.RLIM_INFINITY,) * 2)
    env = dict(os.environ, OMP_NUM_THREADS=str(threads), OMP_STACKSIZE="512M")
    out = subprocess.run([EXE, str(levels), str(reps), "test_3d.cfg", "-box_size=%d" % nc,
                          "-coarse_grid_size=%d %d %d" % (nc, nc, nc)],
                         cwd=TESTS, env=env, capture_output=True, text=True, check=True,
                         preexec_fn=lim)
    f = [l for l in out.stdout.splitlines() if l.startswith("TIMING")][0].split()
    return {"species_s": float(f[2]), "vcycle_s": float(f[4]), "cells": int(f[6])}


def run_port(config, threads):
    code = ("import sys, json; sys.path.insert(0, %r); import bench; "
            "print(json.dumps(bench.cpu_baseline(%r, 0)))" % (REPO, config))
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True,
                         text=True, check=True)
    return json.loads(out.stdout.strip().splitlines()[-1])


def main(tag):
    res = {"cpu": cpu_model(), "logical_cpus": os.cpu_count(), "cases": {}}
    for name, (lvls, nc, reps) in CASES.items():
        for th in (1, 8):
            r = run_ref(lvls, nc, reps, th)
            unit = r["species_s"] + r["vcycle_s"]
            r["ref_unit_step_s"] = unit
            r["ref_cell_updates_per_s"] = r["cells"] / unit
            res["cases"]["%s_omp%d" % (name, th)] = r
            print(name, th, r, flush=True)
    for config, name in (("s1", "s1"), ("s1-64", "s1-64-sample")):
        for th in (1, 8):
            p = run_port(config, th)
            res["cases"]["%s_omp%d" % (name, th)]["port_cell_updates_per_s"] = p["value"]
            print(name, th, "port", p["value"], flush=True)
    out = os.path.join(REPO, "profiles", "%s_ref_cpu_timing.json" % tag)
    json.dump(res, open(out, "w"), indent=1)
    print("wrote", out)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r02")
