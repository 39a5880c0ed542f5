#!/usr/bin/env python3
"""Inputs of scripts/project_scaling.py for a grown driver tree (grown S3 /
S5), in ONE process: the tree is grown once
(bench.py --grow-cells; growing it again per rank count would cost the
call's time), then timed at N = 1 (bench.py's unit step, V-cycle graphs as
bench runs them) and sharded over N thread ranks on one stream
(bench.bench_local --shared-stream) for every size floor given. Run it under
rocprofv3 --kernel-trace; every bench line carries its window on the
trace's clock, so the one trace serves every projection.

Writes <out>/n1.json and <out>/f<floor>/n<N>.json (plus n1.json there).
PROJECTION INPUTS, NOT A MULTI-GPU MEASUREMENT.

Usage: scaling_grown.py <config> <grow_cells> <out> [--ns 2 4 8]
       [--floors 0 1048576] [--steps 5] [--warmup 2] [--grow-seconds 240]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config")
    ap.add_argument("grow_cells", type=float)
    ap.add_argument("out")
    ap.add_argument("--ns", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--floors", type=int, nargs="+", default=[0, 1 << 20])
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--grow-seconds", type=float, default=240.0)
    a = ap.parse_args()
    from afh import capi
    lib = capi.hip_library()
    coarse = bench.coarse_choice("auto", a.config)
    base = bench.build_driver_case(lib, 0, a.config, coarse, int(a.grow_cells), a.grow_seconds)
    os.makedirs(a.out, exist_ok=True)
    # N = 1: bench.py's timed region on the grown tree
    case = bench.DriverCase(base)
    case.fuse_rhs(True, ghosts=False)
    dt = 1e-13
    for k in range(a.warmup):
        bench.unit_step(case, dt, k)
    case.tree.sync()
    t0, ns0 = time.perf_counter(), time.clock_gettime_ns(time.CLOCK_MONOTONIC)
    for k in range(a.steps):
        bench.unit_step(case, dt, a.warmup + k)
    case.tree.sync()
    el, ns1 = time.perf_counter() - t0, time.clock_gettime_ns(time.CLOCK_MONOTONIC)
    cells = base.af.n_leaf_cells()
    n1 = {"config": {"workload": a.config, "leaf_cells": cells, "grown": base.grown},
          "steps": a.steps, "ms_per_step": 1e3 * el / a.steps, "window_ns": [ns0, ns1],
          "value": cells * a.steps / el}
    json.dump(n1, open(os.path.join(a.out, "n1.json"), "w"))
    print("n1", json.dumps({k: n1[k] for k in ("ms_per_step", "value")}), flush=True)
    for floor in a.floors:
        d = os.path.join(a.out, "f%d" % floor)
        os.makedirs(d, exist_ok=True)
        json.dump(n1, open(os.path.join(d, "n1.json"), "w"))
        for n in a.ns:
            args = argparse.Namespace(gpus=n, config=a.config, steps=a.steps, warmup=a.warmup,
                                      oracle=False, shared_stream=True, no_fused_rhs=False,
                                      stored_face_field=False, grow_cells=0,
                                      min_level_cells=floor)
            out = bench.bench_local(args, coarse, base=base)
            json.dump(out, open(os.path.join(d, "n%d.json" % n), "w"))
            print("f%d n%d" % (floor, n), json.dumps(
                {"ms_per_step": out["ms_per_step"], "lp": out["config"]["partition_level"],
                 "exchanges": max(out["exchanges_per_step"]),
                 "MB": max(out["exchange_bytes_per_step"]) / 1e6}), flush=True)


if __name__ == "__main__":
    main()
