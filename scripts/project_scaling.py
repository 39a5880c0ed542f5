#!/usr/bin/env python3
"""Strong-scaling projection from thread-rank runs on one GPU (VERDICT r4,
next-round item 2). PROJECTION, NOT A MEASUREMENT: no multi-GPU node has run
this code.

Inputs, per configuration (scripts/scaling_runs.sh makes them on the GPU box):
  N = 1: bench.py's normal line (wall ms per step, window_ns) and the
         rocprofv3 kernel trace of the same run;
  N > 1: bench.py --transport local --gpus N --shared-stream (every rank a
         thread of one process; all ranks on ONE HIP stream, so their kernels
         run one at a time and each kernel's duration is its own) and its
         kernel trace.
Per rank (host thread that launched the kernels) the kernel busy time inside
the timed window, per step: b_r (the peer-copy blits of the thread ranks
excluded: they stand in for the RCCL transfer, priced by alpha and beta). With the N = 1 run's busy time b_1 and wall
time T_1, the launch / host overhead ratio rho = T_1 / b_1. The projected
step time of N GPUs, one rank each:

    T_N = rho * max_r b_r + E_N * alpha + max_r B_r / beta

E_N: exchanges per step (each a grouped RCCL send/recv or an all-reduce, and
a graph-segment boundary), B_r: bytes rank r sends and receives per step (all
peers, summed: as if every byte crossed one link, one direction at a time),
alpha: 15 us per exchange (RCCL point-to-point latency over xGMI plus the
segment launch; an assumption), beta: 64 GB/s (a conservative half of one
xGMI link). Speed-up T_1 / T_N.

Beside it (round 6), the per-link variant: an MI355X node joins every pair of
its 8 GPUs by an xGMI link of its own, and a link moves both directions at
once, so the bytes term is max over ranks r and peers q of
max(sent_rq, received_rq) / beta (bench.py's peer_bytes_per_step; the same
alpha and beta). Still a projection: the link's real bandwidth and the
overlap of several links are unmeasured here.

Usage: project_scaling.py <config> <dir> <out.json>
  <dir>/n1.json, <dir>/n1_trace.csv, <dir>/nN.json, <dir>/nN_trace.csv
"""
import csv
import glob
import json
import os
import sys

ALPHA_S = 15e-6
BETA_BS = 64e9


def busy_by_thread(trace, window, kernels=None):
    """Kernel time per launching host thread inside [t0, t1] (ns); with
    kernels (a dict), also per thread the time and launches per kernel name
    (template arguments cut)."""
    t0, t1 = window
    out = {}
    with open(trace) as f:
        for row in csv.DictReader(f):
            s, e = int(row["Start_Timestamp"]), int(row["End_Timestamp"])
            if s < t0 or e > t1:
                continue
            # the thread ranks' peer copies stand in for the RCCL transfer,
            # which the model prices separately (alpha, beta)
            if row["Kernel_Name"].startswith("__amd_rocclr_copyBuffer"):
                continue
            tid = row.get("Thread_Id", "0")
            out[tid] = out.get(tid, 0) + (e - s)
            if kernels is not None:
                name = row["Kernel_Name"].split("(")[0]
                k = kernels.setdefault(tid, {}).setdefault(name, [0, 0])
                k[0] += e - s
                k[1] += 1
    return out


def top_kernels(per_kernel, steps, n=12):
    """The n kernels of most time: (name, ms per step, launches per step)."""
    items = sorted(per_kernel.items(), key=lambda kv: -kv[1][0])[:n]
    return [(k, round(v[0] / steps * 1e-6, 4), round(v[1] / steps, 1)) for k, v in items]


def main(config, d, out_path):
    n1 = json.load(open(os.path.join(d, "n1.json")))
    steps1 = n1["steps"]
    k1 = {}
    b1 = busy_by_thread(os.path.join(d, "n1_trace.csv"), n1["window_ns"], k1)
    busy1 = sum(b1.values()) / steps1 * 1e-9
    T1 = n1["ms_per_step"] * 1e-3
    rho = T1 / busy1 if busy1 > 0 else 1.0
    res = {"config": config, "label": "projection, not measured",
           "model": "T_N = rho * max_r busy_r + E_N * alpha + max_r bytes_r / beta",
           "alpha_s": ALPHA_S, "beta_Bps": BETA_BS,
           "n1": {"ms_per_step": T1 * 1e3, "kernel_busy_ms": busy1 * 1e3, "rho": rho,
                  "top_kernels": top_kernels(max(k1.values(), key=lambda v: sum(x[0] for x in
                                                                                 v.values())),
                                             steps1)},
           "ranks": {}}
    for path in sorted(glob.glob(os.path.join(d, "n*.json"))):
        name = os.path.basename(path)[:-5]
        if name == "n1":
            continue
        j = json.load(open(path))
        n = j["n_ranks"]
        kk = {}
        b = busy_by_thread(os.path.join(d, name + "_trace.csv"), j["window_ns"], kk)
        busiest = max(b, key=b.get)
        per = sorted((v / j["steps"] * 1e-9 for v in b.values()), reverse=True)[:n]
        E = max(j["exchanges_per_step"])
        B = max(j["exchange_bytes_per_step"])
        TN = rho * per[0] + E * ALPHA_S + B / BETA_BS
        link = None
        if "peer_bytes_per_step" in j:
            link = max(max(max(s, r) for s, r in zip(p["sent"], p["received"]))
                       for p in j["peer_bytes_per_step"])
        res["ranks"][str(n)] = {
            "busy_ms_per_rank": [x * 1e3 for x in per],
            "busy_sum_ms": sum(per) * 1e3,
            "exchanges_per_step": E, "bytes_per_step_max": B,
            "owned_leaf_cells": j["owned_leaf_cells"],
            "projected_ms_per_step": TN * 1e3,
            "compute_ms": rho * per[0] * 1e3,
            "exchange_latency_ms": E * ALPHA_S * 1e3,
            "exchange_bw_ms": B / BETA_BS * 1e3,
            "projected_speedup": T1 / TN,
            "link_bytes_per_step_max": link,
            "projected_ms_per_step_per_link": None if link is None else
            (rho * per[0] + E * ALPHA_S + link / BETA_BS) * 1e3,
            "projected_speedup_per_link": None if link is None else
            T1 / (rho * per[0] + E * ALPHA_S + link / BETA_BS),
            "partition_level": j["config"].get("partition_level"),
            "min_level_cells": j["config"].get("min_level_cells"),
            "busiest_rank_top_kernels": top_kernels(kk[busiest], j["steps"]),
        }
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
