#!/usr/bin/env python3
"""Steady-state per-step profile of a bench run from a rocprofv3 kernel
trace (--kernel-trace --output-format csv).

The timed region of `bench.py --steps K` is the last K unit steps; each step
ends with the species update (k_update / k_fe_lds, one launch per leaf
level), so the window starts right after the (K+1)-th last run of update
launches. Reports per step: kernel time by kernel, launch count, busy time,
the gaps between consecutive kernels (launch overhead and host
synchronisation) and the span; and for the largest launch of each kernel
its average duration, its algorithmic bytes and the fraction of the 8 TB/s
HBM peak.

Algorithmic bytes follow SURVEY.md 8(d): bytes per cell
of the pass x the cells of the launch. The cells come from the run's own
topology, which bench.py writes when AFH_BENCH_TOPO names a file: per level
the number of boxes, leaves and parents, the box size and the species
counts. The largest launch of a kernel is taken to cover the level with the
most boxes of the list the kernel runs over (all boxes, leaves or parents;
the k-split / tiled pair only runs on levels of 64..255 boxes); a kernel
whose grid is (box cells, boxes) -- the update, the small-box flux and the
residual, which may cover every leaf level in one launch -- takes its boxes
from the launch's grid.

Usage: prof_steady.py <run_kernel_trace.csv> <K> <out.json> <topo.json>
       prof_steady.py --rescore <summary.json> ...
"""
import collections
import csv
import json
import re
import sys

PEAK = 8e12


def rules(topo):
    """[(name regex, bytes per cell, list, level filter)]; first match wins."""
    nc = topo["nc"]
    nq = topo.get("n_charged", topo.get("n_species", 3))
    phi = topo.get("faces_from_phi", False)
    rhs = topo.get("fused_rhs", False)
    small = lambda n: 64 <= n < 256  # noqa: E731  k-split / tiled pair levels
    # the split half-sweep: levels below the fused pair's 64 boxes (nc >= 32),
    # or a stale top level (any)
    split = (lambda n: n < 64) if nc >= 32 else None

    def upd(m):
        # + the rhs of the new state when field_set_rhs is folded in
        ns, np_ = int(m.group(1)), int(m.group(2) or 2)
        return 8 * ns * ((np_ if np_ in (1, 2) else 2) + 1) + 32 + (8 if rhs else 0)

    return [
        (r"k_gsrb_pair2<64, 64, 1, 4>", 24, "ids", small),
        (r"k_gsrb_pair", 24, "ids", None),
        (r"k_gsrb_v", 16, "ids", None),
        (r"k_gsrb\(", 16, "ids", split),
        # with |E| folded in (afh_mg_set_gradient_output): + 8 B written
        (r"k_residual<true, \d, true", 32, "leaves", None),
        (r"k_residual<false, \d, true", 32, "parents", None),
        (r"k_residual<true", 24, "leaves", None),
        (r"k_residual<false", 24, "parents", None),
        (r"k_rstr_fas", 18, "ids", None),
        (r"k_prolong<", 20, "ids", None),
        (r"k_corr_tmp", 24, "parents", None),
        (r"k_parent_rhs", 24, "parents", None),
        # with the face field formed in the flux (faces_from_phi): the
        # gradient reads phi and writes |E|; the flux reads phi instead of
        # three face fields
        (r"k_gradient", 16 if phi else 40, "all", None),
        (r"k_flux_lds|k_flux_staged", (48 if phi else 64) + 192 / nc, "leaves", None),
        (r"k_update<(\d+), \w+(?:, (\d+))?", upd, "leaves", None),
        # the fused species step: the update's bytes less the 3 fluxes read,
        # plus the flux's face-field input (phi: 16 B fewer than upd's 32)
        (r"k_fe_lds<\d+, \d+, (\d+), (\d+)", lambda m: upd(m) - (16 if phi else 0),
         "leaves", None),
        (r"k_gc_faces", 96 / nc, "ids", None),
        (r"k_gc2", 192 / nc, "leaves", None),
        (r"k_set_rhs<", 8 * (nq + 1), "leaves", None),
    ]


def largest(topo, lst, filt):
    if lst == "all":
        return sum(topo["ids"])
    counts = [n for n, tot in zip(topo[lst], topo["ids"]) if filt is None or filt(tot)]
    return max(counts) if counts else 0


def key(name):
    """Kernel name without the argument list."""
    depth = 0
    for i, ch in enumerate(name):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            return name[:i]
    return name


# kernels whose grid is (cells of a box, boxes): one launch may cover every
# leaf level (AFH_ALL_LVL), so the boxes are read from the launch's grid
BOX_GRID = re.compile(r"k_update<|k_flux_staged|k_residual<")
# the fused pair's grid is (boxes x NC/TJ row tiles x KS k-splits) workgroups
# (afh_mg.hip launch_pair2): its boxes follow from the launch's workgroups
PAIR2 = re.compile(r"k_gsrb_pair2<(\d+), (\d+), \d+, (\d+)>")


def algorithmic(name, topo, grid_y=1, groups=0):
    """Algorithmic bytes of the launch: bytes per cell x cells. The boxes come
    from the launch's grid where its shape gives them (BOX_GRID, PAIR2), else
    from the level the kernel's list and filter select."""
    for pat, b, lst, filt in rules(topo):
        m = re.search(pat, name)
        if m:
            per_cell = b(m) if callable(b) else b
            p2 = PAIR2.search(name)
            if p2 and groups:
                nc, tj, ks = (int(x) for x in p2.groups())
                boxes = groups // ((nc // tj) * ks)
            elif BOX_GRID.search(name) and grid_y > 1:
                boxes = grid_y
            else:
                boxes = largest(topo, lst, filt)
            return per_cell * topo["nc"] ** 3 * boxes
    return None


def guard(ent):
    """A fraction of the HBM peak above 1 is a byte-model error, never a
    measurement: such an entry keeps its time and loses its fraction."""
    if ent.get("frac_of_8TBps", 0) > 1:
        for k in ("algorithmic_bytes", "achieved_TBps", "frac_of_8TBps"):
            ent.pop(k, None)
        ent["frac_note"] = "byte model does not fit this launch; no fraction reported"
    return ent


def main(path, k_steps, out, topo_path):
    topo = json.load(open(topo_path))
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    upd = [i for i, r in enumerate(rows)
           if re.search(r"k2?_update|k_fe_lds", r["Kernel_Name"])]
    # a step ends with the update of every leaf level (consecutive launches)
    ends = [i for n, i in enumerate(upd) if n + 1 == len(upd) or upd[n + 1] != i + 1]
    start = ends[-(k_steps + 1)] + 1
    win = rows[start:ends[-1] + 1]
    st = [int(r["Start_Timestamp"]) for r in win]
    en = [int(r["End_Timestamp"]) for r in win]
    busy = sum(e - s for s, e in zip(st, en))
    gaps = sum(max(0, st[i + 1] - en[i]) for i in range(len(win) - 1))
    span = en[-1] - st[0]
    per = collections.defaultdict(lambda: [0, 0.0, []])
    for r in win:
        k = key(r["Kernel_Name"])
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        wg = int(r.get("Workgroup_Size_X") or 1) * int(r.get("Workgroup_Size_Y") or 1) * \
            int(r.get("Workgroup_Size_Z") or 1)
        per[k][0] += 1
        per[k][1] += d
        per[k][2].append((g, d, int(r["Grid_Size_Y"]), g // max(wg, 1)))
    table = []
    for k, (n, tot, lst) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        gmax = max(g for g, _, _, _ in lst)
        big = [d for g, d, _, _ in lst if g == gmax]
        gy = max(y for g, _, y, _ in lst if g == gmax)
        groups = max(w for g, _, _, w in lst if g == gmax)
        avg = sum(big) / len(big)
        ent = {"kernel": k, "launches_per_step": n / k_steps,
               "us_per_step": tot / k_steps, "share": tot * 1e3 / busy,
               "largest_launch_avg_us": avg}
        b = algorithmic(k, topo, gy, groups)
        if b:
            ent.update({"algorithmic_bytes": b, "achieved_TBps": b / (avg * 1e-6) / 1e12,
                        "frac_of_8TBps": b / (avg * 1e-6) / PEAK})
        table.append(guard(ent))
    res = {"config": topo.get("config"), "nc": topo["nc"],
           "leaf_cells": topo["nc"] ** 3 * sum(topo["leaves"]),
           "boxes_per_level": topo["ids"], "leaves_per_level": topo["leaves"],
           "steps": k_steps, "launches_per_step": len(win) / k_steps,
           "span_ms_per_step": span / 1e6 / k_steps,
           "busy_ms_per_step": busy / 1e6 / k_steps,
           "gap_ms_per_step": gaps / 1e6 / k_steps,
           "gap_share": gaps / span if span else 0.0, "kernels": table}
    json.dump(res, open(out, "w"), indent=1)
    print("per step: %.3f ms span, %.3f ms busy, %.3f ms gaps (%.0f %%), %.0f launches" %
          (res["span_ms_per_step"], res["busy_ms_per_step"], res["gap_ms_per_step"],
           100 * res["gap_share"], res["launches_per_step"]))
    for e in table[:18]:
        print("%-40s %5.1f/step %8.1f us/step %5.1f%%  largest %8.1f us %s" % (
            e["kernel"][:40], e["launches_per_step"], e["us_per_step"], 100 * e["share"],
            e["largest_launch_avg_us"],
            ("%.2f TB/s frac %.3f" % (e["achieved_TBps"], e["frac_of_8TBps"]))
            if "achieved_TBps" in e else ""))
    bad = [e["kernel"] for e in table if "frac_note" in e]
    if bad:
        print("no fraction (the byte model does not fit the launch):", bad)


def rescore(path):
    """Apply the guard to a committed summary (JSON): an entry whose fraction
    exceeds 1 keeps its times and loses the fraction."""
    d = json.load(open(path))
    d["kernels"] = [guard(e) for e in d["kernels"]]
    json.dump(d, open(path, "w"), indent=1)


if __name__ == "__main__":
    if sys.argv[1] == "--rescore":
        for f in sys.argv[2:]:
            rescore(f)
    else:
        main(sys.argv[1], int(sys.argv[2]), sys.argv[3], sys.argv[4])
