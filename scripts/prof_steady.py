#!/usr/bin/env python3
"""Steady-state per-step profile of a bench run from a rocprofv3 kernel
trace (--kernel-trace --output-format csv).

The timed region of `bench.py --steps K` is the last K unit steps; each step
ends with the species update (k_update, one launch per leaf level), so the
window starts right after the (K+1)-th last run of k_update launches. Reports per step: kernel time by kernel, launch
count, busy time, the gaps between consecutive kernels (launch overhead and
host synchronisation) and the span; and, for the S1-64 leaf level (largest
launch of each kernel), average duration, algorithmic bytes (DESIGN.md
table) and the fraction of the 8 TB/s HBM peak.

Usage: prof_steady.py <run_kernel_trace.csv> <K> <out.json> [config]
"""
import collections
import csv
import json
import sys

PEAK = 8e12
LEAF = 512 * 64 ** 3          # S1-64 leaf cells
PARENT = 64 * 64 ** 3         # S1-64 level-3 boxes (parents of the leaves)
# kernel (name prefix up to '(') -> (algorithmic bytes per cell, cells)
ALG = {
    "void afh::k_gsrb_pair2<64, 64, 1, 0, true, true, true, 1>": (24, LEAF),
    "void afh::k_gsrb_pair2<64, 64, 1, 0, true, true, true, 4>": (24, PARENT),
    "void afh::k_gsrb_pair2<64, 64": (24, LEAF),
    "void afh::k_gsrb_pair2<64, 16": (24, PARENT),
    "void afh::k_residual<true, 4>": (24, LEAF),
    "void afh::k_residual<false, 4>": (24, PARENT),
    "afh::k_rstr_fas": (18, LEAF),
    "void afh::k_rstr_fas_col<2>": (18, LEAF),
    "void afh::k_prolong<4>": (20, LEAF),
    "afh::k_corr_tmp": (24, PARENT),
    "afh::k_parent_rhs": (24, PARENT),
    "void afh::k_gradient_t<64, 4>": (40, LEAF),
    "void afh::k_gradient_t<64, 4, true>": (40, LEAF),
    "void afh::k_flux_lds<64, 3>": (64 + 192 / 64, LEAF),
    "void afh::k_update<3, false, 1": (8 * 3 * 2 + 32, LEAF),
    "void afh::k_update<3, false, 2": (8 * 3 * 3 + 32, LEAF),
    "afh::k_gc_faces": (96 / 64, LEAF),
    "afh::k_gc2": (2 * 96 / 64, LEAF),
    "void afh::k_set_rhs<true>": (32, LEAF),
}


def key(name):
    for k in ALG:
        if name.startswith(k):
            return k
    return name.split("(")[0]


def main(path, k_steps, out):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    upd = [i for i, r in enumerate(rows) if "k_update" in r["Kernel_Name"]]
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
        per[k][0] += 1
        per[k][1] += d
        per[k][2].append((g, d))
    table = []
    for k, (n, tot, lst) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        gmax = max(g for g, _ in lst)
        big = [d for g, d in lst if g == gmax]
        avg = sum(big) / len(big)
        ent = {"kernel": k, "launches_per_step": n / k_steps,
               "us_per_step": tot / k_steps, "share": tot * 1e3 / busy,
               "largest_launch_avg_us": avg}
        if k in ALG:
            b = ALG[k][0] * ALG[k][1]
            ent.update({"algorithmic_bytes": b, "achieved_TBps": b / (avg * 1e-6) / 1e12,
                        "frac_of_8TBps": b / (avg * 1e-6) / PEAK})
        table.append(ent)
    res = {"steps": k_steps, "launches_per_step": len(win) / k_steps,
           "span_ms_per_step": span / 1e6 / k_steps,
           "busy_ms_per_step": busy / 1e6 / k_steps,
           "gap_ms_per_step": gaps / 1e6 / k_steps, "kernels": table}
    json.dump(res, open(out, "w"), indent=1)
    print("per step: %.3f ms span, %.3f ms busy, %.3f ms gaps, %.0f launches" %
          (res["span_ms_per_step"], res["busy_ms_per_step"], res["gap_ms_per_step"],
           res["launches_per_step"]))
    for e in table[:16]:
        print("%-34s %5.1f/step %8.1f us/step %5.1f%%  leaf %8.1f us %s" % (
            e["kernel"][:34], e["launches_per_step"], e["us_per_step"], 100 * e["share"],
            e["largest_launch_avg_us"],
            ("%.2f TB/s frac %.3f" % (e["achieved_TBps"], e["frac_of_8TBps"]))
            if "achieved_TBps" in e else ""))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), sys.argv[3])
