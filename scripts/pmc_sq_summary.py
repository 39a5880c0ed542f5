#!/usr/bin/env python3
"""Sum SQ counters per dispatch of the largest launches of one kernel from
scripts/pmc_sq.sh passes. Usage: pmc_sq_summary.py <dir> <kernel substring>"""
import collections
import csv
import glob
import os
import sys


def main(d, sub):
    tot = collections.defaultdict(float)
    for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        acc = collections.defaultdict(lambda: collections.defaultdict(float))
        grid = {}
        for r in csv.DictReader(open(f)):
            if sub not in r["Kernel_Name"]:
                continue
            acc[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
            grid[r["Dispatch_Id"]] = int(r["Grid_Size"])
        if not grid:
            continue
        g = max(grid.values())
        big = [k for k in acc if grid[k] == g]
        for k in big:
            for c, v in acc[k].items():
                tot[c] += v / len(big)
    for c, v in sorted(tot.items()):
        print("%-28s %.4g" % (c, v))
    if "SQ_WAVES" in tot:
        w = tot["SQ_WAVES"]
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD",
                  "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH"):
            if c in tot:
                print("%-28s %.1f per wave" % (c, tot[c] / w))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
