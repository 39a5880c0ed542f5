#!/usr/bin/env python3
"""Summarise scripts/pmc_kernel.sh (gpurun_out/pmck/p*): per kernel and grid
size, the mean per dispatch of every collected counter (FETCH_SIZE /
WRITE_SIZE raw, in KiB; see pmc_summary.py for their calibration).

Usage: pmc_kernels_summary.py <pmck dir> <out.json>"""
import csv
import glob
import json
import os
import sys


def main(src, dst):
    acc = {}
    for path in glob.glob(os.path.join(src, "p*", "**", "*counter_collection.csv"),
                          recursive=True):
        per = {}
        for r in csv.DictReader(open(path)):
            key = (r["Kernel_Name"].split("(")[0], int(r["Grid_Size"]))
            d = per.setdefault((key, r["Dispatch_Id"]), {})
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        for (key, _), counters in per.items():
            for c, v in counters.items():
                s = acc.setdefault("%s grid=%d" % key, {}).setdefault(c, [0.0, 0])
                s[0] += v
                s[1] += 1
    out = {k: {c: s[0] / s[1] for c, s in sorted(v.items())} for k, v in sorted(acc.items())}
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
