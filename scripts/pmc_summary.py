#!/usr/bin/env python3
"""Summarise scripts/pmc.sh: HBM bytes per launch of the dominant kernel.

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch. The byte counters are
calibrated with k_calib_copy8 (scripts/pmc_calib.hip), which moves a known
8N bytes each way with the same 8-B/lane access width: corrected bytes =
counter x (known / counter_calib). Only the largest dispatches of the hot
kernel (the leaf level of the workload) are averaged.

Usage: pmc_summary.py <pmc dir> <algorithmic bytes per launch> <out.json>
"""
import csv
import glob
import json
import os
import sys


def per_dispatch(d):
    rows = list(csv.DictReader(open(glob.glob(os.path.join(d, "**", "*counter_collection.csv"),
                                              recursive=True)[0])))
    acc = {}
    for r in rows:
        key = r["Dispatch_Id"]
        a = acc.setdefault(key, {"grid": int(r["Grid_Size"]), "name": r["Kernel_Name"],
                                 "kib": 0.0})
        a["kib"] += float(r["Counter_Value"])
    return list(acc.values())


def main(src, alg_bytes, dst):
    out = {"algorithmic_bytes_per_launch": alg_bytes}
    known = 8.0 * (1 << 28)
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        cal = per_dispatch(os.path.join(src, "calib_" + c))
        cal_b = sum(x["kib"] for x in cal) / len(cal) * 1024.0
        hot = per_dispatch(os.path.join(src, c))
        gmax = max(x["grid"] for x in hot)
        hot = [x for x in hot if x["grid"] == gmax]
        raw = sum(x["kib"] for x in hot) / len(hot) * 1024.0
        out[c.lower() + "_raw_bytes"] = raw
        out[c.lower() + "_calib_factor"] = known / cal_b
        out[c.lower() + "_bytes"] = raw * known / cal_b
        out["kernel"] = hot[0]["name"].split("(")[0]
        out["launches"] = len(hot)
    out["hbm_bytes_per_launch"] = out["fetch_size_bytes"] + out["write_size_bytes"]
    out["traffic_over_algorithmic"] = out["hbm_bytes_per_launch"] / alg_bytes
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]), sys.argv[3])
