#!/usr/bin/env python3
"""Config 4's time loop to its end: the device driver's regression rows
(scripts/s4_timeloop_rows.py on the GPU box) against the reference's own
streamer.f90 run through the shim on the C oracle (oracle/_ref/dropin_streamer,
build container; tests/test_dropin_streamer.py's S4 arguments with
end_time = 2.5 ns, output%dt = 0.05 ns). VERDICT r5 item 3.

usage: s4_collapse_compare.py <device rows .json> <drop-in rtest log>
       <drop-in stdout> <out .json>
Prints per row the largest relative difference and writes the summary.
"""
import json
import sys

import numpy as np


def main(dev_json, ref_log, ref_stdout, out):
    dev = json.load(open(dev_json))
    H = np.array(dev["rows"])
    R = np.loadtxt(ref_log, skiprows=1, ndmin=2)
    n = min(len(H), len(R))
    rel = [float((np.abs(H[k] - R[k]) / np.maximum(np.abs(R[k]), 1e-300)).max())
           for k in range(n)]
    for k in range(n):
        print("row %2d t = %.3e s: max rel %.2e" % (k, R[k][1], rel[k]))
    text = open(ref_stdout, errors="replace").read() if ref_stdout != "-" else ""
    stop = "dt too small" if "dt too small" in text else None
    res = {"what": "config 4 (streamer_3d.cfg + grounded rod electrode, air_chemistry_v2, "
                   "PFMG level-1 solve) from the reference's set-up to the end of its time "
                   "loop: the device driver (afh.driver on libafivo_hip, MI355X) against the "
                   "reference's own src/streamer.f90 through the shim on the C oracle "
                   "(oracle/_ref/dropin_streamer, CPU)",
           "rows_compared": n, "rows_device": len(H), "rows_reference": len(R),
           "max_rel_diff": max(rel) if rel else None, "max_rel_diff_per_row": rel,
           "device_stop": {"it": dev["it"], "time": dev["time"], "dt": dev["dt"],
                           "error": dev["error"]},
           "reference_stop": stop, "reference_last_row_time": float(R[-1][1]),
           "reference_stdout_tail": text[-600:]}
    json.dump(res, open(out, "w"), indent=1)
    print({k: v for k, v in res.items() if k not in ("max_rel_diff_per_row",
                                                       "reference_stdout_tail")})


if __name__ == "__main__":
    main(*sys.argv[1:])
