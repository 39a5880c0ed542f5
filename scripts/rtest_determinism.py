#!/usr/bin/env python3
"""Debug aid: the device regression run test_3d twice per smoother setting
(AFH_GSRB_FUSED_MIN_BOXES unset / 1) in one process; prints whether the
two logs of a setting are identical and how far the settings are apart."""
import os
import sys
sys.path[:0] = ["afivo-streamer_amd", "tests"]
import numpy as np
import golden
from afh import capi
from afh.driver import Simulation

name = sys.argv[1] if len(sys.argv) > 1 else "test_3d"
logs = {}
for mode in ("default", "1"):
    if mode != "default":
        os.environ["AFH_GSRB_FUSED_MIN_BOXES"] = mode
    for rep in range(2):
        sim = Simulation(capi.hip_library(), golden.load("rtest_" + name), device=0)
        logs[(mode, rep)] = sim.run()
        print(mode, rep, "rows", len(logs[(mode, rep)]), flush=True)
    os.environ.pop("AFH_GSRB_FUSED_MIN_BOXES", None)
    a, b = logs[(mode, 0)], logs[(mode, 1)]
    print(mode, "repeat identical:", np.array_equal(a, b),
          "max rel", np.max(np.abs(a - b) / np.maximum(np.abs(a), 1e-300)), flush=True)
a, b = logs[("default", 0)], logs[("1", 0)]
rel = np.abs(a - b) / np.maximum(np.abs(a), 1e-300)
print("default vs fused: max rel per row", np.max(rel, axis=1), flush=True)
