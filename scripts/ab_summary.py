#!/usr/bin/env python3
"""Per-kernel mean durations (us) of scripts/ab.sh runs, one column per
variant (averaged over repetitions)."""
import collections
import glob
import os
import sqlite3
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab"
tab = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sorted(x for x in glob.glob(os.path.join(src, "v*_r*")) if os.path.isdir(x)):
    v = os.path.basename(d).split("_")[0]
    db = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)[0]
    con = sqlite3.connect(db)
    for name, calls, total in con.execute(
            "select name, total_calls, total_duration from top_kernels"):
        tab[name.split("(")[0]][v].append(total / 1e3)
vs = sorted({v for k in tab for v in tab[k]})
rows = sorted(tab.items(), key=lambda kv: -max(sum(x) / len(x) for x in kv[1].values()))
print("%-40s" % "kernel (total ms per run)" + "".join("%10s" % v for v in vs))
for k, d in rows[:25]:
    print("%-40s" % k[:40] + "".join("%10.3f" % (sum(d[v]) / len(d[v])) if v in d else "%10s" % "-"
                                      for v in vs))
