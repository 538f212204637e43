#!/usr/bin/env python3
"""Diagnostic (r6): where a batched exact round's wall time goes, from a rocprofv3 --kernel-trace CSV of a shipped /
C5 bench run (usage: trace_xr.py DIR).  Sorts every kernel by start time and reports, per kernel name, the count and
mean duration, and the idle gaps between consecutive kernels (the device doing nothing) split by what follows."""
import csv
import glob
import sys
from collections import defaultdict

import numpy as np

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))


def short(n):
    return n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:40]


dur = defaultdict(list)
gap_before = defaultdict(list)
prev_end = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    k = short(r["Kernel_Name"])
    dur[k].append(e - s)
    if prev_end is not None:
        gap_before[k].append(max(0, s - prev_end))
    prev_end = max(prev_end or 0, e)
span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
busy = sum(sum(v) for v in dur.values()) / 1e3
print(f"{len(rows)} kernels over {span:.0f} us, kernel time {busy:.0f} us")
for k in sorted(dur, key=lambda k: -sum(dur[k])):
    g = np.array(gap_before.get(k, [0]))
    print(f"  {k:40s} n={len(dur[k]):6d} mean {np.mean(dur[k]) / 1e3:8.2f} us  total {sum(dur[k]) / 1e3:9.0f} us | "
          f"gap before: mean {g.mean() / 1e3:7.2f} us p90 {np.percentile(g, 90) / 1e3:7.2f} total {g.sum() / 1e3:8.0f} us")
