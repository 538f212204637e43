#!/usr/bin/env python3
"""Kernel gaps of a rocprofv3 --kernel-trace run (usage: gaps.py DIR [first-kernel-substring]): the kernels in start
order, per kernel name the mean duration, and the idle time between one kernel's end and the next one's start."""
import csv
import glob
import re
import sys
from collections import defaultdict

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))


def short(n):
    m = re.search(r"(?:kg::|namespace\)::)([A-Za-z_0-9]+)", n)
    return m.group(1) if m else n[:30]


key = sys.argv[2] if len(sys.argv) > 2 else None
if key:  # the steady-state window: from the first kernel matching key
    i0 = next(i for i, r in enumerate(rows) if key in r["Kernel_Name"])
    rows = rows[i0:]
dur, gap_before = defaultdict(list), defaultdict(list)
prev_end = None
for r in rows:
    s, e, k = int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])
    dur[k].append((e - s) / 1e3)
    if prev_end is not None:
        gap_before[k].append(max(0, s - prev_end) / 1e3)
    prev_end = max(prev_end or 0, e)
span = (max(int(r["End_Timestamp"]) for r in rows) - int(rows[0]["Start_Timestamp"])) / 1e3
busy = sum(sum(v) for v in dur.values())
print(f"{len(rows)} kernels over {span:.0f} us, kernel time {busy:.0f} us ({100 * busy / span:.0f} %)")
for k in sorted(dur, key=lambda k: -sum(dur[k])):
    g = gap_before[k]
    print(f"  {k:22s} n={len(dur[k]):5d} mean {sum(dur[k]) / len(dur[k]):8.2f} us   idle before: mean "
          f"{(sum(g) / len(g)) if g else 0:7.2f} us, total {sum(g):9.0f} us")
