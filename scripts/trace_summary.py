#!/usr/bin/env python3
"""Round timeline from a rocprofv3 --kernel-trace CSV: per-kernel durations, the round period (resolve start
to resolve start) and the critical-path gaps (eval end → merge start, merge end → resolve start)."""
import csv
import glob
import sys
from collections import defaultdict

import numpy as np


def short(n):
    for k in ("eval_round", "merge_round", "resolve_round", "ncclDevKernel", "apply_deltas"):
        if k in n:
            return k
    return n[:40]


f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows))
by = defaultdict(list)
for s, e, k in ev:
    by[k].append((s, e))
for k, v in by.items():
    d = np.array([e - s for s, e in v]) / 1e3
    print(f"{k:16s} n={len(v):7d} avg={d.mean():8.2f} us  p50={np.median(d):8.2f}  p90={np.percentile(d, 90):8.2f}")
res = np.array(by.get("resolve_round", []))
mer = np.array(by.get("merge_round", []))
evl = np.array(by.get("eval_round", []))
if len(res) > 10 and len(res) == len(mer):
    per = np.diff(res[:, 0]) / 1e3
    per = per[per < 1000]
    print(f"round period (resolve→resolve start): median {np.median(per):.2f} us  mean {per.mean():.2f}")
    g1 = (res[:, 0] - mer[:, 1]) / 1e3
    print(f"merge end → resolve start: median {np.median(g1):.2f} us")
    if len(evl) == len(mer):
        g2 = (mer[:, 0] - evl[:, 1]) / 1e3
        print(f"eval end → merge start: median {np.median(g2):.2f} us")
        g3 = (evl[1:, 0] - res[:-1, 1]) / 1e3
        print(f"resolve(r) end → eval(r+1) start: median {np.median(g3):.2f} us (negative = overlapped)")
        g4 = (evl[2:, 0] - res[:-2, 1]) / 1e3
        print(f"resolve(r) end → eval(r+2) start: median {np.median(g4):.2f} us")
