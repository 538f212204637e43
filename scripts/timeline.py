#!/usr/bin/env python3
"""Round timeline of a pipelined C3 run from a rocprofv3 --kernel-trace CSV (usage: timeline.py DIR DEPTH).
Per round r (kernels matched by dispatch order): eval / merge / resolve durations, the resolver's own work after
its predecessor ended, the round period, and the gaps on the two dependency chains."""
import csv
import glob
import sys
from collections import defaultdict

import numpy as np


def short(n):
    for k in ("eval_round", "merge_round", "resolve_round", "merge_wave"):
        if k in n:
            return "merge_round" if k == "merge_wave" else k
    return None


f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
D = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rows = list(csv.DictReader(open(f)))
by = defaultdict(list)
for r in rows:
    k = short(r["Kernel_Name"])
    if k:
        by[k].append((int(r.get("Dispatch_Id", 0)), int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
for k in by:
    by[k].sort()
if len(by.get("merge_round", [])) < len(by["eval_round"]) // 2:  # (r5) merge fused into eval_round's tail: a zero-length merge at the eval's end
    by["merge_round"] = [(d, e, e) for d, _, e in by["eval_round"]]
E, M, R = (np.array([(s, e) for _, s, e in by[k]], dtype=np.float64) / 1e3 for k in ("eval_round", "merge_round",
                                                                                      "resolve_round"))
n = min(len(E), len(M), len(R))
E, M, R = E[:n], M[:n], R[:n]
q = lambda x: f"p50 {np.median(x):7.2f}  mean {x.mean():7.2f}  p90 {np.percentile(x, 90):7.2f} us"
print(f"rounds {n}, depth {D}")
print("eval     ", q(E[:, 1] - E[:, 0]))
print("merge    ", q(M[:, 1] - M[:, 0]))
print("resolve  ", q(R[:, 1] - R[:, 0]))
own = R[1:, 1] - np.maximum(R[1:, 0], R[:-1, 1])
print("resolve after predecessor end", q(own))
per = np.diff(R[:, 1])
per = per[per < 2000]
print("period (resolve end → end)", q(per))
print("merge end → resolve start ", q(R[:, 0] - M[:, 1]))
print("eval end → merge start    ", q(M[:, 0] - E[:, 1]))
print("resolve(r-1) end → resolve(r) end", q(R[1:, 1] - R[:-1, 1]))
print("merge(r) end − resolve(r-1) end (>0: the eval chain is late)", q(M[1:, 1] - R[:-1, 1]))
if n > D:
    print(f"resolve(r-{D}) end → eval(r) start", q(E[D:, 0] - R[:-D, 1]))
