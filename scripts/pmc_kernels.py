#!/usr/bin/env python3
"""Per-kernel totals and per-launch averages of every counter in the rocprofv3 --pmc passes under DIR
(usage: pmc_kernels.py DIR).  FETCH_SIZE is doubled (gfx950: 128-B reads counted at 64 B, MI355X_MICROARCH.md);
sizes in KiB as rocprofv3 emits them.  Writes DIR/pmc_kernels.json."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(?:kg::|namespace\)::)([A-Za-z_0-9]+)", name)
    return m.group(1) if m else name[:40]


d = sys.argv[1]
tot = defaultdict(lambda: defaultdict(float))
disp = defaultdict(lambda: defaultdict(set))
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k, c = short(r.get("Kernel_Name", "")), r.get("Counter_Name")
        tot[k][c] += float(r["Counter_Value"])
        disp[k][c].add((f, r.get("Dispatch_Id")))
out = {}
for k in sorted(tot):
    row = {}
    for c, v in tot[k].items():
        n = max(1, len(disp[k][c]))
        if c == "FETCH_SIZE":
            v *= 2
        row[c] = {"total": v, "launches": n, "per_launch": v / n}
    out[k] = row
json.dump(out, open(os.path.join(d, "pmc_kernels.json"), "w"), indent=1)
for k, row in out.items():
    n = max(x["launches"] for x in row.values())
    print(f"{k} ({n} launches):", ", ".join(f"{c}={x['per_launch']:.4g}" for c, x in sorted(row.items())))
