"""Diagnostic: per-phase cycle counts inside the round kernels (KG_STAMPS build; never the product path)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["KOORDGPU_LIB"] = os.path.join(ROOT, "koordinator_amd", "libkoordgpu_stamps.so")
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from koordinator_amd import Engine, abi, framework, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
cfg = framework.build_config(device_id=0)
cl = synth.make_cluster(n, seed=5)
pods = synth.make_pods(3200, seed=6)
with Engine(cfg, n) as e:
    synth.load_into(e, cl)
    e.schedule(pods)
    st = np.zeros((4, 32, 2), dtype=np.uint64)
    abi.check(e.lib, e.lib.kg_debug_stamps(e.h, abi.ptr(st)))
pass
pass
for k, name in enumerate(("eval", "merge", "resolve")):
    pts = [(i, int(st[k, i, 0]), int(st[k, i, 1])) for i in range(32) if st[k, i, 0]]
    if not pts:
        continue
    t0c, t0r = pts[0][1], pts[0][2]
    print(f"== {name}: clock ≈ {(pts[-1][1]-t0c)/max(1,(pts[-1][2]-t0r))*100:.0f} MHz")
    prev = pts[0]
    for i, c, r in pts:
        print(f"  pt{i:2d}: +{c - prev[1]:7d} cyc  (+{(r - prev[2]) * 10:6d} ns)   cum {(r - t0r) * 10:7d} ns")
        prev = (i, c, r)
