"""Diagnostic: per-phase cycle counts inside the round kernels (KG_STAMPS build; never the product path).
usage: stamps.py [nodes] [pods] [depth] [batch]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["KOORDGPU_LIB"] = os.path.join(ROOT, "koordinator_amd", os.environ.get("STAMPS_LIB", "libkoordgpu_stamps.so"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from koordinator_amd import Engine, abi, framework, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
npods = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
depth = int(sys.argv[3]) if len(sys.argv) > 3 else 0
batch = int(sys.argv[4]) if len(sys.argv) > 4 else 32
cfg = framework.build_config(device_id=0, pipeline_depth=depth, batch_pods=batch)
cl = synth.make_cluster(n, seed=synth.BASE_SEED + 3)
pods = synth.make_pods(npods, seed=synth.BASE_SEED + 4)
with Engine(cfg, n) as e:
    synth.load_into(e, cl)
    e.stage(pods)
    e.profile(True)
    st = e.schedule_staged(0, npods)
    prof = e.profile_read()
    buf = np.zeros(4 * 32 * 2 + 64 * 6 + 2 + 64 * 8, dtype=np.uint64)
    abi.check(e.lib, e.lib.kg_debug_stamps(e.h, abi.ptr(buf)))
    stamps = buf[:256].reshape(4, 32, 2)
    diag = buf[256:256 + 384].reshape(64, 6)
    lane = buf[256 + 384 + 2:].reshape(64, 8)
print(f"nodes={n} pods={npods} depth={depth} batch={batch}: rounds={int(st['device_batches'])} "
      f"slow={st['reserved'][0]:.0f} steps={st['reserved'][1]:.0f} seconds={st['seconds']:.4f} "
      f"pods/s={npods / st['seconds']:.0f}")
print("live:", {k: (round(ms / c * 1e3, 2), c) for k, (ms, c) in prof.items()})
for k, name in enumerate(("eval", "merge", "resolve")):
    pts = [(i, int(stamps[k, i, 0]), int(stamps[k, i, 1])) for i in range(32) if stamps[k, i, 0]]
    if not pts:
        continue
    t0c, t0r = pts[0][1], pts[0][2]
    print(f"== {name}: clock ≈ {(pts[-1][1]-t0c)/max(1,(pts[-1][2]-t0r))*100:.0f} MHz")
    prev = pts[0]
    for i, c, r in pts:
        print(f"  pt{i:2d}: +{c - prev[1]:7d} cyc  (+{(r - prev[2]) * 10:6d} ns)   cum {(r - t0r) * 10:7d} ns")
        prev = (i, c, r)

print("== resolver per pod (last launch): cycles since previous pod, pos, slow, new slot")
prev = None
for j in range(64):
    c, b = int(diag[j, 0]), int(diag[j, 1])
    if not c:
        break
    if prev is not None:
        sub = " ".join(f"{int(diag[j - 1, 2 + k]) - prev if diag[j - 1, 2 + k] else -1:5d}" for k in range(4))
        ls = " ".join(f"{int(lane[j - 1, k]) - prev if lane[j - 1, k] > prev else -1:5d}" for k in range(4))
        print(f"  pod {j - 1:2d}: {c - prev:6d} cyc pos={b >> 8:2d} slow={b & 1} new={(b >> 1) & 1}  sub {sub}"
              f"  slow-path [settled, keyed, aux, max] {ls}")
    prev = c
