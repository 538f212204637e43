"""Diagnostic: per-pod cycle stamps of the batched exact resolver (xr_resolve) on a bench workload (KG_STAMPS build;
never the product path).  usage: stamps_xr.py [workload c5|shipped|c5r] [nodes] [pods]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["KOORDGPU_LIB"] = os.path.join(ROOT, "koordinator_amd", os.environ.get("STAMPS_LIB", "libkoordgpu_stamps.so"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import bench  # noqa: E402
from koordinator_amd import Engine, abi, framework  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "c5"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 50000
npods = int(sys.argv[3]) if len(sys.argv) > 3 else 5000
F = framework
if wl == "shipped":
    profile = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.NODE_NUMA_RESOURCE, F.DEVICE_SHARE, F.RESERVATION),
                        score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.NODE_NUMA_RESOURCE: 1, F.DEVICE_SHARE: 1,
                               F.RESERVATION: 5000})
elif wl == "c5":
    profile = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.RESERVATION, F.DEVICE_SHARE),
                        score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.RESERVATION: 5000, F.DEVICE_SHARE: 1})
else:
    profile = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.RESERVATION),
                        score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.RESERVATION: 5000})
cfg = framework.build_config(device_id=0, profile=profile)
work = bench.Work(wl, n, cfg)
pods = work.make_pods(npods, seed=work.seed + 1)
work.set_queue(pods)
with Engine(cfg, work.cluster.n) as e:
    work.load(e)
    e.stage(pods)
    e.profile(True)
    st = e.schedule_staged(0, npods)
    prof = e.profile_read()
    buf = np.zeros(4 * 32 * 2 + 64 * 6 + 2 + 64 * 8, dtype=np.uint64)
    abi.check(e.lib, e.lib.kg_debug_stamps(e.h, abi.ptr(buf)))
    diag = buf[256:256 + 384].reshape(64, 6)
    lane = buf[256 + 384 + 2:].reshape(64, 8)
print(f"{wl} nodes={n} pods={npods}: rounds={int(st['device_batches'])} seconds={st['seconds']:.4f} "
      f"pods/s={npods / st['seconds']:.0f}")
print("live:", {k: (round(ms / c * 1e3, 2), c) for k, (ms, c) in prof.items()})
print("== xr_resolve per pod (last launch): cycles since previous pod start; nM; sub-stamps after "
      "[modified-row eval, stop rule, candidate pick, Reserve]")
prev = None
for j in range(64):
    c, b = int(diag[j, 0]), int(diag[j, 1])
    if not c:
        break
    if prev is not None:
        pc = int(diag[j - 1, 0])
        sub = " ".join(f"{int(diag[j - 1, 2 + k]) - pc if diag[j - 1, 2 + k] else -1:6d}" for k in range(4))
        rs = " ".join(f"{int(lane[j - 1, k]) - pc if lane[j - 1, k] else -1:6d}" for k in range(6))
        print(f"  pod {j - 1:2d}: {c - prev:7d} cyc nM={int(diag[j - 1, 1]):2d}  sub {sub}  reserve {rs}")
    prev = c
