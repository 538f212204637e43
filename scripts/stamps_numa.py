"""Diagnostic: per-pod cycle stamps inside resolve_round_numa at C4 size (KG_STAMPS dev build; never the product).
usage: stamps_numa.py [nodes] [pods] [batch]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["KOORDGPU_LIB"] = os.path.join(ROOT, "koordinator_amd", os.environ.get("STAMPS_LIB", "libkoordgpu_dev.so"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from koordinator_amd import Engine, abi, framework, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
npods = int(sys.argv[2]) if len(sys.argv) > 2 else 4000
batch = int(sys.argv[3]) if len(sys.argv) > 3 else 16
F = framework
profile = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.NODE_NUMA_RESOURCE),
                    score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.NODE_NUMA_RESOURCE: 1})
cfg = framework.build_config(device_id=0, batch_pods=batch, pods_per_wave=1, profile=profile)
cl, numa = synth.make_numa_cluster(n, seed=synth.BASE_SEED + 4)
pods = synth.make_numa_pods(npods, seed=synth.BASE_SEED + 5)
with Engine(cfg, n) as e:
    synth.load_numa_into(e, cl, numa)
    e.stage(pods)
    e.profile(True)
    st = e.schedule_staged(0, npods)
    prof = e.profile_read()
    buf = np.zeros(4 * 32 * 2 + 64 * 6 + 2 + 64 * 8, dtype=np.uint64)  # + the lane stamps kg_debug_stamps also copies
    abi.check(e.lib, e.lib.kg_debug_stamps(e.h, abi.ptr(buf)))
    diag = buf[256:256 + 384].reshape(64, 6)
    lane = buf[256 + 384 + 2:].reshape(64, 8)
print(f"nodes={n} pods={npods} batch={batch}: rounds={int(st['device_batches'])} seconds={st['seconds']:.4f} "
      f"pods/s={npods / st['seconds']:.0f}")
print("live:", {k: (round(ms / c * 1e3, 2), c) for k, (ms, c) in prof.items()})
merges, fallbacks = int(buf[256 + 384]), int(buf[256 + 384 + 1])
print(f"NUMA hint merges: {merges}, all-permutation fallback passes: {fallbacks} "
      f"({100.0 * fallbacks / max(merges, 1):.2f} %)")
print("== resolver per pod (last launch): cycles; nM; sub: rescored / winner row ready / reserved")
prev = None
for j in range(64):
    c = int(diag[j, 0])
    if not c:
        break
    if prev is not None:
        sub = " ".join(f"{int(diag[j - 1, 2 + k]) - prev if diag[j - 1, 2 + k] else -1:7d}" for k in range(3))  # rescored / winner ready / reserved
        ls = " ".join(f"{int(lane[j - 1, k]) - prev if lane[j - 1, k] else -1:7d}" for k in range(5))
        print(f"  pod {j - 1:2d}: {c - prev:7d} cyc nM={int(diag[j - 1, 1]):2d}  sub {sub}  filt "
              f"{int(diag[j - 1, 5]) - prev if diag[j - 1, 5] else -1:7d}  lanes [e row loaded, rescored, reserve in, out] {ls}")
    prev = c
