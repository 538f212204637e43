"""Diagnostic: per-pod cycle stamps inside the two-wave resolve_round_numa2 at C4 size (KG_STAMPS dev build).
usage: stamps_numa.py [nodes] [pods] [batch]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["KOORDGPU_LIB"] = os.path.join(ROOT, "koordinator_amd", os.environ.get("STAMPS_LIB", "libkoordgpu_dev.so"))
if os.path.isabs(os.environ.get("STAMPS_LIB", "")):
    os.environ["KOORDGPU_LIB"] = os.environ["STAMPS_LIB"]
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
print("== two-wave resolver per pod (last launch), cycles from the scorer's phase A start:")
print("   scorer A [views refreshed, e staged, rows evaluated] | reserver A: Reserve, eval | phase B | pod period")
prev = None
for j in range(64):
    t = [int(x) for x in diag[j]]
    if not t[0]:
        break
    s0 = t[0]
    per = (t[0] - prev) if prev else 0
    ls = [int(x) - s0 if int(x) else -1 for x in lane[j][:3]]
    print(f"  pod {j:2d}: S {t[1] - s0:7d} {ls} | R {t[2] - s0:6d} -> {t[3] - s0 if t[3] else -1:7d} -> {t[4] - s0:7d} | "
          f"B end {t[5] - s0:7d} | period {per:7d}")
    prev = t[0]
