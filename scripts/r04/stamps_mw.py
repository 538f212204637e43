"""Diagnostic (KG_STAMPS build of profile 15): look-ahead resolver per-pod stamps of the last launch.
Chain: cycles of each pod and its sub-steps [T read, decided, placed, published]; helper(j): its
[start, rows advanced, keyed, T published] relative to the chain's start of pod j (negative = ahead)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["KOORDGPU_LIB"] = os.path.join(ROOT, "koordinator_amd", os.environ.get("STAMPS_LIB", "libkoordgpu_dev.so"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from koordinator_amd import Engine, abi, framework, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
npods = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
depth = int(sys.argv[3]) if len(sys.argv) > 3 else 0
cfg = framework.build_config(device_id=0, pipeline_depth=depth)
cl = synth.make_cluster(n, seed=synth.BASE_SEED + 3)
pods = synth.make_pods(npods, seed=synth.BASE_SEED + 4)
with Engine(cfg, n) as e:
    synth.load_into(e, cl)
    e.stage(pods)
    st = e.schedule_staged(0, npods)
    buf = np.zeros(4 * 32 * 2 + 64 * 6 + 2 + 64 * 8, dtype=np.uint64)
    abi.check(e.lib, e.lib.kg_debug_stamps(e.h, abi.ptr(buf)))
    stamps = buf[:256].reshape(4, 32, 2).astype(np.int64)
    diag = buf[256:256 + 384].reshape(64, 6).astype(np.int64)
    lane = buf[256 + 384 + 2:].reshape(64, 8).astype(np.int64)
r = int(st["device_batches"])
print(f"nodes={n} pods={npods}: rounds={r} re-scores/pod={st['reserved'][0] / npods:.2f} waits/pod="
      f"{st['reserved'][1] / npods:.2f} active/round={st['reserved'][2] / r * 1e6:.1f} us")
pts = [(i, int(stamps[2, i, 0]), int(stamps[2, i, 1])) for i in range(32) if stamps[2, i, 0]]
if pts:
    print("resolver points:", " ".join(f"pt{i}:+{c - pts[0][1]}" for i, c, _ in pts),
          f"(clock {(pts[-1][1] - pts[0][1]) / max(1, pts[-1][2] - pts[0][2]) * 100:.0f} MHz)")
for j in range(63):
    c, c1 = int(diag[j, 0]), int(diag[j + 1, 0])
    if not c or not c1:
        break
    sub = " ".join(f"{int(diag[j, 2 + k]) - c:6d}" for k in range(4))
    hl = " ".join(f"{int(lane[j, k]) - c:8d}" if lane[j, k] else "       -" for k in range(4))
    print(f"pod {j:2d}: {c1 - c:6d} cyc waits={int(diag[j, 1])}  chain [T, decided, placed, published] {sub}"
          f"   helper [start, rows, keyed, T] {hl}")
