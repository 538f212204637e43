"""Diagnostic (r6): drive numa_eval.hip builds over C4 rows / pods; cycles per step and a bit-for-bit comparison of the
results between the builds.  usage: numa_eval.py lib_a.so [lib_b.so ...]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from koordinator_amd import abi, framework, synth  # noqa: E402

F = framework
profile = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.NODE_NUMA_RESOURCE),
                    score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.NODE_NUMA_RESOURCE: 1})
cfg = framework.build_config(device_id=0, batch_pods=16, pods_per_wave=1, profile=profile).reshape(-1)[0]
NP = np.array([cfg["numa_filter"], cfg["numa_score"], cfg["weight_numa"], cfg["numa_scoring_strategy"],
               cfg["numa_numa_scoring_strategy"], cfg["numa_scoring_weights"][0], cfg["numa_scoring_weights"][1],
               cfg["numa_numa_scoring_weights"][0], cfg["numa_numa_scoring_weights"][1],
               1 if cfg["numa_numa_scoring_strategy"] == abi.STRATEGY["MostAllocated"] else 0], dtype=np.int32)
R = int(os.environ.get("R", "24"))
P = int(os.environ.get("P", "768"))
cl, numa = synth.make_numa_cluster(2000, seed=synth.BASE_SEED + 4)
rng = np.random.default_rng(7)
rows = np.sort(rng.choice(2000, R, replace=False))
req = np.zeros((2000, 2), dtype=np.int64)
np.add.at(req, cl.existing_node, cl.existing_pods["requests"][:, [abi.RES_CPU, abi.RES_MEMORY]])
node_req = np.ascontiguousarray(np.stack([req[rows, 0], req[rows, 1], cl.nodes["allocatable"][rows, abi.RES_CPU],
                                          cl.nodes["allocatable"][rows, abi.RES_MEMORY]], axis=1).astype(np.int64))
nodes = np.ascontiguousarray(numa[rows])
pods = np.ascontiguousarray(synth.make_numa_pods(P, seed=synth.BASE_SEED + 5))
cpuset = np.isin(pods["qos"], [abi.QOS["LSR"], abi.QOS["LSE"]]) & (pods["requests"][:, abi.RES_CPU] % 1000 == 0) & \
    (pods["requests"][:, abi.RES_CPU] > 0)

out = []
MODES = {6: "pair: waves 0 + 1", 7: "pair: waves 0 + 2", 1: "admit only", 2: "filter only", 3: "score only (nil affinity)", 4: "reserve = feasible only",
         5: "reserve = take_cpus only"}
for lib_path in sys.argv[1:]:
  for mode in [0] + [int(m) for m in os.environ.get("MODES", "").split(",") if m]:
      lib = ctypes.CDLL(os.path.abspath(lib_path))
      cyc = np.zeros((P, 3), dtype=np.uint64)
      res = np.zeros((P, 64, 2), dtype=np.int64)
      cps = np.zeros((P, 5), dtype=np.uint64)
      p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
      rc = lib.micro_numa(p(nodes), p(node_req), ctypes.c_int(R), p(pods), ctypes.c_int(P), p(NP),
                          ctypes.c_int(int(cfg["numa_default_cpu_bind_policy"])), p(cyc), p(res), p(cps),
                            ctypes.c_int(mode))
      assert rc == 0, rc
      if mode >= 6:
          print(f"{lib_path} [{MODES[mode]}]: R={R} P={P}  wave 0 eval mean {cyc[:, 0].astype(float).mean():.0f} | "
                f"second wave (one row, uniform) eval mean {cyc[:, 1].astype(float).mean():.0f}")
          continue
      ok = (cps[:, 4] >> 1) & 1
      placed = cps[:, 4] & 1
      e = cyc[:, 0].astype(np.float64)
      r = cyc[:, 1].astype(np.float64)
      print(f"{lib_path} [{MODES.get(mode, 'eval + reserve')}]: R={R} P={P}  eval mean {e.mean():.0f} p50 {np.median(e):.0f} max {e.max():.0f} | "
            f"reserve cpuset mean {r[(ok == 1) & cpuset].mean():.0f} p50 {np.median(r[(ok == 1) & cpuset]):.0f}, "
            f"other mean {r[(ok == 1) & ~cpuset].mean():.0f} | view mean {cyc[:, 2].astype(np.float64).mean():.0f} | "
            f"feasible {(res[:, :R, 0] >= 0).mean():.3f} placed {placed.sum()}/{ok.sum()}")
      if mode == 0:
          out.append((res[:, :R].copy(), cps.copy()))
for k in range(1, len(out)):
    same = np.array_equal(out[0][0], out[k][0]) and np.array_equal(out[0][1], out[k][1])
    print(f"results {sys.argv[1]} vs {sys.argv[1 + k]}: {'IDENTICAL' if same else 'DIFFER'}")
    if not same:
        d = np.argwhere(out[0][0] != out[k][0])
        print("  first eval differences (pod, row, field):", d[:8].tolist())
        d = np.argwhere(out[0][1] != out[k][1])
        print("  first reserve differences (pod, word):", d[:8].tolist())
        sys.exit(1)
