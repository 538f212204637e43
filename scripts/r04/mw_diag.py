"""Resolver diagnostics on the C3 cluster: per-round active time, chain re-scores and helper waits per pod.
usage: KG_RESOLVER=mw|1wave python scripts/r04/mw_diag.py [nodes] [pods] [depth]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from koordinator_amd import Engine, framework, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
m = int(sys.argv[2]) if len(sys.argv) > 2 else 40_000
depth = int(sys.argv[3]) if len(sys.argv) > 3 else 0
cfg = framework.build_config(pipeline_depth=depth)
cl = synth.make_cluster(n, seed=synth.BASE_SEED + 3)
pods = synth.make_pods(2 * m, seed=synth.BASE_SEED + 4)
with Engine(cfg, cl.n) as e:
    synth.load_into(e, cl)
    e.stage(pods)
    e.schedule_staged(0, m // 4)  # warm
    t = time.perf_counter()
    st = e.schedule_staged(m // 4, m)
    dt = time.perf_counter() - t
    r = int(st["device_batches"])
    print(f"{os.environ.get('KG_RESOLVER', 'mw')} depth={depth or 2} nodes={n} pods={m}: {m / dt:,.0f} pods/s, "
          f"{dt / r * 1e6:.1f} us/round, active {st['reserved'][2] / r * 1e6:.1f} us/round, "
          f"chain re-scores {st['reserved'][0] / m:.2f}/pod, helper waits {st['reserved'][1] / m:.2f}/pod, "
          f"{m / r:.1f} pods/round", flush=True)
