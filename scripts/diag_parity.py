"""Diagnostic: locate a GPU/oracle placement mismatch (batch shape sweep + eval-path check)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from koordinator_amd import Engine, framework, synth  # noqa: E402
from oracle import oracle  # noqa: E402

cl = synth.make_cluster(500, seed=synth.BASE_SEED)
pods = synth.make_pods(2000, seed=synth.BASE_SEED + 1)
for B, ppw in [(1, 1), (2, 1), (2, 2), (4, 1), (32, 2)]:
    cfg = framework.build_config(batch_pods=B, pods_per_wave=ppw)
    on, osc, _ = oracle.schedule_cluster(cfg, cl, pods)
    with Engine(cfg, cl.n) as e:
        synth.load_into(e, cl)
        gn, gs, st = e.schedule(pods)
        bad = np.nonzero(gn != on)[0]
        print(f"B={B} ppw={ppw}: mismatches {len(bad)} first {bad[:5]} gpu {gn[bad[:5]]} {gs[bad[:5]]} "
              f"oracle {on[bad[:5]]} {osc[bad[:5]]} rounds {st['device_batches']}", flush=True)
with Engine(framework.build_config(), cl.n) as e:
    synth.load_into(e, cl)
    e.stage(pods[:100])
    print("eval path mismatches:", e.debug_eval_paths())
