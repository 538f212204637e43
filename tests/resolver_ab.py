"""Parity of the look-ahead resolver (resolve_mw, selected with KG_RESOLVER=mw, read once per process): run as a
child process by test_parity_gpu.test_lookahead_resolver_parity.  Exit status 0 = every case matched the oracle."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from koordinator_amd import Engine, abi, framework, synth  # noqa: E402
from oracle import oracle  # noqa: E402


def parity(cfg, cluster, pods):
    on, os_, st = oracle.schedule_cluster(cfg, cluster, pods, n_threads=4)
    with Engine(cfg, cluster.n) as e:
        synth.load_into(e, cluster)
        gn, gs, _ = e.schedule(pods)
        s = e.read_state()
    bad = np.nonzero((gn != on) | (gs != os_))[0]
    assert bad.size == 0, f"first mismatch at pod {bad[:5]}: gpu {gn[bad[:5]]} oracle {on[bad[:5]]}"
    assert np.array_equal(s["requested_cpu"], st["requested"][:, abi.RES_CPU])
    assert np.array_equal(s["num_pods"], st["num_pods"])


def main():
    assert os.environ.get("KG_RESOLVER") == "mw"
    cl = synth.make_cluster(1500, seed=23)
    pods = synth.make_pods(4000, seed=24)
    for depth, batch in [(1, 32), (2, 32), (3, 32), (4, 13), (2, 64)]:
        parity(framework.build_config(batch_pods=batch, pods_per_wave=8, pipeline_depth=depth), cl, pods)
    n = 300  # tie-heavy: identical nodes, most pods take the re-score path
    nodes = np.concatenate([framework.make_node({"cpu": "16", "memory": "64Gi"}) for _ in range(n)])
    metrics = np.concatenate([framework.make_node_metric(update_time_ns=synth.T0_NS,
                                                         node_usage={"cpu": "1", "memory": "1Gi"}) for _ in range(n)])
    ties = synth.Cluster(nodes, metrics, np.zeros(0, dtype=abi.POD_DTYPE), np.zeros(0, dtype=np.int32),
                         synth.T0_NS + 10**9)
    parity(framework.build_config(pipeline_depth=2), ties, synth.make_pods(2500, seed=25))
    print("resolve_mw parity: ok")


if __name__ == "__main__":
    main()
