"""Synthetic generator determinism and the oracle's threaded scheduling loop (CPU)."""
import numpy as np

from koordinator_amd import abi, framework, synth
from oracle import oracle


def test_generator_is_deterministic():
    a = synth.make_cluster(300, seed=7)
    b = synth.make_cluster(300, seed=7)
    assert a.nodes.tobytes() == b.nodes.tobytes() and a.metrics.tobytes() == b.metrics.tobytes()
    assert a.existing_pods.tobytes() == b.existing_pods.tobytes()
    p = synth.make_pods(1000, seed=3)
    assert p.tobytes() == synth.make_pods(1000, seed=3).tobytes()
    assert (p["requests"][:, abi.RES_CPU] > 0).all() and (p["requests"][:, abi.RES_MEMORY] > 0).all()


def test_threaded_oracle_matches_sequential():
    cfg = framework.build_config()
    cl = synth.make_cluster(700, seed=11)
    pods = synth.make_pods(2000, seed=12)
    n1, s1, st1 = oracle.schedule_cluster(cfg, cl, pods, n_threads=1)
    n4, s4, st4 = oracle.schedule_cluster(cfg, cl, pods, n_threads=4)
    assert np.array_equal(n1, n4) and np.array_equal(s1, s4) and st1.tobytes() == st4.tobytes()


def test_oracle_lowest_index_tie_break():
    cfg = framework.build_config()
    nodes = np.concatenate([framework.make_node({"cpu": "8", "memory": "16Gi"}) for _ in range(5)])
    metrics = np.concatenate([framework.make_node_metric(update_time_ns=0, node_usage={"cpu": "0", "memory": "0"})
                              for _ in range(5)])
    st = oracle.states(5)
    pods = np.concatenate([framework.make_pod({"cpu": "1", "memory": "1Gi"}) for _ in range(3)])
    node, score = oracle.schedule(cfg, nodes, metrics, st, pods, now_ns=10**9)
    # identical nodes: first pod → node 0; node 0 then scores lower → node 1, then node 2
    assert list(node) == [0, 1, 2]
