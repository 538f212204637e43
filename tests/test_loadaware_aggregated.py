"""LoadAware percentile (aggregated) usage: Filter against Aggregated.UsageThresholds on the chosen
AggregatedNodeUsages entry (load_aware.go:155-161, 173-224; helper.go:58-140) and Score on
Aggregated.ScoreAggregationType (load_aware.go:307-326).  The oracle is pinned by the reference's aggregated test
cases (tests/golden/loadaware_*.json, scope core: test_golden_oracle.py); here the engine is checked against it on
synthetic clusters whose nodes report several periods / percentiles, some none."""
import numpy as np
import pytest

from koordinator_amd import Engine, abi, framework as F, synth
from oracle import oracle

MI, GI = 1 << 20, 1 << 30


def aggregated_cluster(n_nodes, seed):
    """make_cluster's nodes + AggregatedNodeUsages (5m / 30m / 1h periods; avg, p50, p90, p95, p99 each present
    70 %) on 80 % of the nodes with a NodeMetric, and a custom AggregatedUsage annotation on 10 % of them."""
    cluster = synth.make_cluster(n_nodes, seed=seed)
    rng = np.random.default_rng(seed + 1)
    m = cluster.metrics
    cpu = cluster.nodes["allocatable"][:, abi.RES_CPU]
    mem = cluster.nodes["allocatable"][:, abi.RES_MEMORY]
    for i in np.nonzero(m["has_node_metric"] & (rng.random(n_nodes) < 0.8))[0]:
        k = int(rng.integers(1, 4))
        m["agg_count"][i] = k
        for d in range(k):
            m["agg_duration_ns"][i, d] = int(rng.choice([300, 1800, 3600])) * 10**9
            for t in range(5):
                if rng.random() < 0.7:
                    m["agg_usage"][i, d, t, 0] = int(rng.random() * 0.9 * cpu[i])
                    m["agg_usage"][i, d, t, 1] = int(rng.random() * 0.95 * mem[i] / MI) * MI
                    m["agg_present"][i, d, t] = 3
    nodes = cluster.nodes
    cust = rng.random(n_nodes) < 0.1
    nodes["custom_agg_thresholds"] = -1
    nodes["custom_agg_thresholds"][cust, abi.RES_CPU] = rng.integers(40, 90, cust.sum())
    nodes["custom_agg_type"] = np.where(cust, abi.AGG_TYPES["p90"], 0)
    nodes["flags"] |= np.where(cust, abi.NODE_HAS_CUSTOM_THRESHOLDS, 0)
    return cluster


def config(filter_type="p95", filter_dur=300, score_type="p95", score_dur=0):
    la = F.LoadAwareSchedulingArgs(aggregated=dict(usage_thresholds={"cpu": 60, "memory": 80}, usage_type=filter_type,
                                                   usage_duration_s=filter_dur, score_type=score_type,
                                                   score_duration_s=score_dur))
    return F.build_config(la=la)


def test_oracle_aggregation_matters():
    cluster = aggregated_cluster(400, 11)
    pods = synth.make_pods(1500, seed=12)
    outs = []
    for cfg in (config(), F.build_config()):
        st = oracle.states(cluster.n)
        oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
        outs.append(oracle.schedule(cfg, cluster.nodes, cluster.metrics, st, pods, cluster.now_ns, 4)[0])
    assert not np.array_equal(outs[0], outs[1])


@pytest.mark.gpu
@pytest.mark.parametrize("ft,fd,stype,sd", [("p95", 300, "p95", 0), ("avg", 0, "p99", 1800), ("p50", 3600, "", 0),
                                            ("", 0, "p90", 300)])
def test_aggregated_parity(ft, fd, stype, sd):
    cfg = config(ft, fd, stype, sd)
    cluster = aggregated_cluster(2000, 21)
    pods = synth.make_pods(4000, seed=22)
    st = oracle.states(cluster.n)
    oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
    want, want_score = oracle.schedule(cfg, cluster.nodes, cluster.metrics, st, pods, cluster.now_ns, 8)
    with Engine(cfg, cluster.n) as e:
        synth.load_into(e, cluster)
        node, score, _ = e.schedule(pods)
    bad = np.nonzero(node != want)[0]
    assert bad.size == 0, f"first mismatch at pod {bad[0]}: {node[bad[0]]} vs oracle {want[bad[0]]}"
    assert np.array_equal(score, want_score)
