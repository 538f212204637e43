"""NodeNUMAResource CPU amplification: filterAmplifiedCPUs (plugin.go:336-373), the
amplified cpu request of cpu-bind pods in getResourceOptions (:470-510), the amplified cpuset part of the NUMA
allocations (node_allocation.go:155-177) and of Requested in Score (scoring.go:95-120, 150-168).

The oracle is pinned by the reference's TestFilterWithAmplifiedCPUs table (tests/golden/numa_amplify.json,
tests/golden/make_golden_numa_amp.py); the engine is checked against it case by case and on synthetic C4 clusters
with amplified nodes (placements, totals, cpusets, NodeAllocation: bit-exact)."""
import numpy as np
import pytest

import golden_cases as G
from koordinator_amd import Engine, abi, framework as F, synth
from oracle import oracle

PROFILE = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.NODE_NUMA_RESOURCE),
                    score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.NODE_NUMA_RESOURCE: 1})
NUMA_ONLY = F.Profile(filter=(F.NODE_NUMA_RESOURCE,), score={F.NODE_NUMA_RESOURCE: 1})
GOLD = G.load("numa_amplify.json")


def _amp(v, r):
    return int(np.ceil(v * r)) if r > 1 else v


def golden_case(c):
    """(cfg, kg_node_numa, pod, node requested cpu, node allocatable (cpu, memory)) of one case."""
    s, n, k, t = GOLD["topology"]
    cpus = s * n * k * t
    r = c["ratio"]
    zones = [{"cpu": str(_amp(cpus // (s * n), r)), "memory": GOLD["zone_memory"]}] * (s * n) if c["nrt"] else None
    alloc = list(range(c["existing"])) if c["existing_cpuset"] and c["nrt"] else ()
    nn = F.make_node_numa(s if c["nrt"] else 0, n, k, t, numa_resources=zones, allocated_cpus=alloc,
                          cpu_amplification_ratio=r)
    if c["pod"] is None:
        pod = F.make_pod({})
    elif c["pod_cpuset"]:
        pod = F.make_pod({"cpu": str(c["pod"])}, priority_class="koord-prod", qos="LSR")
    else:
        pod = F.make_pod({"cpu": str(c["pod"])}, priority_class="koord-prod")
    return F.build_config(profile=NUMA_ONLY), nn, pod, c["existing"] * 1000, (_amp(cpus, r) * 1000, 40 << 30)


@pytest.mark.parametrize("c", GOLD["cases"], ids=lambda c: c["name"].replace(" ", "_"))
def test_golden_filter_amplified_oracle(c):
    cfg, nn, pod, req, alloc = golden_case(c)
    ok, _, _ = oracle.numa_eval(cfg, nn, pod, (req, 0), alloc)
    assert ("Success" if ok else "Unschedulable") == c["want"], c["source_line"]


def _cluster(n_nodes, seed):
    cluster, numa = synth.make_numa_cluster(n_nodes, seed=seed)
    ratio = synth.amplify_numa_cluster(cluster, numa, frac=0.4, seed=seed + 1)
    return cluster, numa, ratio


def test_oracle_amplification_changes_placements():
    cfg = F.build_config(profile=PROFILE)
    cluster, numa, ratio = _cluster(200, 61)
    pods = synth.make_numa_pods(800, seed=62)
    st = oracle.states(cluster.n)
    oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
    node, _, cpus, _ = oracle.schedule_full(cfg, cluster.nodes, cluster.metrics, st, pods, cluster.now_ns, 4,
                                            numa_buf=oracle.numa_states(numa))
    numa0 = numa.copy()
    numa0["cpu_amplification_ratio"] = 0  # same capacities, amplification accounting off
    st0 = oracle.states(cluster.n)
    oracle.add_pods(cfg, st0, cluster.existing_pods, cluster.existing_node)
    node0, _, _, _ = oracle.schedule_full(cfg, cluster.nodes, cluster.metrics, st0, pods, cluster.now_ns, 4,
                                          numa_buf=oracle.numa_states(numa0))
    assert (ratio > 1).sum() > 50 and not np.array_equal(node, node0)
    assert (np.isin(node, np.nonzero(ratio > 1)[0]) & (cpus.any(axis=1))).any()  # cpuset pods land on them


@pytest.mark.gpu
@pytest.mark.parametrize("c", GOLD["cases"], ids=lambda c: c["name"].replace(" ", "_"))
def test_golden_filter_amplified_device(c):
    cfg, nn, pod, req, alloc = golden_case(c)
    with Engine(cfg, 1) as e:
        e.upsert_nodes(F.make_node({"cpu": f"{alloc[0]}m", "memory": str(alloc[1])}))
        e.upsert_numa(nn)
        if req:
            e.add_pods(F.make_pod({"cpu": f"{req}m"}), np.zeros(1, np.int32))
        ok, _, _ = e.evaluate_numa(pod)
    assert ("Success" if ok[0] else "Unschedulable") == c["want"], c["source_line"]


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [16, 1])
def test_amplified_cluster_parity(batch):
    cfg = F.build_config(profile=PROFILE, batch_pods=batch, pods_per_wave=1)
    cluster, numa, _ = _cluster(500, 71 + batch)
    pods = synth.make_numa_pods(2000 if batch > 1 else 400, seed=72)
    st = oracle.states(cluster.n)
    oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
    buf = oracle.numa_states(numa)
    want, want_score, want_cpus, _ = oracle.schedule_full(cfg, cluster.nodes, cluster.metrics, st, pods,
                                                          cluster.now_ns, 8, numa_buf=buf)
    with Engine(cfg, cluster.n) as e:
        synth.load_numa_into(e, cluster, numa)
        node, score, _ = e.schedule(pods)
        bad = np.nonzero(node != want)[0]
        assert bad.size == 0, f"first mismatch at pod {bad[0]}: {node[bad[0]]} vs oracle {want[bad[0]]}"
        assert np.array_equal(score, want_score)
        assert np.array_equal(e.fetch_cpusets(0, len(pods)), want_cpus)
        ga, gc, gm = e.read_numa()
        wa, wc, wm = oracle.numa_state_read(buf, cluster.n)
        assert np.array_equal(ga, wa) and np.array_equal(gc, wc) and np.array_equal(gm, wm)


@pytest.mark.gpu
def test_evaluate_numa_amplified_matches_oracle():
    cfg = F.build_config(profile=PROFILE)
    cluster, numa, _ = _cluster(256, 81)
    pods = synth.make_numa_pods(24, seed=82)
    st = oracle.states(cluster.n)
    oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
    alloc = cluster.nodes["allocatable"]
    with Engine(cfg, cluster.n) as e:
        synth.load_numa_into(e, cluster, numa)
        for k in range(len(pods)):
            ok, sc, af = e.evaluate_numa(pods[k:k + 1])
            for i in range(cluster.n):
                want = oracle.numa_eval(cfg, numa[i:i + 1], pods[k:k + 1],
                                        (st["requested"][i, abi.RES_CPU], st["requested"][i, abi.RES_MEMORY]),
                                        (alloc[i, abi.RES_CPU], alloc[i, abi.RES_MEMORY]))
                assert (bool(ok[i]), int(sc[i]), int(af[i])) == want, (k, i)


def _cpubind_amplified_case():
    """One 32-cpu node (2 sockets x 1 NUMA x 8 cores x 2 threads) at cpu ratio 2, SingleNUMANode policy, and an LSR
    pod asking 4 cpus: the hints see the amplified 8000m, the per-NUMA split takes the ORIGINAL 4000m
    (resource_manager.go:205-210), so the pod is placed with 4 cpus and NUMA node 0 records 4000m."""
    cfg = F.build_config(profile=PROFILE)
    zones = [{"cpu": "32", "memory": str(64 << 30)}] * 2
    nn = F.make_node_numa(2, 1, 8, 2, numa_policy="SingleNUMANode", numa_resources=zones, cpu_amplification_ratio=2.0)
    node = F.make_node({"cpu": "64", "memory": str(128 << 30)})
    metric = F.make_node_metric(present=False)
    pod = F.make_pod({"cpu": "4", "memory": str(1 << 30)}, priority_class="koord-prod", qos="LSR")
    return cfg, nn, node, metric, pod


def test_cpubind_amplified_split_oracle():
    cfg, nn, node, metric, pod = _cpubind_amplified_case()
    st = oracle.states(1)
    buf = oracle.numa_states(nn)
    got, _, cpus, _, nalloc = oracle.schedule_full(cfg, node, metric, st, pod, 0, 1, numa_buf=buf,
                                                   with_numa_alloc=True)
    assert got[0] == 0
    assert len(F.cpuset_of(cpus[0])) == 4
    _, c, m = oracle.numa_state_read(buf, 1)
    assert c[0].tolist() == [4000, 0, 0, 0] and m[0].tolist() == [1 << 30, 0, 0, 0]
    oracle.unreserve(cfg, st, pod, 0, numa_buf=buf, cpus=cpus[0], numa_alloc=nalloc[0])
    a, c, m = oracle.numa_state_read(buf, 1)
    assert not a.any() and not c.any() and not m.any()


@pytest.mark.gpu
def test_cpubind_amplified_split_device():
    cfg, nn, node, metric, pod = _cpubind_amplified_case()
    with Engine(cfg, 1) as e:
        e.upsert_nodes(node)
        e.update_metrics(metric, 0)
        e.upsert_numa(nn)
        got, _, _ = e.schedule(pod)
        assert got[0] == 0
        assert len(F.cpuset_of(e.fetch_cpusets(0, 1)[0])) == 4
        _, c, m = e.read_numa()
        assert c[0].tolist() == [4000, 0, 0, 0] and m[0].tolist() == [1 << 30, 0, 0, 0]
        e.unreserve(0, 1)
        a, c, m = e.read_numa()
        assert not a.any() and not c.any() and not m.any()
