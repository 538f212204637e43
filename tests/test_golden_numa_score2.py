"""NodeNUMAResource Score against two more of the reference's tables (transcribed by
tests/golden/make_golden_numa_score2.py with source lines):

* TestPlugin_Score (scoring_test.go:332-554): Score with no Filter before it (a Score-only profile, so no stored
  affinity), MostAllocated over cpu, cpuset pods under FullPCPUs / SpreadByPCPUs, the node NUMA-allocate-strategy and
  node cpu-bind-policy labels.  Three cases write a preFilterState PreFilter never produces; they are skipped with the
  reason in the fixture.
* TestScoreWithAmplifiedCPUs (scoring_test.go:556-814): scoreWithAmplifiedCPUs and the amplified cpuset part of
  Requested on ratio-2 nodes, cpuset and non-cpuset pods, LeastAllocated and MostAllocated.

Each case runs on the oracle and, through kg_pods_evaluate_numa, on the device."""
import numpy as np
import pytest

import golden_cases as G
from koordinator_amd import Engine, framework as F
from koordinator_amd.quantity import resource_value
from oracle import oracle

SCORE_ONLY = F.Profile(filter=(), score={F.NODE_NUMA_RESOURCE: 1})
PS = G.load("numa_plugin_score.json")
AMP = G.load("numa_score_amplified.json")


def plugin_score_case(c):
    """(cfg, kg_node_numa, pod, node allocatable (cpu, memory)) of a TestPlugin_Score case."""
    numa = F.NodeNUMAResourceArgs(scoring_strategy=PS["strategy"], scoring_resources=PS["resources"])
    cfg = F.build_config(profile=SCORE_ONLY, numa=numa)
    topo = c["topo"]
    if topo:
        nn = F.make_node_numa(*topo, numa_allocate_strategy=c["labels"].get("numa_allocate_strategy"),
                              node_cpu_bind_policy=c["labels"].get("node_cpu_bind_policy", ""))
        cpus = topo[0] * topo[1] * topo[2] * topo[3]
    else:
        nn = F.make_node_numa()
        cpus = 96
    if c["needed"]:
        pod = F.make_pod({"cpu": str(c["needed"])}, priority_class="koord-prod", qos="LSR",
                         preferred_cpu_bind_policy=c["preferred"])
    else:
        pod = F.make_pod({})
    return cfg, nn, pod, (cpus * 1000, resource_value("memory", PS["node_memory"]))


def amplified_nodes(c):
    """Per node of a TestScoreWithAmplifiedCPUs case: (kg_node_numa, requested (cpu, mem), allocatable (cpu, mem))."""
    out = []
    s, n, k, t = AMP["topology"]
    ex = AMP["existing_pod"]
    for nd in AMP["nodes"]:
        r = nd["ratio"]
        alloc = (resource_value("cpu", nd["cpu"]), resource_value("memory", nd["memory"]))
        req = (0, 0) if c["existing"] is None else (resource_value("cpu", ex["cpu"]), resource_value("memory", ex["memory"]))
        if c["nrt"]:
            per = int(np.ceil(n * k * t * r)) if r > 1 else n * k * t  # Amplify(CPUsPerNode, ratio)
            zones = [{"cpu": str(per), "memory": AMP["zone_memory"]}] * (s * n)
            held = list(range(req[0] // 1000)) if c["existing"] else []
            nn = F.make_node_numa(s, n, k, t, numa_resources=zones, allocated_cpus=held, cpu_amplification_ratio=r)
        else:
            nn = F.make_node_numa(cpu_amplification_ratio=r)
        out.append((nn, req, alloc))
    return out


def amplified_case(c):
    numa = F.NodeNUMAResourceArgs(scoring_strategy=c["strategy"], scoring_resources=AMP["resources"])
    cfg = F.build_config(profile=SCORE_ONLY, numa=numa)
    p = AMP["pod"]
    pod = F.make_pod({"cpu": p["cpu"], "memory": p["memory"]}, priority_class="koord-prod",
                     qos="LSR" if c["pod_cpuset"] else "")
    return cfg, pod


@pytest.mark.parametrize("c", PS["cases"], ids=lambda c: c["source_line"].split(":")[-1])
def test_plugin_score_oracle(c):
    cfg, nn, pod, alloc = plugin_score_case(c)
    ok, score, _ = oracle.numa_eval(cfg, nn, pod, (0, 0), alloc)
    assert ok and score == c["want"], c["source_line"]


@pytest.mark.parametrize("c", AMP["cases"], ids=lambda c: c["source_line"].split(":")[-1])
def test_score_amplified_oracle(c):
    cfg, pod = amplified_case(c)
    got = [oracle.numa_eval(cfg, nn, pod, req, alloc)[1] for nn, req, alloc in amplified_nodes(c)]
    assert got == c["want"], c["source_line"]


def _device_score(cfg, nn, pod, req, alloc):
    with Engine(cfg, 1) as e:
        e.upsert_nodes(F.make_node({"cpu": f"{alloc[0]}m", "memory": str(alloc[1])}))
        e.upsert_numa(nn)
        if req[0] or req[1]:
            e.add_pods(F.make_pod({"cpu": f"{req[0]}m", "memory": str(req[1])}), np.zeros(1, np.int32))
        ok, sc, _ = e.evaluate_numa(pod)
    return bool(ok[0]), int(sc[0])


@pytest.mark.gpu
@pytest.mark.parametrize("c", PS["cases"], ids=lambda c: c["source_line"].split(":")[-1])
def test_plugin_score_device(c):
    cfg, nn, pod, alloc = plugin_score_case(c)
    assert _device_score(cfg, nn, pod, (0, 0), alloc) == (True, c["want"]), c["source_line"]


@pytest.mark.gpu
@pytest.mark.parametrize("c", AMP["cases"], ids=lambda c: c["source_line"].split(":")[-1])
def test_score_amplified_device(c):
    cfg, pod = amplified_case(c)
    got = [_device_score(cfg, nn, pod, req, alloc)[1] for nn, req, alloc in amplified_nodes(c)]
    assert got == c["want"], c["source_line"]
