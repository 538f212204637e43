"""The NodeNUMAResource oracle restatement (oracle/numa.c) against the reference's own test tables
(tests/golden/numa_*.json, transcribed by tests/golden/make_golden_numa.py with source lines)."""
import numpy as np
import pytest

import golden_cases as G
from koordinator_amd import framework
from koordinator_amd.quantity import resource_value
from oracle import oracle

NUMA_PROFILE = framework.Profile(filter=(framework.NODE_NUMA_RESOURCE,), score={framework.NODE_NUMA_RESOURCE: 1})


def _cases(name):
    d = G.load(name)
    return [(d, c) for c in d["cases"]]


def _id(dc):
    c = dc[1]
    return c.get("name", c["source_line"].split(":")[-1]).replace(" ", "_")


@pytest.mark.parametrize("dc", _cases("numa_take_cpus.json"), ids=_id)
def test_take_cpus(dc):
    _, c = dc
    s, n, k, t = c["topo"]
    total = s * n * k * t
    avail = [x for x in range(total) if x not in set(c["alloc"])]
    got = oracle.take_cpus(tuple(c["topo"]), avail, c["need"], c["policy"], c["strategy"])
    assert got == sorted(c["want"]), c["source_line"]


@pytest.mark.parametrize("dc", _cases("numa_take_cpus_exclusive.json"), ids=_id)
def test_take_cpus_exclusive(dc):
    """TestTakeCPUsWithExclusivePolicy: the pod's exclusive policy filters the cores / NUMA nodes holding cpus of
    the same policy; the allocated cpus hold alloc_policy."""
    _, c = dc
    s, n, k, t = c["topo"]
    total = s * n * k * t
    avail = [x for x in range(total) if x not in set(c["alloc"])]
    seed = c["alloc"] if c["alloc_policy"] == c["excl"] else []
    got = oracle.take_cpus(tuple(c["topo"]), avail, c["need"], c["policy"], c["strategy"],
                           exclusive_policy=c["excl"], exclusive_cpus=seed)
    assert got == sorted(c["want"]), c["source_line"]


def filter_case(c):
    """(config, kg_node_numa, kg_pod) of one TestPlugin_Filter case."""
    cfg = framework.build_config(profile=NUMA_PROFILE)
    zones = [{"cpu": "8", "memory": "32Gi"}] * 2  # CPUsPerNode cores + 32Gi per zone (:779-786)
    nn = framework.make_node_numa(2, 1, 4, 2, numa_policy=c["numa_policy"], node_cpu_bind_policy=c["node_bind"],
                                  numa_resources=zones)
    pod = framework.make_pod({"cpu": str(c["cpus"])}, priority_class="koord-prod", qos="LSR",
                             required_cpu_bind_policy=c["required"], preferred_cpu_bind_policy=c["preferred"])
    return cfg, nn, pod


@pytest.mark.parametrize("dc", _cases("numa_filter.json"), ids=_id)
def test_filter(dc):
    _, c = dc
    cfg, nn, pod = filter_case(c)
    ok, _, _ = oracle.numa_eval(cfg, nn, pod, (0, 0), (96000, 512 << 30))
    assert ("Success" if ok else "UnschedulableAndUnresolvable") == c["want"], c["source_line"]


def reserve_case(c):
    cfg = framework.build_config(profile=NUMA_PROFILE)
    nn = framework.make_node_numa(*c["topo"], node_cpu_bind_policy=c["node_bind"],
                                  numa_allocate_strategy=c["strategy"], allocated_cpus=c["alloc"])
    pod = framework.make_pod({"cpu": str(c["cpus"])}, priority_class="koord-prod", qos="LSR",
                             preferred_cpu_bind_policy=c["preferred"])
    return cfg, nn, pod


@pytest.mark.parametrize("dc", _cases("numa_reserve.json"), ids=_id)
def test_reserve(dc):
    _, c = dc
    cfg, nn, pod = reserve_case(c)
    rc, cpus = oracle.numa_reserve(cfg, nn, pod)
    if c["want"] is None:
        assert rc != 0, c["source_line"]
    else:
        assert rc == 0 and cpus == sorted(c["want"]), c["source_line"]


def score_nodes(c):
    """Per node of a TestNUMANodeScore case: (kg_node_numa, requested (cpu, mem), allocatable (cpu, mem))."""
    out = []
    for i, nd in enumerate(c["nodes"]):
        count = c["numa_counts"][i]
        cpu_m, mem = resource_value("cpu", nd["cpu"]), resource_value("memory", nd["memory"])
        zones = [{"cpu": f"{cpu_m // count}m", "memory": str(mem // count)}] * count
        pods = [e for e in c["existing"] if e["node"] == i]
        req_c = sum(resource_value("cpu", e["cpu"]) for e in pods)
        req_m = sum(resource_value("memory", e["memory"]) for e in pods)
        cpus = set()
        for e in pods:
            if e["qos"] == "LSR":  # AllowUseCPUSet: cpus 0..n-1 (:291-298)
                cpus |= set(range(resource_value("cpu", e["cpu"]) // 1000))
        alloc = {0: {"cpu": f"{req_c}m", "memory": str(req_m)}} if pods else None
        nn = framework.make_node_numa(count, 1, cpu_m // 1000 // 2 // count, 2, numa_policy=nd["numa_policy"],
                                      numa_resources=zones, allocated_cpus=sorted(cpus), numa_allocated=alloc)
        out.append((nn, (req_c, req_m), (cpu_m, mem)))
    return out


def score_case(c):
    numa = framework.NodeNUMAResourceArgs(scoring_strategy=c["strategy"])
    cfg = framework.build_config(profile=NUMA_PROFILE, numa=numa)
    p = c["pod"]
    pod = framework.make_pod({"cpu": p["cpu"], "memory": p["memory"]},
                             priority_class="koord-prod" if p["qos"] == "LSR" else "", qos=p["qos"])
    return cfg, pod


@pytest.mark.parametrize("dc", _cases("numa_score.json"), ids=_id)
def test_score(dc):
    _, c = dc
    cfg, pod = score_case(c)
    got = []
    for nn, req, alloc in score_nodes(c):
        ok, score, _ = oracle.numa_eval(cfg, nn, pod, req, alloc)
        assert ok, c["source_line"]
        got.append(score)
    assert got == c["want"], c["source_line"]


def affinity_case(doc, c):
    numa = framework.NodeNUMAResourceArgs(numa_scoring_strategy=c["numa_strategy"])
    cfg = framework.build_config(profile=NUMA_PROFILE, numa=numa)
    count = c["count"]
    cpu_m, mem = 104000, 256 << 30
    zones = [{"cpu": f"{cpu_m // count}m", "memory": str(mem // count)}] * count
    alloc = {}
    for z, pods in c["existing"].items():
        alloc[int(z)] = {"cpu": f"{sum(resource_value('cpu', a) for a, _ in pods)}m",
                         "memory": str(sum(resource_value("memory", b) for _, b in pods))}
    nn = framework.make_node_numa(count, 1, 104 // 2 // count, 2, numa_policy=c["policy"], numa_resources=zones,
                                  numa_allocated=alloc)
    pod = framework.make_pod({"cpu": doc["pod"]["cpu"], "memory": doc["pod"]["memory"]})
    return cfg, nn, pod


@pytest.mark.parametrize("dc", _cases("numa_affinity.json"), ids=_id)
def test_affinity(dc):
    doc, c = dc
    cfg, nn, pod = affinity_case(doc, c)
    ok, _, mask = oracle.numa_eval(cfg, nn, pod, (0, 0), (104000, 256 << 30))
    assert ok, c["source_line"]
    assert [b for b in range(4) if (mask >> b) & 1] == c["want"], c["source_line"]
