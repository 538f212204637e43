"""The oracle (CPU restatement) against the golden vectors transcribed from the reference's own tests.

This pins the oracle before it is trusted as the checker of the HIP engine.  Cases whose scope is "next"
(aggregated usages, PodsMetric-based estimation) are skipped with the reason."""
import numpy as np
import pytest

import golden_cases as G
from koordinator_amd import abi, framework
from oracle import oracle


@pytest.mark.parametrize("dc", G.cases("estimator_pod.json"), ids=G.case_id)
def test_estimate_pod(dc):
    doc, case = dc
    cfg = G.config(doc, case)
    got = oracle.estimate_pod(cfg, G.pod(case["pod"]))
    assert got == (case["want"]["cpu"], case["want"]["memory"]), case["source_line"]


@pytest.mark.parametrize("dc", G.cases("estimator_node.json"), ids=G.case_id)
def test_estimate_node(dc):
    _, case = dc
    node = framework.make_node(case["allocatable"], raw_allocatable=case["raw"])
    for k, v in G.quantity_map(case["want"]).items():
        assert oracle.estimate_node(node, abi.RESOURCE_SLOTS[k]) == v, case["source_line"]


def _filter_cases():
    return G.cases("loadaware_filter.json") + G.cases("loadaware_filter_expired.json")


@pytest.mark.parametrize("dc", _filter_cases(), ids=G.case_id)
def test_loadaware_filter(dc):
    doc, case = dc
    cfg = G.config(doc, case)
    got = oracle.loadaware_filter(cfg, G.node(doc, case), G.metric(case), G.pod(case.get("pod")), G.NOW_NS)
    assert got in (0, 1), f"unsupported ({got})"
    assert ("Success" if got == 0 else "Unschedulable") == case["want"], case["source_line"]


@pytest.mark.parametrize("dc", G.cases("loadaware_score.json"), ids=G.case_id)
def test_loadaware_score(dc):
    doc, case = dc
    cfg = G.config(doc, case)
    st = oracle.states(1)
    a = G.assigned(case)
    if len(a):
        oracle.add_pods(cfg, st, a, np.zeros(len(a), dtype=np.int32))
    m = G.metric(case)
    pm = G.pods_metric(case)
    if len(pm):  # PodsMetric reported: the estimated / actual usage terms of the assigned pods
        oracle.set_la_terms(st, 0, oracle.la_node_terms(cfg, m, pm, G.oracle_assigned(cfg, a)))
    got = oracle.loadaware_score(cfg, G.node(doc, case), m, st, G.pod(case.get("pod")), G.NOW_NS)
    assert got == case["want"], case["source_line"]


def test_every_reference_case_is_in_scope():
    """The aggregated-usage cases (round 1) and the PodsMetric-based estimation cases (round 2, load_aware_test.go
    :1203 and :1588) moved into scope: no fixture is skipped any more."""
    nxt = [c["name"] for f in ("loadaware_filter.json", "loadaware_score.json")
           for c in G.load(f)["cases"] if c["scope"] == "next"]
    assert nxt == [], nxt
    lines = {int(c["source_line"].rsplit(":", 1)[1]) for c in G.load("loadaware_score.json")["cases"]}
    assert {1203, 1588} <= lines


@pytest.mark.parametrize("req,cap,want", [(0, 0, 0), (5, 0, 0), (11, 10, 0), (10, 10, 0), (0, 10, 100),
                                          (1, 3, 66), (60000, 96000, 37), (-5, 10, 150)])
def test_least_requested_known_answers(req, cap, want):
    # loadaware/load_aware.go:388-397: ((capacity - requested) * 100) / capacity with Go truncation
    assert oracle.least_requested(req, cap) == want


def test_fit_known_answers():
    """Upstream NodeResourcesFit (parity unpinned: no reference test exists) — hand-derived values from the
    v1.24 formulas restated in nodenumaresource/scoring.go:191-230 + least_allocated.go:30-58."""
    cfg = framework.build_config()
    node = framework.make_node({"cpu": "4", "memory": "8Gi"}, allowed_pods=2)
    st = oracle.states(1)
    st[0]["requested"][0], st[0]["requested"][1] = 1000, 2 << 30
    st[0]["nonzero"][:] = (1000, 2 << 30)
    st[0]["num_pods"] = 1
    pod = framework.make_pod({"cpu": "1", "memory": "2Gi"})
    assert oracle.fit_filter(node, st, pod) == 0
    # cpu: (4000-2000)*100/4000 = 50; mem: (8Gi-4Gi)*100/8Gi = 50 → 50
    assert oracle.fit_score(cfg, node, st, pod) == 50
    big = framework.make_pod({"cpu": "3500m"})
    assert oracle.fit_filter(node, st, big) == abi.REJECT_FIT_CPU
    st[0]["num_pods"] = 2
    assert oracle.fit_filter(node, st, pod) & abi.REJECT_FIT_PODS
    zero = framework.make_pod({})
    assert oracle.fit_filter(node, st, zero) == abi.REJECT_FIT_PODS  # zero-request pods skip resource checks
