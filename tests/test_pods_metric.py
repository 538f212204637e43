"""LoadAware Score with NodeMetric.Status.PodsMetric: the estimation of assigned pods
(load_aware.go:291-335 Score, :337-376 estimatedAssignedPodUsed, helper.go:43-56 report interval / update-time tests,
helper.go:153-186 buildPodMetricMap / sumPodUsages) and the podAssignCache it reads (Reserve / Unreserve at
load_aware.go:260-267, informer add / delete).

An assigned pod is *estimated* (counted as max(EstimatePod, reported usage)) when its usage is not reported, it was
assigned after the metric's UpdateTime, within one report interval before it, or the aggregated score usage is nil;
the estimated pods' reported usage leaves NodeUsage (when NodeUsage covers it).  A ScoreAccordingProdUsage prod pod
sees only prod pods and their reported usages instead of NodeUsage.

Pinned by the reference's two PodsMetric golden cases (load_aware_test.go:1203, :1588 — test_golden_oracle.py) and
here by a second, map-based restatement of the Go flow on random single-node cases; the engine is then checked
bit-exact against the oracle on clusters, across schedule → metric update → Unreserve → schedule sequences."""
import numpy as np
import pytest

from koordinator_amd import Engine, abi, framework as F, synth
from oracle import oracle

GI, MI = 1 << 30, 1 << 20
NOW = 1_800_000_000 * 10**9
S = 10**9


# ---- the reference flow restated with maps (second restatement, independent of oracle.c's term encoding) -------
def py_score(cfg, node, m, pm, assigned, pod, agg):
    """load_aware.go:269-335 for one node; pm rows = POD_METRIC_DTYPE, assigned rows = OR_ASSIGNED_DTYPE;
    agg = None (plain NodeUsage) or "p95" over the longest period (at most one period in these cases)."""
    prod_pod = int(pod["priority_class"][0]) == abi.PRIO_PROD and bool(cfg["la_score_according_prod_usage"][0])
    pod_metrics = {}  # buildPodMetricMap: uid → {resource: usage}
    for r in pm:
        if prod_pod and not r["prod"]:
            continue
        pod_metrics[int(r["uid"])] = {k: int(r["usage"][k]) for k in (0, 1) if (int(r["usage_present"]) >> k) & 1}
    est = oracle.estimate_pod(cfg, pod)
    used = {0: est[0], 1: est[1]}
    upd = int(m["update_time_unix_nano"]) if m["has_update_time"] else -(1 << 63)
    interval = int(m["report_interval_ns"]) or 60 * S
    target = None
    if agg is not None and m["has_node_metric"] and m["agg_count"] > 0 and m["agg_present"][0, abi.AGG_TYPES[agg] - 1]:
        target = {k: int(m["agg_usage"][0, abi.AGG_TYPES[agg] - 1, k]) for k in (0, 1)}
    agg_nil = agg is not None and target is None
    estimated = set()
    for a in assigned:
        if prod_pod and not a["prod"]:
            continue
        usage = pod_metrics.get(int(a["uid"]), {})
        t = int(a["time"])
        if not usage or t > upd or (t < upd and upd - t < interval) or agg_nil:
            for k in (0, 1):
                v = int(a["est"][k])
                if k in usage and usage[k] > v:
                    v = usage[k]
                used[k] += v
            estimated.add(int(a["uid"]))
    pod_usages, est_usages = {0: 0, 1: 0}, {0: 0, 1: 0}
    for uid, usage in pod_metrics.items():
        for k, v in usage.items():
            (est_usages if uid in estimated else pod_usages)[k] += v
    if prod_pod:
        for k in (0, 1):
            used[k] += pod_usages[k]
    elif m["has_node_metric"]:
        node_usage = target if agg is not None else {k: int(m["node_usage"][k]) for k in (0, 1)
                                                     if m["node_usage_present"][k]}
        for k, q in (node_usage or {}).items():
            if est_usages[k] != 0 and q >= est_usages[k]:
                q -= est_usages[k]
            used[k] += q
    w = cfg["la_resource_weights"][0]
    s = sum(oracle.least_requested(used[k], oracle.estimate_node(node, k)) * int(w[k]) for k in (0, 1))
    return s // int(w[0] + w[1])


def _cfg(prod_usage, agg):
    la = F.LoadAwareSchedulingArgs(score_according_prod_usage=prod_usage,
                                   aggregated=None if agg is None else dict(score_type=agg, score_duration_s=0))
    return F.build_config(la=la)


def _random_case(rng):
    node = F.make_node({"cpu": str(int(rng.choice([16, 64, 96]))), "memory": f"{int(rng.choice([64, 256, 512]))}Gi"})
    cpu, mem = int(node["allocatable"][0, abi.RES_CPU]), int(node["allocatable"][0, abi.RES_MEMORY])
    interval = int(rng.choice([0, 30, 60, 300])) * S
    upd = NOW - int(rng.integers(0, 100)) * S
    present = int(rng.integers(1, 4))
    nu = {}
    if present & 1:
        nu["cpu"] = f"{int(rng.integers(0, cpu))}m"
    if present & 2:
        nu["memory"] = str(int(rng.integers(0, mem // MI)) * MI)
    m = F.make_node_metric(present=True, update_time_ns=upd, node_usage=nu if rng.random() < 0.9 else None,
                           report_interval_ns=interval)
    if rng.random() < 0.5:  # one 5m period; p95 present or not
        m["agg_count"] = 1
        m["agg_duration_ns"][0, 0] = 300 * S
        t = abi.AGG_TYPES["p95"] - 1
        m["agg_usage"][0, 0, t] = (int(rng.integers(0, cpu)), int(rng.integers(0, mem // MI)) * MI)
        m["agg_present"][0, 0, t] = 3 if rng.random() < 0.7 else 0
    k = int(rng.integers(0, 7))
    pods = synth.make_pods(max(k, 1), seed=int(rng.integers(1 << 30)))[:k]
    prod = rng.random(k) < 0.5
    pods["priority_class"] = np.where(prod, abi.PRIO_PROD, abi.PRIO_BATCH)
    pods["uid"] = np.arange(1, k + 1)
    eff = interval or 60 * S
    deltas = [-2 * eff, -eff, -eff + 1, -1, 0, 1, 5 * S]
    pods["assign_time_unix_nano"] = [upd + int(rng.choice(deltas)) for _ in range(k)]
    rows = []
    for u in range(1, k + 4):  # the assigned pods (some) and pods the lister knows on other nodes
        if rng.random() < 0.35:
            continue
        r = np.zeros(1, dtype=abi.POD_METRIC_DTYPE)
        r["uid"] = u
        r["usage"] = (int(rng.integers(0, cpu // 2)), int(rng.integers(0, mem // 2 // MI)) * MI)
        r["usage_present"] = int(rng.choice([0, 1, 2, 3, 3, 3]))
        r["prod"] = int(prod[u - 1]) if u <= k else int(rng.random() < 0.5)
        rows.append(r)
    pm = np.concatenate(rows) if rows else np.zeros(0, dtype=abi.POD_METRIC_DTYPE)
    m["pods_metric_count"] = len(pm)
    return node, m, pods, pm


def _assigned_rows(cfg, pods):
    out = np.zeros(len(pods), dtype=oracle.OR_ASSIGNED_DTYPE)
    for k in range(len(pods)):
        out[k]["uid"] = pods[k]["uid"]
        out[k]["time"] = pods[k]["assign_time_unix_nano"]
        out[k]["est"] = oracle.estimate_pod(cfg, pods[k:k + 1])
        out[k]["prod"] = int(pods[k]["priority_class"] == abi.PRIO_PROD)
    return out


def _oracle_one(cfg, node, m, pods, pm, pod):
    st = oracle.states(1)
    if len(pods):
        oracle.add_pods(cfg, st, pods, np.zeros(len(pods), dtype=np.int32))
    if len(pm):
        oracle.set_la_terms(st, 0, oracle.la_node_terms(cfg, m, pm, _assigned_rows(cfg, pods)))
    return oracle.loadaware_score(cfg, node, m, st, pod, NOW)


@pytest.mark.parametrize("prod_usage,agg", [(False, None), (True, None), (False, "p95"), (True, "p95")])
def test_oracle_terms_match_reference_flow(prod_usage, agg):
    cfg = _cfg(prod_usage, agg)
    rng = np.random.default_rng(1000 + 2 * prod_usage + (agg is not None))
    probe = synth.make_pods(8, seed=77)
    probe["priority_class"][::2] = abi.PRIO_PROD
    n_pm = 0
    for _ in range(250):
        node, m, pods, pm = _random_case(rng)
        n_pm += len(pm) > 0
        assigned = _assigned_rows(cfg, pods)
        for j in range(len(probe)):
            pod = probe[j:j + 1]
            want = py_score(cfg, node, m[0], pm, assigned, pod, agg)
            got = _oracle_one(cfg, node, m, pods, pm, pod)
            assert got == want, (j, m, pm, assigned)
    assert n_pm > 150


def test_oracle_pods_metric_changes_scores():
    """The PodsMetric terms move scores relative to the plain NodeUsage path (so the GPU parity below tests them)."""
    cfg = _cfg(False, None)
    rng = np.random.default_rng(7)
    diff = 0
    probe = synth.make_pods(1, seed=3)
    for _ in range(100):
        node, m, pods, pm = _random_case(rng)
        if not len(pm):
            continue
        a = _oracle_one(cfg, node, m, pods, pm, probe)
        m0 = m.copy()
        m0["pods_metric_count"] = 0
        b = _oracle_one(cfg, node, m0, pods, pm[:0], probe)
        diff += a != b
    assert diff > 20


# ---- GPU: the engine against the oracle --------------------------------------------------------------------------
def _pm_cluster(n_nodes, seed, agg=False):
    """make_cluster + uids / assign times on the existing pods + PodsMetric on 60 % of the nodes with a metric."""
    cl = synth.make_cluster(n_nodes, seed=seed)
    rng = np.random.default_rng(seed + 5)
    ex = cl.existing_pods
    ex["uid"] = np.arange(1, len(ex) + 1)
    ex["priority_class"] = np.where(rng.random(len(ex)) < 0.5, abi.PRIO_PROD, ex["priority_class"])
    m = cl.metrics
    upd = m["update_time_unix_nano"]
    m["report_interval_ns"] = rng.choice([0, 30 * S, 60 * S], n_nodes)
    off = rng.choice([-600 * S, -61 * S, -59 * S, -1, 0, 1, 5 * S], len(ex))
    ex["assign_time_unix_nano"] = upd[cl.existing_node] + off
    if agg:
        has = (m["has_node_metric"] != 0) & (rng.random(n_nodes) < 0.7)
        t = abi.AGG_TYPES["p95"] - 1
        m["agg_count"] = np.where(has, 1, 0)
        m["agg_duration_ns"][:, 0] = np.where(has, 300 * S, 0)
        m["agg_usage"][:, 0, t, 0] = (m["node_usage"][:, abi.RES_CPU] * 0.9).astype(np.int64)
        m["agg_usage"][:, 0, t, 1] = m["node_usage"][:, abi.RES_MEMORY]
        m["agg_present"][:, 0, t] = np.where(has, 3, 0)
    pms = {}
    for i in np.nonzero((m["has_node_metric"] != 0) & (rng.random(n_nodes) < 0.6))[0]:
        on = np.nonzero(cl.existing_node == i)[0]
        rows = []
        for j in on:
            if rng.random() < 0.8:
                r = np.zeros(1, dtype=abi.POD_METRIC_DTYPE)
                r["uid"] = ex[j]["uid"]
                r["usage"] = (int(rng.integers(0, 8000)), int(rng.integers(0, 16 * 1024)) * MI)
                r["usage_present"] = int(rng.choice([3, 3, 3, 1, 0]))
                r["prod"] = int(ex[j]["priority_class"] == abi.PRIO_PROD)
                rows.append(r)
        if rows:
            pms[int(i)] = np.concatenate(rows)
            m["pods_metric_count"][i] = len(rows)
    return cl, pms


def _oracle_state(cfg, cl, pms, assigned_pods, assigned_node, metrics):
    st = oracle.states(cl.n)
    oracle.add_pods(cfg, st, assigned_pods, assigned_node)
    for i, pm in pms.items():
        on = np.nonzero(assigned_node == i)[0]
        oracle.set_la_terms(st, i, oracle.la_node_terms(cfg, metrics[i], pm, _assigned_rows(cfg, assigned_pods[on])))
    return st


def _queue(n, seed, uid0):
    pods = synth.make_pods(n, seed=seed)
    rng = np.random.default_rng(seed)
    pods["priority_class"] = np.where(rng.random(n) < 0.4, abi.PRIO_PROD, pods["priority_class"])
    pods["uid"] = np.arange(uid0, uid0 + n)
    return pods


@pytest.mark.gpu
@pytest.mark.parametrize("prod_usage,agg", [(False, None), (True, None), (False, "p95"), (True, "p95")])
def test_gpu_pods_metric_parity(prod_usage, agg):
    cfg = _cfg(prod_usage, agg)
    cl, pms = _pm_cluster(1500, 950 + 2 * prod_usage + (agg is not None), agg=agg is not None)
    pods = _queue(4000, 960, 1 << 40)
    st = _oracle_state(cfg, cl, pms, cl.existing_pods, cl.existing_node, cl.metrics)
    want, want_score = oracle.schedule(cfg, cl.nodes, cl.metrics, st, pods, cl.now_ns, 8)
    with Engine(cfg, cl.n) as e:
        synth.load_into(e, cl)
        for i, pm in pms.items():
            e.set_pods_metric(i, pm)
        got, score, _ = e.schedule(pods)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"first mismatch at pod {bad[:5]}: gpu {got[bad[:5]]} oracle {want[bad[:5]]}"
    np.testing.assert_array_equal(score, want_score)


@pytest.mark.gpu
def test_gpu_pods_metric_sequence():
    """schedule → NodeMetric update (new UpdateTime, PodsMetric now reporting some placed pods) → Unreserve of a
    third of the placed pods → delete of some existing pods → schedule → per-node Score of probe pods."""
    cfg = _cfg(True, None)
    cl, pms = _pm_cluster(800, 970)
    q1, q2 = _queue(1500, 971, 1 << 40), _queue(1500, 972, 1 << 41)
    with Engine(cfg, cl.n) as e:
        synth.load_into(e, cl)
        for i, pm in pms.items():
            e.set_pods_metric(i, pm)
        st = _oracle_state(cfg, cl, pms, cl.existing_pods, cl.existing_node, cl.metrics)
        want1, _ = oracle.schedule(cfg, cl.nodes, cl.metrics, st, q1, cl.now_ns, 8)
        got1, _, _ = e.schedule(q1)
        np.testing.assert_array_equal(got1, want1)
        t_place = cl.now_ns + 1  # Reserve time: the engine clock (newest metric ingest time) + 1 ns
        # new metrics: UpdateTime 30 s after the placements (within 60 s intervals, beyond 30 s ones)
        rng = np.random.default_rng(973)
        m2 = cl.metrics.copy()
        m2["update_time_unix_nano"] = np.where(m2["has_update_time"] != 0, t_place + 30 * S, 0)
        now2 = t_place + 40 * S
        placed = np.nonzero(got1 >= 0)[0]
        pms2 = {}
        for i, pm in pms.items():
            extra = [j for j in placed if got1[j] == i and rng.random() < 0.6]
            rows = [pm]
            for j in extra:
                r = np.zeros(1, dtype=abi.POD_METRIC_DTYPE)
                r["uid"] = q1[j]["uid"]
                r["usage"] = (int(rng.integers(0, 6000)), int(rng.integers(0, 8 * 1024)) * MI)
                r["usage_present"] = 3
                r["prod"] = int(q1[j]["priority_class"] == abi.PRIO_PROD)
                rows.append(r)
            pms2[i] = np.concatenate(rows)
            m2["pods_metric_count"][i] = len(pms2[i])
        e.update_metrics(m2, now2)
        for i, pm in pms2.items():
            e.set_pods_metric(i, pm)
        mask = np.zeros(len(q1), dtype=np.uint8)
        mask[::3] = 1
        e.unreserve(0, len(q1), mask)
        e.remove_pods(cl.existing_pods[:150], cl.existing_node[:150])
        # the oracle's view: existing pods left + placed pods kept, with their assign times
        kept = placed[mask[placed] == 0]
        q1t = q1.copy()
        q1t["assign_time_unix_nano"] = t_place
        a_pods = np.concatenate([cl.existing_pods[150:], q1t[kept]])
        a_node = np.concatenate([cl.existing_node[150:], got1[kept]]).astype(np.int32)
        st2 = _oracle_state(cfg, cl, pms2, a_pods, a_node, m2)
        probe = _queue(12, 974, 1 << 42)
        for k in range(len(probe)):
            _, _, la = e.evaluate(probe[k:k + 1])
            want = [oracle.loadaware_score(cfg, cl.nodes[i:i + 1], m2[i:i + 1], st2[i:i + 1], probe[k:k + 1], now2)
                    for i in range(cl.n)]
            np.testing.assert_array_equal(la, want)
        want2, want2_score = oracle.schedule(cfg, cl.nodes, m2, st2, q2, now2, 8)
        got2, score2, _ = e.schedule(q2)
        bad = np.nonzero(got2 != want2)[0]
        assert bad.size == 0, f"first mismatch at pod {bad[:5]}: gpu {got2[bad[:5]]} oracle {want2[bad[:5]]}"
        np.testing.assert_array_equal(score2, want2_score)


@pytest.mark.gpu
def test_refused_pods_add_leaves_state_unchanged():
    """(r5) kg_pods_add validates every pod — its group fields included — before it changes any state: a
    call refused for a bad group bit leaves the podAssignCache mirror, the node table and the group counters as they
    were, so the retried call gives exactly the state of an engine that only saw the valid call."""
    prof = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.POD_TOPOLOGY_SPREAD),
                     score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.POD_TOPOLOGY_SPREAD: 2})
    cfg = F.build_config(profile=prof)
    cl, pms = _pm_cluster(200, 990)
    pm_nodes = sorted(pms)[:4]
    add = _queue(4, 991, 1 << 42)
    add["match_groups"] = 1
    bad = add.copy()
    bad["match_groups"][3] = 1 << 40  # a group bit beyond the 16 groups: KG_E_INVALID
    idx = np.array(pm_nodes, dtype=np.int32)
    probe = _queue(300, 992, 1 << 43)
    out = []
    for refused_first in (True, False):
        with Engine(cfg, cl.n) as e:
            synth.load_into(e, cl)
            for i, pm in pms.items():
                e.set_pods_metric(i, pm)
            if refused_first:
                with pytest.raises(abi.KoordGPUError):
                    e.add_pods(bad, idx)
            e.add_pods(add, idx)
            st = e.read_state()
            grp = e.read_pod_groups()
            node, score, _ = e.schedule(probe)
            out.append((st, grp, node, score))
    (s1, g1, n1, sc1), (s2, g2, n2, sc2) = out
    for k in s1:
        np.testing.assert_array_equal(s1[k], s2[k], err_msg=k)
    for a, b in zip(g1, g2):
        np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(n1, n2)
    np.testing.assert_array_equal(sc1, sc2)
