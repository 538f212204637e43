"""Upstream default plugins a stock koord-scheduler profile keeps: TaintToleration, NodeAffinity and
NodeResourcesBalancedAllocation on the engine's exact per-pod pass (csrc/defaults_dev.h), the host compiler of
labels / taints / tolerations / node affinity into bitmasks (koordinator_amd/predicates.py) and the oracle
(oracle/defaults.c).

Parity status: the reference runs these plugins from k8s.io/kubernetes v1.24.15 (go.mod:57, 275), which is neither
vendored under /root/reference nor importable here, and the reference's only fixture touching them
(frameworkext/debug_test.go:91-174) holds already-computed per-plugin Scores.  The cases below are hand-derived from
the published v1.24 algorithm and modelled on the upstream tests' scenarios (taint_toleration_test.go
TestTaintTolerationScore, node_affinity_test.go TestNodeAffinityPriority, balanced_allocation_test.go): "parity
unpinned" against the reference itself.  Device vs oracle is bit-exact (placements, weighted totals, node state)."""
import numpy as np
import pytest

from koordinator_amd import Engine, abi, framework as F, synth
from koordinator_amd.predicates import NO_EXECUTE, NO_SCHEDULE, PREFER_NO_SCHEDULE, PredicateTable
from oracle import oracle

E = lambda k, op, v=None: {"key": k, "operator": op, **({"values": v} if v is not None else {})}


def _pod():
    return F.make_pod({"cpu": "1", "memory": "1Gi"})


# ---- host compiler: label operators (labels.Requirement.Matches) ----
@pytest.mark.parametrize("labels,req,want", [
    ({"a": "1"}, E("a", "In", ["1", "2"]), True),
    ({"a": "3"}, E("a", "In", ["1", "2"]), False),
    ({}, E("a", "In", ["1"]), False),
    ({"a": "3"}, E("a", "NotIn", ["1"]), True),
    ({}, E("a", "NotIn", ["1"]), True),  # NotIn holds on an absent key
    ({"a": "1"}, E("a", "NotIn", ["1"]), False),
    ({"a": ""}, E("a", "Exists"), True),
    ({}, E("a", "Exists"), False),
    ({}, E("a", "DoesNotExist"), True),
    ({"a": "x"}, E("a", "DoesNotExist"), False),
    ({"a": "10"}, E("a", "Gt", ["9"]), True),
    ({"a": "9"}, E("a", "Gt", ["9"]), False),
    ({"a": "x"}, E("a", "Gt", ["9"]), False),  # label not an integer
    ({"a": "10"}, E("a", "Gt", ["x"]), False),  # value not an integer: the term never matches
    ({"a": "10"}, E("a", "Gt", ["1", "2"]), False),  # Gt needs exactly one value
    ({}, E("a", "Lt", ["9"]), False),
    ({"a": "-3"}, E("a", "Lt", ["2"]), True),
    ({"a": "1"}, E("a", "Bogus", ["1"]), False),  # unknown operator
    # strconv.ParseInt(s, 10, 64): no underscores, spaces or hex; int64 range
    ({"a": "1_0"}, E("a", "Gt", ["9"]), False),
    ({"a": "10"}, E("a", "Gt", ["0_9"]), False),
    ({"a": " 10"}, E("a", "Gt", ["9"]), False),
    ({"a": "0x10"}, E("a", "Gt", ["9"]), False),
    ({"a": "+10"}, E("a", "Gt", ["9"]), True),
    ({"a": "99999999999999999999"}, E("a", "Gt", ["9"]), False),  # 20 digits: out of int64
    ({"a": "9223372036854775807"}, E("a", "Gt", ["9"]), True),
    ({"a": "-9223372036854775808"}, E("a", "Lt", ["0"]), True),
    ({"a": "-9223372036854775809"}, E("a", "Lt", ["0"]), False),
])
def test_requirement_operators(labels, req, want):
    t = PredicateTable()
    pod = t.fill_pod(_pod(), required_terms=[{"matchExpressions": [req]}])
    got = oracle.default_plugins(t.node_row(labels), pod)["affinity_filter"]
    assert got == want


def test_match_fields_and_empty_terms():
    t = PredicateTable()
    name_in = {"matchFields": [E("metadata.name", "In", ["n1"])]}
    other = {"matchFields": [E("metadata.labels", "In", ["n1"])]}  # only metadata.name is a valid field
    cases = [([name_in], "n1", True), ([name_in], "n2", False), ([other], "n1", False),
             ([], "n1", False),  # required affinity with no terms matches nothing
             ([{}], "n1", False),  # an empty term matches nothing
             ([{}, name_in], "n1", True)]
    for terms, name, want in cases:
        pod = t.fill_pod(_pod(), required_terms=terms)
        assert oracle.default_plugins(t.node_row({}, name=name), pod)["affinity_filter"] == want, (terms, name)
    pod = t.fill_pod(_pod())  # no required affinity: every node
    assert oracle.default_plugins(t.node_row({}), pod)["affinity_filter"]


def test_node_selector():
    t = PredicateTable()
    pod = t.fill_pod(_pod(), node_selector={"disk": "ssd", "zone": "a"})
    assert oracle.default_plugins(t.node_row({"disk": "ssd", "zone": "a", "x": "y"}), pod)["affinity_filter"]
    assert not oracle.default_plugins(t.node_row({"disk": "ssd"}), pod)["affinity_filter"]
    assert not oracle.default_plugins(t.node_row({"disk": "hdd", "zone": "a"}), pod)["affinity_filter"]
    # nodeSelector AND required terms
    pod = t.fill_pod(_pod(), node_selector={"disk": "ssd"},
                     required_terms=[{"matchExpressions": [E("zone", "In", ["b"])]}])
    assert not oracle.default_plugins(t.node_row({"disk": "ssd", "zone": "a"}), pod)["affinity_filter"]
    assert oracle.default_plugins(t.node_row({"disk": "ssd", "zone": "b"}), pod)["affinity_filter"]


# ---- tolerations (Toleration.ToleratesTaint) and TaintToleration Filter ----
@pytest.mark.parametrize("tol,taint,want", [
    ({"key": "k", "operator": "Equal", "value": "v", "effect": NO_SCHEDULE}, ("k", "v", NO_SCHEDULE), True),
    ({"key": "k", "value": "v"}, ("k", "v", NO_EXECUTE), True),  # empty effect: every effect; empty op = Equal
    ({"key": "k", "value": "w"}, ("k", "v", NO_SCHEDULE), False),
    ({"key": "k", "operator": "Exists"}, ("k", "any", NO_SCHEDULE), True),
    ({"operator": "Exists"}, ("other", "x", NO_EXECUTE), True),  # empty key + Exists: every taint
    ({"key": "k", "operator": "Exists", "effect": NO_SCHEDULE}, ("k", "v", PREFER_NO_SCHEDULE), False),
    ({"key": "j", "operator": "Exists"}, ("k", "v", NO_SCHEDULE), False),
    ({"key": "k", "operator": "Bogus"}, ("k", "v", NO_SCHEDULE), False),
])
def test_tolerations(tol, taint, want):
    t = PredicateTable()
    row = t.node_row({}, [{"key": taint[0], "value": taint[1], "effect": taint[2]}])
    pod = t.fill_pod(_pod(), tolerations=[tol])
    d = oracle.default_plugins(row, pod)
    if taint[2] == PREFER_NO_SCHEDULE:  # never blocks; counts when not tolerated
        assert d["taint_filter"] and d["taint_count"] == (0 if want else 1)
    else:
        assert d["taint_filter"] == want and d["taint_count"] == 0


def _normalized(raws, reverse):
    mx = max(raws)
    return [oracle.normalize_default(r, mx, reverse) for r in raws]


def test_taint_score_scenarios():
    """The scenarios of TestTaintTolerationScore (upstream taint_toleration_test.go), derived by hand."""
    T = lambda k, v, e=PREFER_NO_SCHEDULE: {"key": k, "value": v, "effect": e}
    cases = [
        # tolerated vs intolerable PreferNoSchedule taint
        ([{"key": "foo", "operator": "Equal", "value": "bar", "effect": PREFER_NO_SCHEDULE}],
         [[T("foo", "bar")], [T("foo", "blah")]], [100, 0]),
        # all taints tolerated, whatever their number
        ([{"key": "foo", "operator": "Equal", "value": "bar", "effect": PREFER_NO_SCHEDULE},
          {"key": "cpu-type", "operator": "Equal", "value": "arm64", "effect": PREFER_NO_SCHEDULE}],
         [[], [T("cpu-type", "arm64")], [T("foo", "bar"), T("cpu-type", "arm64")]], [100, 100, 100]),
        # the more intolerable taints, the lower the score
        ([{"key": "foo", "operator": "Equal", "value": "bar", "effect": PREFER_NO_SCHEDULE}],
         [[], [T("cpu-type", "arm64")], [T("cpu-type", "arm64"), T("disk-type", "ssd")]], [100, 50, 0]),
        # only PreferNoSchedule taints / tolerations count
        ([{"key": "cpu-type", "operator": "Equal", "value": "arm64", "effect": NO_SCHEDULE},
          {"key": "disk-type", "operator": "Equal", "value": "ssd", "effect": PREFER_NO_SCHEDULE}],
         [[T("cpu-type", "arm64", NO_SCHEDULE)], [T("cpu-type", "arm64")],
          [T("cpu-type", "arm64", NO_SCHEDULE), T("disk-type", "ssd")]], [100, 0, 100]),
        ([], [[], []], [100, 100]),  # no taints, no tolerations
    ]
    for tol, node_taints, want in cases:
        t = PredicateTable()
        rows = [t.node_row({}, ts) for ts in node_taints]
        pod = t.fill_pod(_pod(), tolerations=tol)
        raws = [oracle.default_plugins(r, pod)["taint_count"] for r in rows]
        assert _normalized(raws, True) == want, (tol, node_taints)


def test_node_affinity_score_scenarios():
    """The scenarios of TestNodeAffinityPriority (upstream node_affinity_test.go), derived by hand."""
    l1, l2, l3 = {"foo": "bar"}, {"key": "value"}, {"az": "az1"}
    l4, l5 = {"abc": "az11", "def": "az22"}, {"foo": "bar", "key": "value", "az": "az1"}
    a1 = [(2, {"matchExpressions": [E("foo", "In", ["bar"])]})]
    a2 = [(2, {"matchExpressions": [E("foo", "In", ["bar"])]}), (4, {"matchExpressions": [E("key", "In", ["value"])]}),
          (5, {"matchExpressions": [E("foo", "In", ["bar"]), E("key", "In", ["value"]), E("az", "In", ["az1"])]})]
    a0 = [(0, {"matchExpressions": [E("foo", "In", ["bar"])]})]  # weight 0 is skipped
    cases = [(None, [l1, l2, l3], [0, 0, 0]), (a1, [l4, l2, l3], [0, 0, 0]), (a1, [l1, l2, l3], [100, 0, 0]),
             (a2, [l1, l5, l2], [18, 100, 36]), (a0, [l1, l2], [0, 0])]
    for pref, labels, want in cases:
        t = PredicateTable()
        pod = t.fill_pod(_pod(), preferred=pref)
        raws = [oracle.default_plugins(t.node_row(lb), pod)["affinity_sum"] for lb in labels]
        assert _normalized(raws, False) == want, (pref, labels)


def _go_balanced(alloc, req, pod, resources=3):
    """balancedResourceScorer with Python floats (IEEE binary64, as Go's float64): an independent restatement."""
    f = []
    for r in range(2):
        if resources >> r & 1 and alloc[r] != 0:
            f.append(min(float(req[r] + pod[r]) / float(alloc[r]), 1.0))
    std = abs((f[0] - f[1]) / 2) if len(f) == 2 else 0.0
    return int((1 - std) * 100.0)


@pytest.mark.parametrize("alloc,req,pod,want", [
    ((4000, 10000), (0, 0), (0, 0), 100),          # nothing scheduled, nothing requested
    ((4000, 10000), (0, 0), (3000, 5000), 87),     # 0.75 vs 0.5
    ((6000, 10000), (0, 0), (3000, 5000), 100),    # 0.5 vs 0.5
    ((10000, 20000), (3000, 5000), (3000, 5000), 95),
    ((4000, 10000), (0, 0), (5000, 5000), 75),     # cpu fraction capped at 1
    ((0, 10000), (0, 0), (3000, 9000), 100),       # zero Allocatable: the resource is left out
    ((10000, 20000), (6000, 0), (1000, 2000), 70),
    ((3, 7), (1, 0), (0, 2), None),
])
def test_balanced_allocation(alloc, req, pod, want):
    got = oracle.balanced_score(alloc[0], alloc[1], req[0], req[1], pod[0], pod[1])
    assert got == _go_balanced(alloc, req, pod)
    if want is not None:
        assert got == want
    assert oracle.balanced_score(alloc[0], alloc[1], req[0], req[1], pod[0], pod[1], 1) == 100  # one resource


def test_balanced_random_vs_python_floats():
    rng = np.random.default_rng(7)
    for _ in range(3000):
        alloc = (int(rng.integers(0, 200_000)), int(rng.integers(0, 1 << 40)))
        req = (int(rng.integers(0, 200_000)), int(rng.integers(0, 1 << 40)))
        pod = (int(rng.integers(0, 20_000)), int(rng.integers(0, 1 << 34)))
        assert oracle.balanced_score(*alloc, *req, *pod) == _go_balanced(alloc, req, pod)


def test_debug_table_weighted_sum():
    """frameworkext/debug_test.go:91-174: the framework's total is the sum of the weighted per-plugin Scores
    (v1beta2 weights: PodTopologySpread 2, the rest 1) — the composition rsv_select / the oracle use."""
    rows = {"cn-hangzhou.10.0.4.51": (87, 96, 94, 200, 100, 577), "cn-hangzhou.10.0.4.50": (85, 96, 93, 200, 100, 574),
            "cn-hangzhou.10.0.4.19": (55, 95, 91, 200, 100, 541), "cn-hangzhou.10.0.4.18": (15, 90, 82, 200, 100, 487)}
    for la, bal, fit, spread, taint, total in rows.values():
        assert la + bal + fit + spread + taint == total


def test_profile_config_fields():
    prof = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.TAINT_TOLERATION, F.NODE_AFFINITY),
                     score={F.NODE_RESOURCES_FIT: 1, F.TAINT_TOLERATION: 3, F.NODE_AFFINITY: 2,
                            F.BALANCED_ALLOCATION: 1})
    c = F.build_config(profile=prof)[0]
    assert (c["taint_filter"], c["taint_score"], c["weight_taint"]) == (1, 1, 3)
    assert (c["affinity_filter"], c["affinity_score"], c["weight_affinity"]) == (1, 1, 2)
    assert (c["balanced_score"], c["weight_balanced"], c["balanced_resources"]) == (1, 1, 3)


# ---- device parity (exact pass) ----
STOCK = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.TAINT_TOLERATION, F.NODE_AFFINITY),
                  score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.TAINT_TOLERATION: 1, F.NODE_AFFINITY: 1,
                         F.BALANCED_ALLOCATION: 1})
VARIANTS = {
    "stock": STOCK,
    "filters_only": F.Profile(filter=STOCK.filter, score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1}),
    "scores_only": F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE), score=dict(STOCK.score)),
    "balanced_only": F.Profile(filter=(F.NODE_RESOURCES_FIT,), score={F.BALANCED_ALLOCATION: 3}),
    "v1beta3_weights": F.Profile(filter=STOCK.filter, score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1,
                                                             F.TAINT_TOLERATION: 3, F.NODE_AFFINITY: 2,
                                                             F.BALANCED_ALLOCATION: 1}),
}


def _world(n_nodes, n_pods, seed):
    cluster = synth.make_cluster(n_nodes, seed=seed)
    pods = synth.make_pods(n_pods, seed=seed + 1)
    _, preds = synth.make_predicates(n_nodes, pods, seed=seed + 2)
    return cluster, pods, preds


def _oracle(cfg, cluster, pods, preds, n_threads=8):
    st = oracle.states(cluster.n)
    oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
    node, score, _ = oracle.schedule_resv(cfg, cluster.nodes, cluster.metrics, st, None, pods, cluster.now_ns,
                                          n_threads=n_threads, preds=preds)
    return node, score, st


def test_oracle_stock_profile_effects():
    """The plugins bite: hard taints and required affinity reject nodes, scores move placements."""
    cluster, pods, preds = _world(400, 600, 31)
    base = F.build_config(profile=F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE),
                                            score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1}))
    n0, _, _ = _oracle(base, cluster, pods, preds)
    n1, _, _ = _oracle(F.build_config(profile=STOCK), cluster, pods, preds)
    assert (n1 >= 0).mean() > 0.5 and (n0 != n1).mean() > 0.3
    placed = n1 >= 0
    hard = preds["taints_hard"][n1[placed]] & ~pods["tolerated_taints"][placed]
    assert not hard.any()


@pytest.mark.gpu
@pytest.mark.parametrize("variant", list(VARIANTS))
def test_device_matches_oracle(variant):
    cfg = F.build_config(profile=VARIANTS[variant])
    cluster, pods, preds = _world(3000, 1200, 41)
    want, want_score, st = _oracle(cfg, cluster, pods, preds)
    with Engine(cfg, cluster.n) as e:
        synth.load_into(e, cluster)
        e.upsert_predicates(preds)
        node, score = e.schedule(pods)[:2]
        state = e.read_state()
    assert np.array_equal(node, want) and np.array_equal(score, want_score)
    assert np.array_equal(state["requested_cpu"], st["requested"][:, abi.RES_CPU])
    assert np.array_equal(state["requested_mem"], st["requested"][:, abi.RES_MEMORY])


@pytest.mark.gpu
def test_single_pod_calls_and_predicate_updates():
    """One pod per call, and node rows replaced mid-queue (a node gains a taint, labels change)."""
    cfg = F.build_config(profile=STOCK)
    cluster, pods, preds = _world(900, 300, 51)
    rng = np.random.default_rng(52)
    later = preds.copy()
    sel = rng.choice(cluster.n, 200, replace=False)
    later["taints_hard"][sel] |= 1
    later["predicates"][sel] = rng.permutation(later["predicates"])[:200]
    st = oracle.states(cluster.n)
    oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
    w1 = oracle.schedule_resv(cfg, cluster.nodes, cluster.metrics, st, None, pods[:150], cluster.now_ns, n_threads=8,
                              preds=preds)
    w2 = oracle.schedule_resv(cfg, cluster.nodes, cluster.metrics, st, None, pods[150:], cluster.now_ns, n_threads=8,
                              preds=later)
    with Engine(cfg, cluster.n) as e:
        synth.load_into(e, cluster)
        e.upsert_predicates(preds)
        e.stage(pods)
        for j in range(150):
            e.schedule_staged(j, 1)
        e.upsert_predicates(later[sel], sel.astype(np.int32))
        for j in range(150, len(pods)):
            e.schedule_staged(j, 1)
        node, score = e.fetch(0, len(pods))
    assert np.array_equal(node, np.concatenate([w1[0], w2[0]]))
    assert np.array_equal(score, np.concatenate([w1[1], w2[1]]))


@pytest.mark.gpu
def test_table_growth_refused_until_recompiled():
    """ABI 11: the caller's taint / predicate tables only grow, and a row compiled before an id existed
    leaves it undecided.  A node row carrying a taint the staged pods' tolerations were not compiled against, or a
    staged pod using a predicate the node rows were not compiled against, makes the schedule call fail loudly until
    the pods are re-staged / the rows re-sent; a tolerate-all pod (no key, Exists, no effect) holds for any taint."""
    cfg = F.build_config(profile=STOCK)
    cluster = synth.make_cluster(500, seed=61)
    pods = synth.make_pods(200, seed=62)
    table, preds = synth.make_predicates(500, pods, seed=63)
    assert ((pods["flags"] & abi.POD_TAINT_TABLE) != 0).any()
    assert (pods["tolerated_taints"] == np.uint64((1 << 64) - 1)).any()  # tolerate-all pods, no table flag
    with Engine(cfg, cluster.n) as e:
        synth.load_into(e, cluster)
        e.upsert_predicates(preds)
        e.stage(pods)
        e.schedule_staged(0, 50)
        t_new = table.taint_id("fresh", "x", NO_SCHEDULE)  # a node gains a taint the pods were not compiled against
        row = preds[7:8].copy()
        row["taints_hard"] |= np.uint64(1 << t_new)
        e.upsert_predicates(row, np.array([7], dtype=np.int32))
        with pytest.raises(abi.KoordGPUError, match="re-stage"):
            e.schedule_staged(50, 10)
        pods2 = pods.copy()  # re-compiled: no toleration of these pods names "fresh"
        dep = (pods2["flags"] & abi.POD_TAINT_TABLE) != 0
        pods2["taint_count"][dep] = len(table.taints)
        e.stage(pods2)
        e.schedule_staged(50, 10)
        extra = pods2[60:61].copy()  # a pod interns a predicate the node rows were not compiled against
        table.fill_pod(extra, node_selector={"fresh-label": "y"})
        e.stage(np.concatenate([pods2[:60], extra]))
        with pytest.raises(abi.KoordGPUError, match="re-send the node rows"):
            e.schedule_staged(60, 1)
        rows2 = preds.copy()  # no node has the label: recompiled rows decide the predicate as not holding
        rows2["taints_hard"][7] = row["taints_hard"][0]
        rows2["predicate_count"] = len(table.preds)
        e.upsert_predicates(rows2)
        node, _, _ = e.schedule(extra)
        assert node[0] == -1


@pytest.mark.gpu
def test_shipped_profile_with_stock_defaults():
    """The shipped koord profile plus the upstream defaults a v1beta2 profile keeps (weights 1)."""
    import test_shipped_profile as S
    prof = F.Profile(filter=S.PROFILE.filter + (F.TAINT_TOLERATION, F.NODE_AFFINITY),
                     score=dict(S.PROFILE.score, **{F.TAINT_TOLERATION: 1, F.NODE_AFFINITY: 1,
                                                    F.BALANCED_ALLOCATION: 1}))
    cfg = S.config(profile=prof)
    cluster, numa, dev, rsv, pods, quotas = S.workload(1500, 900, 61)
    _, preds = synth.make_predicates(cluster.n, pods, seed=63)
    st = oracle.states(cluster.n)
    oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
    buf, r, d, q = oracle.numa_states(numa), rsv.copy(), dev.copy(), quotas.copy()
    want = oracle.schedule_resv(cfg, cluster.nodes, cluster.metrics, st, r, pods, cluster.now_ns, devices=d,
                                quotas=q, n_threads=8, with_minors=True, numa_buf=buf, with_numa=True, preds=preds)
    with Engine(cfg, cluster.n) as e:
        synth.load_shipped_into(e, cluster, numa, dev, rsv, quotas)
        e.upsert_predicates(preds)
        node, score = e.schedule(pods)[:2]
        slot = e.fetch_reservations(0, len(pods))
        minors = e.fetch_devices(0, len(pods))
        cpus = e.fetch_cpusets(0, len(pods))
    assert np.array_equal(node, want[0]) and np.array_equal(score, want[1])
    assert np.array_equal(slot, want[2]) and np.array_equal(minors, want[3]) and np.array_equal(cpus, want[4])
    assert (node >= 0).mean() > 0.4


# ---- ImageLocality (ABI 10): image_locality.go restated; cases hand-derived from the published v1.24 formula ----
MIB = 1024 * 1024


def _go_image_priority(sum_scores, n_containers):
    """calculatePriority with Go int64 semantics (operands non-negative here, so // is Go's truncation)."""
    lo, hi = 23 * MIB, 1000 * MIB * n_containers
    s = lo if sum_scores < lo else (hi if sum_scores > hi else sum_scores)
    return 100 * (s - lo) // (hi - lo) if hi != lo else 0


def test_normalized_image_name():
    from koordinator_amd.predicates import normalized_image_name as nn
    assert nn("nginx") == "nginx:latest"
    assert nn("nginx:1.2") == "nginx:1.2"
    assert nn("host:5000/nginx") == "host:5000/nginx:latest"  # a registry port is not a tag
    assert nn("host:5000/nginx:1.2") == "host:5000/nginx:1.2"


@pytest.mark.parametrize("node_images,containers,want", [
    # one container, its 300 MiB image on one of two nodes: spread 0.5 → 150 MiB → 100·127/977 = 12 on node 0
    ([[(["img/a:v1"], 300 * MIB)], []], ["img/a:v1"], [12, 0]),
    # below minThreshold (23 MiB) scores 0 even where the image is present
    ([[(["img/a:v1"], 40 * MIB)], []], ["img/a:v1"], [0, 0]),
    # a 2 GiB image on both nodes: clamped to maxThreshold → 100
    ([[(["img/b:v1"], 2048 * MIB)], [(["img/b:v1"], 2048 * MIB)]], ["img/b:v1"], [100, 100]),
    # two containers: maxThreshold doubles; the same image twice counts twice
    ([[(["img/b:v1"], 1000 * MIB)], [(["img/b:v1"], 1000 * MIB)]], ["img/b:v1", "img/b:v1"], [100, 100]),
    ([[(["img/b:v1"], 1000 * MIB)], [(["img/c:v1"], 500 * MIB)]], ["img/b:v1", "img/c:v1"],
     [_go_image_priority(500 * MIB, 2), _go_image_priority(250 * MIB, 2)]),
    # an untagged container image resolves to ':latest', which a node lists under a second name
    ([[(["img/d:v2", "img/d:latest"], 600 * MIB)], []], ["img/d"], [_go_image_priority(300 * MIB, 1), 0]),
    # no node holds the image
    ([[(["img/a:v1"], 300 * MIB)], []], ["img/zzz:v1"], [0, 0]),
])
def test_image_locality_cases(node_images, containers, want):
    from koordinator_amd.predicates import ImageTable
    t = ImageTable(node_images)
    pod = t.fill_pod(_pod(), containers)
    rows = np.zeros(len(node_images), dtype=abi.NODE_PRED_DTYPE)
    rows["images"] = [t.node_mask(i) for i in range(len(node_images))]
    rows["image_count"] = t.image_count()
    got = [oracle.default_plugins(rows[i], pod)["image_score"] for i in range(len(node_images))]
    assert got == want


def test_image_locality_random_vs_python():
    """The oracle's restatement against an independent Python one over the synthetic image world."""
    cluster = synth.make_cluster(300, seed=71)
    pods = synth.make_pods(400, seed=72)
    preds = np.zeros(cluster.n, dtype=abi.NODE_PRED_DTYPE)
    table = synth.make_images(cluster.n, pods, preds, seed=73)
    for j in range(0, len(pods), 7):
        for i in range(0, cluster.n, 11):
            s = 0
            for c in range(int(pods[j]["n_containers"])):
                b = int(pods[j]["container_image_bit"][c])
                if b >= 0 and (int(preds[i]["images"]) >> b) & 1:
                    s += int(pods[j]["container_image_score"][c])
            want = _go_image_priority(s, int(pods[j]["n_containers"]))
            assert oracle.default_plugins(preds[i], pods[j])["image_score"] == want
    assert len(table.bits) > 20


IMAGE_PROFILE = F.Profile(filter=STOCK.filter, score=dict(STOCK.score, **{F.IMAGE_LOCALITY: 1}))


def test_oracle_image_locality_moves_placements():
    cluster, pods, preds = _world(400, 600, 81)
    synth.make_images(cluster.n, pods, preds, seed=82)
    n0, _, _ = _oracle(F.build_config(profile=STOCK), cluster, pods, preds)
    n1, _, _ = _oracle(F.build_config(profile=IMAGE_PROFILE), cluster, pods, preds)
    assert (n0 != n1).mean() > 0.1


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["stock_plus_image", "image_only"])
def test_device_image_locality_matches_oracle(variant):
    prof = IMAGE_PROFILE if variant == "stock_plus_image" else F.Profile(
        filter=(F.NODE_RESOURCES_FIT,), score={F.NODE_RESOURCES_FIT: 1, F.IMAGE_LOCALITY: 2})
    cfg = F.build_config(profile=prof)
    cluster, pods, preds = _world(2500, 900, 91)
    synth.make_images(cluster.n, pods, preds, seed=92)
    want, want_score, _ = _oracle(cfg, cluster, pods, preds)
    with Engine(cfg, cluster.n) as e:
        synth.load_into(e, cluster)
        e.upsert_predicates(preds)
        node, score = e.schedule(pods)[:2]
    assert np.array_equal(node, want) and np.array_equal(score, want_score)
    assert (node >= 0).mean() > 0.5


def test_image_table_counts_are_cluster_wide_known_deviation():
    """ADVICE r3, a documented deviation: k8s v1.24's cache.addNodeImageStates copies len(state.nodes)
    into a node's ImageStateSummary when that node is added or updated, so a node added before a second holder of the
    same image keeps NumNodes = 1 until its own next update.  ImageTable — and the device, which takes one scaled score
    per container — uses the cluster-wide count on every node.  The two agree once every holder has been re-added
    after the last one arrived (an informer resync).  Parity unpinned: upstream is not vendored."""
    from koordinator_amd.predicates import ImageTable
    size = 600 * MIB
    t = ImageTable([[(["img/a:v1"], size)], [(["img/a:v1"], size)], []])  # nodes 0 and 1 hold the image, 3 nodes
    pod = t.fill_pod(_pod(), ["img/a:v1"])
    assert int(pod["container_image_score"][0][0]) == int(float(size) * (2.0 / 3.0))  # NumNodes = 2 on both
    rows = np.zeros(3, dtype=abi.NODE_PRED_DTYPE)
    rows["images"] = [t.node_mask(i) for i in range(3)]
    rows["image_count"] = t.image_count()
    got = [oracle.default_plugins(rows[i], pod)["image_score"] for i in range(3)]
    assert got[0] == got[1] and got[2] == 0

    def calc(scaled):  # calculatePriority(sumImageScores, 1 container): clamp to [23 MiB, 1000 MiB], scale to 0..100
        s = min(max(scaled, 23 * MIB), 1000 * MIB)
        return 100 * (s - 23 * MIB) // (1000 * MIB - 23 * MIB)
    upstream_v124 = [calc(int(float(size) * (1.0 / 3.0))), calc(int(float(size) * (2.0 / 3.0))), 0]  # node 0 added first
    assert got[1] == upstream_v124[1] and got[0] != upstream_v124[0]  # the deviation, on the earlier-added holder only
