"""(ABI 12) PodTopologySpread and InterPodAffinity with topologyKey kubernetes.io/hostname or topology.kubernetes.io/zone
on the exact per-pod pass.

The reference runs both from k8s.io/kubernetes v1.24.15 (not vendored): the oracle restates the published plugins
(oracle/defaults.c) and is pinned by hand-derived cases below ("parity unpinned" against the reference beyond them;
the only reference-held anchor is frameworkext/debug_test.go:91-174, where PodTopologySpread contributes 200 = weight 2
× MaxNodeScore to every node of a pod without soft constraints — test_spread_score_without_constraint_is_max).
Bar for the device: bit-exact placements, totals and the final per-node group counters against the oracle."""
import math

import numpy as np
import pytest

from koordinator_amd import Engine, abi, framework as F, synth
from koordinator_amd.predicates import PodGroupTable
from oracle import oracle

SPREAD_ONLY = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.POD_TOPOLOGY_SPREAD),
                        score={F.NODE_RESOURCES_FIT: 1, F.POD_TOPOLOGY_SPREAD: 2})
IPA_ONLY = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.INTER_POD_AFFINITY),
                     score={F.NODE_RESOURCES_FIT: 1, F.INTER_POD_AFFINITY: 1})
STOCK = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.TAINT_TOLERATION, F.NODE_AFFINITY,
                          F.POD_TOPOLOGY_SPREAD, F.INTER_POD_AFFINITY),
                  score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.TAINT_TOLERATION: 1, F.NODE_AFFINITY: 1,
                         F.BALANCED_ALLOCATION: 1, F.POD_TOPOLOGY_SPREAD: 2, F.INTER_POD_AFFINITY: 1})


def _grp(**kw):
    g = np.zeros(1, dtype=oracle.GROUP_DTYPE)
    for k, v in kw.items():
        g[k][0, :len(v)] = v
    return g


def _gpod(**kw):
    p = np.zeros(1, dtype=abi.POD_DTYPE)
    for k, v in kw.items():
        p[k] = v
    return p


# ---- hand-derived cases of the restated plugins ----------------------------------------------------------------
def _spread_pod(*cons, match=1):
    """cons: (group, maxSkew, flags) in the pod's order."""
    p = _gpod(match_groups=match, n_spread=len(cons))
    for c, (g, k, f) in enumerate(cons):
        p["spread_group"][0, c], p["spread_max_skew"][0, c], p["spread_flags"][0, c] = g, k, f
    return p


def test_spread_score_cases():
    """scoring.go: one hostname constraint, counts [0, 1, 3] over 3 filtered nodes, maxSkew 1: weight log(5) → raw
    [0, 1, 4], normalized 100 · (4 + 0 − s) / 4 = [100, 75, 0]; two constraints sum in the pod's order, each
    float64(cnt)·w + float64(maxSkew − 1), truncated once."""
    L = oracle.lib()
    pod = _spread_pod((1, 1, 0))
    w = np.array([math.log(5), 0, 0, 0])
    raw = [L.or_spread_raw(oracle.p(np.array([c, 0, 0, 0], dtype=np.int64)), oracle.p(w), oracle.p(pod))
           for c in (0, 1, 3)]
    assert raw == [0, int(1 * math.log(5)), int(3 * math.log(5))] == [0, 1, 4]
    assert [L.or_spread_normalize(r, 0, 4) for r in raw] == [100, 75, 0]
    two = _spread_pod((1, 3, abi.SPREAD_ZONE), (1, 1, 0), (2, 1, abi.SPREAD_HARD))  # the hard one does not score
    w2 = np.array([math.log(4 + 2), math.log(10 + 2), 0, 0])
    got = L.or_spread_raw(oracle.p(np.array([7, 2, 9, 0], dtype=np.int64)), oracle.p(w2), oracle.p(two))
    assert got == int((7 * math.log(6) + 2) + (2 * math.log(12) + 0))


def test_spread_score_without_constraint_is_max():
    """A pod without a ScheduleAnyway constraint: Score 0 everywhere, NormalizeScore gives MaxNodeScore (the 200 of
    debug_test.go:140-144 = weight 2 × 100)."""
    L = oracle.lib()
    pod = _spread_pod((1, 1, abi.SPREAD_HARD))
    assert L.or_spread_raw(oracle.p(np.array([7, 0, 0, 0], dtype=np.int64)), oracle.p(np.ones(4)), oracle.p(pod)) == 0
    assert 2 * L.or_spread_normalize(0, 0, 0) == 200


def test_spread_node_keys():
    """nodeLabelsMatchSpreadConstraints: a zone-keyed constraint needs the node's zone label (per kind)."""
    L = oracle.lib()
    pod = _spread_pod((1, 1, abi.SPREAD_HARD | abi.SPREAD_ZONE), (1, 1, 0))
    zoned, bare = np.zeros(1, dtype=abi.NODE_PRED_DTYPE), np.zeros(1, dtype=abi.NODE_PRED_DTYPE)
    zoned["zone"] = 2
    assert L.or_spread_has_keys(oracle.p(zoned), oracle.p(pod), 1) == 1
    assert L.or_spread_has_keys(oracle.p(bare), oracle.p(pod), 1) == 0
    assert L.or_spread_has_keys(oracle.p(bare), oracle.p(pod), 0) == 1  # the ScheduleAnyway one is hostname-keyed


def _zones(**kw):
    z = np.zeros(1, dtype=oracle.IPA_ZONES_DTYPE)
    for k, v in kw.items():
        if k == "entries":
            z[k] = v
        else:
            z[k][0, :len(v)] = v
    return z


def test_interpod_filter_cases():
    L = oracle.lib()
    none = _zones()
    f = lambda g, pod, zone=0, z=none: L.or_interpod_filter(oracle.p(g), oracle.p(pod), zone, oracle.p(z))
    # required anti-affinity to group 0: a node holding a matching pod rejects
    anti = _gpod(pod_anti_affinity=1)
    assert f(_grp(cnt=[1]), anti) == 0
    assert f(_grp(cnt=[0]), anti) == 1
    # an existing pod's anti-affinity term of a group the incoming pod matches
    mine = _gpod(match_groups=2)
    assert f(_grp(anti=[0, 1]), mine) == 0
    assert f(_grp(anti=[1, 0]), mine) == 1
    # required affinity to group 2: needs a matching pod on the node; the first pod of a series (affinityCounts
    # empty and the pod matches its own terms) passes anywhere
    aff = _gpod(pod_affinity_group=3, pod_affinity_terms=4, match_groups=4)
    assert f(_grp(cnt=[0, 0, 1]), aff) == 1
    assert f(_grp(), aff) == 1  # first of a series
    assert f(_grp(), aff, 0, _zones(entries=1)) == 0
    stranger = _gpod(pod_affinity_group=3, pod_affinity_terms=4, match_groups=0)  # does not match its own terms
    assert f(_grp(), stranger) == 0


def test_interpod_zone_filter_cases():
    """Zone-keyed terms: satisfyPodAffinity needs the node's zone label (even for the first pod of a series) and its
    zone pair's count; anti-affinity pairs reject every node of the zone; a node without the label has no pair."""
    L = oracle.lib()
    f = lambda g, pod, zone, z: L.or_interpod_filter(oracle.p(g), oracle.p(pod), zone, oracle.p(z))
    aff = _gpod(pod_affinity_group=1, pod_affinity_terms_zone=1, match_groups=1)
    assert f(_grp(), aff, 2, _zones(aff=[0, 3], entries=1)) == 1  # zone 2 holds 3 matching pods
    assert f(_grp(), aff, 1, _zones(aff=[0, 3], entries=1)) == 0
    assert f(_grp(), aff, 1, _zones()) == 1  # first of a series, in a labelled zone
    assert f(_grp(), aff, 0, _zones()) == 0  # "All topology labels must exist on the node"
    both = _gpod(pod_affinity_group=1, pod_affinity_terms=1, pod_affinity_terms_zone=1, match_groups=1)
    assert f(_grp(cnt=[1]), both, 1, _zones(aff=[1], entries=1)) == 1
    assert f(_grp(cnt=[0]), both, 1, _zones(aff=[1], entries=1)) == 0  # the hostname pair is empty
    anti = _gpod(pod_anti_affinity_zone=2)
    assert f(_grp(), anti, 1, _zones(anti_in=[1])) == 0
    assert f(_grp(), anti, 2, _zones(anti_in=[1])) == 1
    assert f(_grp(), anti, 0, _zones(anti_in=[1])) == 1
    assert f(_grp(), _gpod(match_groups=1), 3, _zones(anti_ex=[0, 0, 2])) == 0


def test_interpod_zone_maps():
    """or_ipa_zones_add: the zone pairs sum the nodes' counters; affinityCounts' emptiness sees hostname pairs on any
    node and zone pairs only on labelled nodes."""
    L = oracle.lib()
    pod = _gpod(pod_affinity_group=1, pod_affinity_terms_zone=1, pod_anti_affinity_zone=2, match_groups=0b100,
                n_pod_preferred=2, pod_preferred_group=[1, 2, 0, 0], pod_preferred_weight=[10, -5, 0, 0],
                pod_preferred_zone=0b10)
    z = _zones()
    for g, zone in ((_grp(cnt=[1, 2, 0], anti_z=[0, 0, 1], symw_z=[0, 0, 4]), 1), (_grp(cnt=[0, 1]), 1),
                    (_grp(cnt=[5, 5], anti_z=[0, 0, 9]), 0)):
        L.or_ipa_zones_add(oracle.p(z), oracle.p(g), zone, oracle.p(pod))
    assert z["aff"][0, 0] == 1 and z["anti_in"][0, 0] == 3 and z["anti_ex"][0, 0] == 1
    assert z["score"][0, 0] == -5 * 3 + 4 and z["entries"][0] == 1  # only the zone-keyed preferred term
    z0 = _zones()
    L.or_ipa_zones_add(oracle.p(z0), oracle.p(_grp(cnt=[5])), 0, oracle.p(pod))
    assert z0["entries"][0] == 0  # an unlabelled node makes no zone pair
    raw = L.or_interpod_raw(oracle.p(_grp(cnt=[2, 7])), oracle.p(pod), 1, oracle.p(z))
    assert raw == 10 * 2 + (-5 * 3 + 4)  # hostname term on the node + the zone pair


def test_interpod_score_cases():
    """processExistingPod summed on one node: the pod's preferred affinity (+10 × 2 matching pods) and anti-affinity
    (−5 × 1), plus the node's pods' terms matching the pod (symmetric weights 7); min-max normalisation in float64."""
    L = oracle.lib()
    pod = _gpod(match_groups=0b100, n_pod_preferred=2, pod_preferred_group=[1, 2, 0, 0],
                pod_preferred_weight=[10, -5, 0, 0])
    g = _grp(cnt=[2, 1, 0], symw=[100, 100, 7])
    assert L.or_interpod_raw(oracle.p(g), oracle.p(pod), 0, oracle.p(_zones())) == 20 - 5 + 7
    assert [L.or_interpod_normalize(r, -5, 10) for r in (-5, 0, 10)] == [0, int(100.0 * (5 / 15)), 100]
    assert L.or_interpod_normalize(3, 3, 3) == 0


def test_groups_apply_counts_terms():
    g = np.zeros(1, dtype=oracle.GROUP_DTYPE)
    pod = _gpod(match_groups=0b11, pod_anti_affinity=0b100, pod_affinity_terms=0b1000, n_pod_preferred=1,
                pod_preferred_group=[2, 0, 0, 0], pod_preferred_weight=[-30, 0, 0, 0])
    oracle.groups_apply(g, 0, pod, 1, hard_weight=5)
    assert list(g["cnt"][0, :4]) == [1, 1, 0, 0] and list(g["anti"][0, :4]) == [0, 0, 1, 0]
    assert list(g["symw"][0, :4]) == [0, -30, 0, 5]
    oracle.groups_apply(g, 0, pod, -1, hard_weight=5)
    assert not g["cnt"].any() and not g["anti"].any() and not g["symw"].any()
    zp = _gpod(match_groups=1, pod_anti_affinity_zone=0b10, pod_affinity_terms_zone=0b100, n_pod_preferred=2,
               pod_preferred_group=[4, 4, 0, 0], pod_preferred_weight=[3, -2, 0, 0], pod_preferred_zone=0b10)
    oracle.groups_apply(g, 0, zp, 1, hard_weight=5)
    assert list(g["anti_z"][0, :4]) == [0, 1, 0, 0] and list(g["anti"][0, :4]) == [0, 0, 0, 0]
    assert list(g["symw_z"][0, :4]) == [0, 0, 5, -2] and list(g["symw"][0, :4]) == [0, 0, 0, 3]


# ---- composed scheduling on the oracle: the plugins' visible effects ---------------------------------------------
def _flat(n, cpu="64", mem="256Gi"):
    nodes = np.concatenate([F.make_node({"cpu": cpu, "memory": mem}) for _ in range(n)])
    metrics = np.concatenate([F.make_node_metric(present=False, node_usage=None) for _ in range(n)])
    return synth.Cluster(nodes, metrics, np.zeros(0, dtype=abi.POD_DTYPE), np.zeros(0, dtype=np.int32), 10**18)


def _run_oracle(cfg, cluster, pods, preds=None, n_threads=4):
    st = oracle.states(cluster.n)
    oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
    g = oracle.groups_init(cluster.n, cluster.existing_pods, cluster.existing_node,
                           int(cfg["hard_pod_affinity_weight"][0]))
    node, score, _ = oracle.schedule_resv(cfg, cluster.nodes, cluster.metrics, st, None, pods, cluster.now_ns,
                                          n_threads=n_threads, preds=preds, groups=g)
    return node, score, st, g


def _replicas(n, table, **kw):
    pods = np.concatenate([F.make_pod(requests={"cpu": "1", "memory": "1Gi"}) for _ in range(n)])
    for j in range(n):
        table.fill_pod(pods[j:j + 1], {"app": "web"}, "default", **kw)
    return pods


def _zoned(n, zones):
    cl = _flat(n)
    preds = np.zeros(n, dtype=abi.NODE_PRED_DTYPE)
    preds["zone"] = zones
    return cl, preds


def test_oracle_zone_spread_round_robin():
    """maxSkew 1 over zones: 6 nodes in zones [1, 1, 2, 2, 3, 3] — each pod lands in an emptiest zone (lowest node
    first); a node without the zone label is never chosen."""
    t = PodGroupTable()
    sel = {"matchLabels": {"app": "web"}}
    pods = _replicas(6, t, spread=[{"maxSkew": 1, "labelSelector": sel, "topologyKey": "topology.kubernetes.io/zone"}])
    cl, preds = _zoned(7, [0, 1, 1, 2, 2, 3, 3])
    node, _, _, g = _run_oracle(F.build_config(profile=SPREAD_ONLY), cl, pods, preds)
    assert list(node) == [1, 3, 5, 1, 3, 5] or sorted(node[:3]) == [1, 3, 5]
    assert 0 not in node
    zone_of = np.array([0, 1, 1, 2, 2, 3, 3])
    assert sorted(np.bincount(zone_of[node], minlength=4)[1:]) == [2, 2, 2]


def test_oracle_system_default_constraints_ignore_no_node():
    """(ABI 13) requireAllTopologies = len(pod.Spec.TopologySpreadConstraints) > 0 || !systemDefaulted
    (podtopologyspread PreScore, k8s v1.24.15).  Three equal nodes in zones [1, 2, none] holding 2 / 0 / 1 pods of the
    app; a pod of the app with the system defaults (hostname maxSkew 3 + zone maxSkew 5, ScheduleAnyway).  Hand-derived:
    * system-defaulted: no node ignored; hostname weight log(3 + 2), zone weight log(#{zone 1, zone 2, ""} + 2) =
      log 5; the zone sums count only nodes carrying the key (zone 1: 2, zone 2: 0); raw node 0 = int(2w+2 + 2w+4) = 12,
      node 1 = int(2 + 4) = 6, node 2 (no zone label: hostname term only) = int(w + 2) = 3; normalized 100·(15 − s)/12
      = [25, 75, 100]; Fit 99 everywhere (1m / 1Mi pods) → totals 99 + 2·[25, 75, 100]: node 2 wins with 299;
    * the same constraints given by the pod itself: node 2 is ignored (0), weights log(2 + 2), raw [11, 6] →
      normalized [54, 100] → node 1 wins with 299."""
    t = PodGroupTable()
    sel = {"matchLabels": {"app": "web"}}
    t.group(sel, ("default",))  # the group exists before the existing pods' match bits are compiled
    cl, preds = _zoned(3, [1, 2, 0])

    def tiny(n, **kw):
        pods = np.concatenate([F.make_pod(requests={"cpu": "1m", "memory": "1Mi"}) for _ in range(n)])
        for j in range(n):
            t.fill_pod(pods[j:j + 1], {"app": "web"}, "default", **kw)
        return pods

    cl = synth.Cluster(cl.nodes, cl.metrics, tiny(3), np.array([0, 0, 2], dtype=np.int32), cl.now_ns)
    sysdef = tiny(1, system_default_selector=sel)
    assert (sysdef["spread_flags"][0, :2] & abi.SPREAD_SYSTEM_DEFAULT).all()
    own = sysdef.copy()
    own["spread_flags"] &= ~abi.SPREAD_SYSTEM_DEFAULT
    cfg = F.build_config(profile=SPREAD_ONLY)
    node, score, _, _ = _run_oracle(cfg, cl, sysdef, preds)
    assert (int(node[0]), int(score[0])) == (2, 299)
    node, score, _, _ = _run_oracle(cfg, cl, own, preds)
    assert (int(node[0]), int(score[0])) == (1, 299)


def test_system_default_without_owners_adds_no_constraints():
    """ buildDefaultConstraints returns nil when DefaultSelector is empty (a pod without owners): the
    system defaults add no constraint, so the pod is not spread against every pod of the namespace."""
    t = PodGroupTable()
    for sel in ({}, {"matchLabels": {}}, {"matchLabels": {}, "matchExpressions": []}):
        pod = F.make_pod(requests={"cpu": "1m", "memory": "1Mi"})
        t.fill_pod(pod, {"app": "web"}, "default", system_default_selector=sel)
        assert int(pod["n_spread"][0]) == 0 and not pod["spread_flags"].any()
    pod = F.make_pod(requests={"cpu": "1m", "memory": "1Mi"})
    t.fill_pod(pod, {"app": "web"}, "default", system_default_selector={"matchLabels": {"app": "web"}})
    assert int(pod["n_spread"][0]) == 2
    cl, preds = _zoned(3, [1, 2, 0])
    node, _, _, _ = _run_oracle(F.build_config(profile=SPREAD_ONLY), cl, F.make_pod(requests={"cpu": "1m"}), preds)
    assert node[0] == 0  # no constraint: the equal nodes tie, lowest index


def test_oracle_hard_spread_round_robin():
    """maxSkew 1 on four equal nodes: each pod lands on an emptiest node, lowest index first."""
    t = PodGroupTable()
    sel = {"matchLabels": {"app": "web"}}
    pods = _replicas(8, t, spread=[{"maxSkew": 1, "labelSelector": sel}])
    node, _, _, g = _run_oracle(F.build_config(profile=SPREAD_ONLY), _flat(4), pods)
    assert list(node) == [0, 1, 2, 3, 0, 1, 2, 3]
    assert list(g["cnt"][:4, 0]) == [2, 2, 2, 2]


def test_oracle_anti_affinity_one_per_node():
    t = PodGroupTable()
    sel = {"matchLabels": {"app": "web"}}
    pods = _replicas(5, t, required_anti_affinity=[{"labelSelector": sel}])
    node, _, _, _ = _run_oracle(F.build_config(profile=IPA_ONLY), _flat(3), pods)
    assert sorted(node[:3]) == [0, 1, 2] and list(node[3:]) == [-1, -1]


def test_oracle_affinity_follows_the_first_pod():
    """The first pod of a series passes anywhere (no pod matches, it matches its own term); the rest must share a
    node with a matching pod, and the preferred weight of the symmetric term keeps them together."""
    t = PodGroupTable()
    sel = {"matchLabels": {"app": "web"}}
    pods = _replicas(4, t, required_affinity=[{"labelSelector": sel}])
    node, _, _, _ = _run_oracle(F.build_config(profile=IPA_ONLY), _flat(6), pods)
    assert (node == node[0]).all() and node[0] >= 0


def test_oracle_preferred_anti_affinity_spreads():
    t = PodGroupTable()
    sel = {"matchLabels": {"app": "web"}}
    pods = _replicas(3, t, preferred_anti_affinity=[{"weight": 100, "podAffinityTerm": {"labelSelector": sel}}])
    node, _, _, _ = _run_oracle(F.build_config(profile=IPA_ONLY), _flat(3), pods)
    assert sorted(node) == [0, 1, 2]


ZONE = "topology.kubernetes.io/zone"
WEB = {"matchLabels": {"app": "web"}}
ZONE_WORLDS = {  # (nodes' zones, replicas, PodGroupTable.fill_pod keywords) of the zone-keyed InterPodAffinity cases
    "anti": ([1, 1, 2, 2, 3, 3, 0, 0], 6, dict(required_anti_affinity=[{"labelSelector": WEB, "topologyKey": ZONE}])),
    "affinity": ([0, 1, 1, 2, 2, 3, 3], 5, dict(required_affinity=[{"labelSelector": WEB, "topologyKey": ZONE}])),
    "preferred": ([1, 2, 3, 1, 2, 3], 6, dict(preferred_anti_affinity=[
        {"weight": 100, "podAffinityTerm": {"labelSelector": WEB, "topologyKey": ZONE}}])),
}


def _zone_world(name):
    zones, n, kw = ZONE_WORLDS[name]
    cl, preds = _zoned(len(zones), zones)
    return cl, _replicas(n, PodGroupTable(), **kw), preds, np.array(zones)


def test_oracle_zone_anti_affinity_one_per_zone():
    """Required anti-affinity with the zone key: one replica per zone, then the nodes without a zone label (the
    term has no pair there) take the rest."""
    cl, pods, preds, zone = _zone_world("anti")
    node, _, _, g = _run_oracle(F.build_config(profile=IPA_ONLY), cl, pods, preds)
    assert (node >= 0).all()
    assert sorted(zone[node[:3]]) == [1, 2, 3] and (zone[node[3:]] == 0).all()
    assert list(g["anti_z"][:, 0]) == list(np.bincount(node, minlength=len(zone)))


def test_oracle_zone_affinity_follows_the_first_pod():
    """Required affinity with the zone key: the first pod of the series goes to a labelled node, the rest to its
    zone (any node of it), never to the node without the label."""
    cl, pods, preds, zone = _zone_world("affinity")
    node, _, _, _ = _run_oracle(F.build_config(profile=IPA_ONLY), cl, pods, preds)
    assert (node > 0).all() and (zone[node] == zone[node[0]]).all()
    assert len(set(node)) == 2  # NodeResourcesFit spreads them over the zone's two nodes


def test_oracle_zone_preferred_anti_affinity_spreads_zones():
    cl, pods, preds, zone = _zone_world("preferred")
    node, _, _, _ = _run_oracle(F.build_config(profile=IPA_ONLY), cl, pods, preds)
    assert sorted(zone[node[:3]]) == [1, 2, 3] and sorted(np.bincount(zone[node])[1:]) == [2, 2, 2]


def test_pod_group_table_compiles_selectors():
    t = PodGroupTable()
    g1 = t.group({"matchLabels": {"app": "web"}}, ("default",))
    g2 = t.group({"matchExpressions": [{"key": "tier", "operator": "In", "values": ["fe", "be"]}]}, ("default", "x"))
    g3 = t.group(None, ("default",))  # nil selector matches nothing
    both = t.conjunction([g1, g2])
    assert t.matches(g1, {"app": "web"}, "default") and not t.matches(g1, {"app": "web"}, "other")
    assert t.matches(g2, {"tier": "be"}, "x") and not t.matches(g2, {}, "x")
    assert not t.matches(g3, {"app": "web"}, "default")
    assert t.matches(both, {"app": "web", "tier": "fe"}, "default") and not t.matches(both, {"app": "web"}, "default")
    pod = np.zeros(1, dtype=abi.POD_DTYPE)
    t.fill_pod(pod, {"app": "web", "tier": "fe"}, "default",
               required_affinity=[{"labelSelector": {"matchLabels": {"app": "web"}}},
                                  {"labelSelector": {"matchExpressions": [{"key": "tier", "operator": "In",
                                                                           "values": ["fe", "be"]}]},
                                   "namespaces": ["default", "x"]}])
    assert pod["pod_affinity_group"][0] == both
    assert pod["pod_affinity_terms"][0] == (1 << (g1 - 1)) | (1 << (g2 - 1))
    assert (pod["match_groups"][0] >> (both - 1)) & 1
    with pytest.raises(NotImplementedError):
        t.fill_pod(pod, {}, "default", spread=[{"maxSkew": 1, "topologyKey": "topology.kubernetes.io/region",
                                                "labelSelector": {}}])
    t.fill_pod(pod, {}, "default", spread=[{"maxSkew": 2, "topologyKey": "topology.kubernetes.io/zone",
                                            "labelSelector": {}, "whenUnsatisfiable": "ScheduleAnyway"}])
    assert pod["n_spread"][0] == 1 and pod["spread_flags"][0, 0] == abi.SPREAD_ZONE


def test_duplicate_required_affinity_terms_stay_on_go_path():
    """(r5) Upstream adds HardPodAffinityWeight once per required term (processExistingPod); the ABI's
    group bitmask would count two identical terms once, so PodGroupTable refuses such a pod."""
    t = PodGroupTable()
    pod = F.make_pod(requests={"cpu": "1"})
    term = {"labelSelector": {"matchLabels": {"app": "db"}}, "topologyKey": "kubernetes.io/hostname"}
    with pytest.raises(NotImplementedError):
        t.fill_pod(pod, {"app": "web"}, "default", required_affinity=[term, dict(term)])
    t.fill_pod(pod, {"app": "web"}, "default", required_affinity=[term])  # one term is fine
    assert pod["pod_affinity_terms"][0] != 0


# ---- device vs oracle -------------------------------------------------------------------------------------------
def _world(n_nodes, n_pods, seed, with_preds=True, zones=True):
    cluster = synth.make_cluster(n_nodes, seed=seed)
    synth.make_pod_groups(cluster.existing_pods, seed=seed + 3, zones=zones)
    pods = synth.make_pods(n_pods, seed=seed + 1)
    synth.make_pod_groups(pods, seed=seed + 4, zones=zones)
    preds = synth.make_predicates(n_nodes, pods, seed=seed + 2, no_zone=0.05)[1] if with_preds else None
    return cluster, pods, preds


def _device(cfg, cluster, pods, preds, calls=1):
    with Engine(cfg, cluster.n) as e:
        synth.load_into(e, cluster)
        if preds is not None:
            e.upsert_predicates(preds)
        e.stage(pods)
        bounds = np.linspace(0, len(pods), calls + 1).astype(int)
        for a, b in zip(bounds[:-1], bounds[1:]):
            e.schedule_staged(int(a), int(b - a))
        node, score = e.fetch(0, len(pods))
        groups = e.read_pod_groups(zone=True)
        state = e.read_state()
    return node, score, groups, state


def _check(cfg, cluster, pods, preds, calls=1):
    want, want_score, st, g = _run_oracle(cfg, cluster, pods, preds, n_threads=8)
    node, score, (cnt, anti, symw, anti_z, symw_z), state = _device(cfg, cluster, pods, preds, calls)
    bad = np.nonzero((node != want) | (score != want_score))[0]
    assert len(bad) == 0, f"first mismatch at pod {bad[0]}: gpu ({node[bad[0]]}, {score[bad[0]]}) " \
                          f"oracle ({want[bad[0]]}, {want_score[bad[0]]})"
    assert np.array_equal(cnt, g["cnt"][:cluster.n]) and np.array_equal(anti, g["anti"][:cluster.n])
    assert np.array_equal(symw, g["symw"][:cluster.n])
    assert np.array_equal(anti_z, g["anti_z"][:cluster.n]) and np.array_equal(symw_z, g["symw_z"][:cluster.n])
    assert np.array_equal(state["requested_cpu"], st["requested"][:, abi.RES_CPU])
    return want


def test_oracle_zone_constraints_bite():
    """Zone constraints change placements against hostname-only ones, and every zone-keyed DoNotSchedule pod lands
    on a node carrying a zone label."""
    cfg = F.build_config(profile=SPREAD_ONLY)
    cluster, pods, preds = _world(300, 200, 65)
    node, _, _, _ = _run_oracle(cfg, cluster, pods, preds)
    cluster2, pods2, preds2 = _world(300, 200, 65, zones=False)
    node2, _, _, _ = _run_oracle(cfg, cluster2, pods2, preds2)
    assert (node != node2).any()
    hz = ((pods["spread_flags"] & (abi.SPREAD_HARD | abi.SPREAD_ZONE)) == (abi.SPREAD_HARD | abi.SPREAD_ZONE)).any(1)
    placed = node >= 0
    assert (preds["zone"][node[hz & placed]] > 0).all() and (hz & placed).any()


@pytest.mark.gpu
@pytest.mark.parametrize("name,profile", [("spread", SPREAD_ONLY), ("interpod", IPA_ONLY), ("stock", STOCK)])
def test_device_matches_oracle(name, profile):
    cluster, pods, preds = _world(2000, 600, 61)
    node = _check(F.build_config(profile=profile), cluster, pods, preds, calls=2)
    assert (node >= 0).mean() > 0.5


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(ZONE_WORLDS))
def test_device_zone_interpod_cases(name):
    """The zone-keyed InterPodAffinity worlds above, on the device (one pod per call and one call for all)."""
    cl, pods, preds, _ = _zone_world(name)
    for calls in (1, len(pods)):
        _check(F.build_config(profile=IPA_ONLY), cl, pods, preds, calls)


@pytest.mark.gpu
def test_device_system_default_constraints():
    """(ABI 13) A third of the pods without constraints of their own carry the system defaults (hostname + zone,
    ScheduleAnyway, KG_SPREAD_SYSTEM_DEFAULT) on a cluster where 5 % of the nodes lack the zone label: device vs oracle
    bit-exact, in one call and one pod per call."""
    cluster = synth.make_cluster(1500, seed=131)
    synth.make_pod_groups(cluster.existing_pods, seed=134, zones=True)
    pods = synth.make_pods(300, seed=132)
    synth.make_pod_groups(pods, seed=135, zones=True, system_default=0.35)
    assert ((pods["spread_flags"][:, 0] & abi.SPREAD_SYSTEM_DEFAULT) != 0).sum() >= 15
    preds = synth.make_predicates(1500, pods, seed=133, no_zone=0.05)[1]
    for calls in (1, 300):
        _check(F.build_config(profile=STOCK), cluster, pods, preds, calls)


@pytest.mark.gpu
def test_device_matches_oracle_10k_nodes():
    """The verdict's bar: both plugins in the stock profile at 10k nodes (HardPodAffinityWeight 3)."""
    cluster, pods, preds = _world(10_000, 400, 71)
    _check(F.build_config(profile=STOCK, hard_pod_affinity_weight=3), cluster, pods, preds, calls=3)


@pytest.mark.gpu
def test_device_single_pod_calls_and_unreserve():
    """One pod per call, then Unreserve of every other placed pod: the group counters go back exactly."""
    cfg = F.build_config(profile=STOCK)
    cluster, pods, preds = _world(500, 120, 81)
    want = _check(cfg, cluster, pods, preds, calls=120)
    with Engine(cfg, cluster.n) as e:
        synth.load_into(e, cluster)
        e.upsert_predicates(preds)
        e.stage(pods)
        e.schedule_staged(0, len(pods))
        before = e.read_pod_groups()
        mask = (np.arange(len(pods)) % 2 == 0).astype(np.uint8)
        e.unreserve(0, len(pods), mask)
        after = e.read_pod_groups()
    g = oracle.groups_init(cluster.n, cluster.existing_pods, cluster.existing_node)
    for j in np.nonzero(want >= 0)[0]:
        if not mask[j]:
            oracle.groups_apply(g, int(want[j]), pods[j:j + 1], 1)
    assert not np.array_equal(before[0], after[0])
    assert np.array_equal(after[0], g["cnt"][:cluster.n]) and np.array_equal(after[2], g["symw"][:cluster.n])


@pytest.mark.gpu
def test_pods_add_remove_feed_the_counters():
    cfg = F.build_config(profile=STOCK)
    cluster, pods, preds = _world(300, 50, 91)
    g = oracle.groups_init(cluster.n, cluster.existing_pods, cluster.existing_node)
    with Engine(cfg, cluster.n) as e:
        synth.load_into(e, cluster)
        cnt, anti, symw = e.read_pod_groups()
        assert np.array_equal(cnt, g["cnt"][:cluster.n]) and np.array_equal(anti, g["anti"][:cluster.n])
        assert np.array_equal(symw, g["symw"][:cluster.n])
        e.remove_pods(cluster.existing_pods[:100], cluster.existing_node[:100])
        for k in range(100):
            oracle.groups_apply(g, int(cluster.existing_node[k]), cluster.existing_pods[k:k + 1], -1)
        assert np.array_equal(e.read_pod_groups()[0], g["cnt"][:cluster.n])
