"""The preemption dry run's Filter (kg_pods_filter_preemption): the restored node minus the victims
(NodeInfo.RemovePod) under NodeResourcesFit + LoadAware, and the Reservation Filter with the victims' requests as
`preemptible` / `preemptibleInRRs` (reservation/plugin.go:254-315 AddPod / RemovePod, :318-428 Filter and
filterWithReservations, :433-482 fitsNode).

Pinned by the reference's own tables: TestFilterWithPreemption (plugin_test.go:575-668) and the preemption rows of
Test_filterWithReservations (plugin_test.go:866-1260).  Those tests write the cycle state directly; here each row is
the NodeInfo + reservation that BeforePreFilter's restore turns into that state (podRequested, rAllocated, matched)
and the victims whose RemovePod builds that preemptible map, so the same rows run on the oracle (CPU) and through
the C ABI on the device (GPU).  Bar: bit-exact KG_REJECT_* bits."""
import numpy as np
import pytest

from koordinator_amd import Engine, abi, framework as F, synth
from oracle import oracle
from test_reservation_oracle import PROFILE

GI = 1 << 30
RSV_ONLY = F.Profile(filter=(F.RESERVATION,), score={F.NODE_RESOURCES_FIT: 1})
REJ = abi.REJECT_RESERVATION


def _pod(cpu_m, mem=0, affinity=False, owner=1):
    req = {"cpu": f"{cpu_m}m"}
    if mem:
        req["memory"] = str(mem)
    p = F.make_pod(requests=req, limits=req)
    p["reservation_owner_mask"] = owner
    p["reservation_flags"] = abi.POD_RSV_AFFINITY if affinity else 0
    return p


def _victims(spec):
    """[(cpu_m, mem, slot)] -> (POD_DTYPE[k], int32[k]): slot -1 = the victim was not allocated from a reservation
    (RemovePod adds it to preemptible), s >= 0 = from slot s (preemptibleInRRs[s])."""
    v = np.zeros(len(spec), dtype=abi.POD_DTYPE)
    for k, (c, m, *_rest) in enumerate(spec):
        req = {"cpu": f"{c}m"} if c else {}
        if m:
            req["memory"] = str(m)
        v[k] = F.make_pod(requests=req, limits=req)[0]
        if _rest[1:] == ["reserve"]:  # a reservation's reserve pod (RemovePod skips it: plugin.go:286)
            v[k]["flags"] |= abi.POD_RESERVE
    return v, np.array([t[2] for t in spec], dtype=np.int32)


def _rsv(policy, owner, alloc_cpu, allocd_cpu, assigned):
    r = np.zeros(1, dtype=abi.NODE_RSV_DTYPE)
    r["n"] = 1
    r["owner"][0, 0] = owner
    r["available"][0, 0] = 1
    r["policy"][0, 0] = policy
    r["allocatable_cpu"][0, 0] = alloc_cpu
    r["allocated_cpu"][0, 0] = allocd_cpu
    r["assigned"][0, 0] = assigned
    return r


# Each case: the node's NodeInfo requested cpu (before the restore), the reservation, the pod, the victims and the
# reference's expected verdict.  Node: 32 cpu / 32Gi / 100 pods (the tests' node).
# unmatched (owner group 5, the pod owns group 0), assigned: podRequested = 36 - 4 = 32, rAllocated none
_UNMATCHED = dict(requested=36000, rsv=(abi.RSV_POLICY["Default"], 5, 4000, 4000, 1))
_DEFAULT = dict(rsv=(abi.RSV_POLICY["Default"], 0, 6000, 6000, 1))          # matched, rAllocated = 6
_RESTRICTED = dict(rsv=(abi.RSV_POLICY["Restricted"], 0, 6000, 6000, 1))
CASES = [
    dict(ref="plugin_test.go:594 non-reservations with preemption", **_UNMATCHED,
         pod=(4000, 0, False), victims=[(4000, 0, -1)], want=0),
    dict(ref="plugin_test.go:615 failed non-reservations with preemption", **_UNMATCHED,
         pod=(4000, 0, False), victims=[(2000, 0, -1)], want=REJ),
    dict(ref="plugin_test.go:636 preemption but no preemptible resources", **_UNMATCHED,
         pod=(4000, 0, False), victims=[], want=0),
    # (r5) plugin.go:286: RemovePod returns before counting a reserve pod.  The victim still leaves the
    # NodeInfo copy (NodeResourcesFit passes), but it adds nothing to preemptible: fitsNode needs 32 − 2 + 4 ≤ 32 and
    # rejects, where two ordinary 2-cpu victims make 32 − 4 + 4 and pass (the :594 row split in two)
    dict(ref="plugin.go:286 RemovePod skips a reserve-pod victim", **_UNMATCHED,
         pod=(4000, 0, False), victims=[(2000, 0, -1), (2000, 0, -1, "reserve")], want=REJ),
    dict(ref="plugin.go:286-control two ordinary victims", **_UNMATCHED,
         pod=(4000, 0, False), victims=[(2000, 0, -1), (2000, 0, -1)], want=0),
    dict(ref="plugin_test.go:867 default reservations with preemption", requested=36000, **_DEFAULT,
         pod=(4000, 0, False), victims=[(4000, 0, 0)], want=0),
    dict(ref="plugin_test.go:912 default reservations, preempt from reservation and node", requested=38000,
         **_DEFAULT, pod=(4000, 0, False), victims=[(2000, 0, -1), (2000, 0, 0)], want=0),
    dict(ref="plugin_test.go:962 failed default reservations, preempt from reservation", requested=38000,
         **_DEFAULT, pod=(4000, 0, True), victims=[(2000, 0, 0)], want=REJ),
    dict(ref="plugin_test.go:1008 failed default reservations, preempt from node", requested=38000, **_DEFAULT,
         pod=(4000, 0, True), victims=[(2000, 0, -1)], want=REJ),
    dict(ref="plugin_test.go:1052 restricted reservations, preempt from reservation", requested=38000,
         **_RESTRICTED, pod=(4000, 0, False), victims=[(4000, 0, 0)], want=0),
    dict(ref="plugin_test.go:1100 failed restricted reservations, preempt from node", requested=38000,
         **_RESTRICTED, pod=(4000, 0, True), victims=[(4000, 0, -1)], want=REJ),
    dict(ref="plugin_test.go:1148 failed restricted, preempt from reservation and node", requested=38000,
         **_RESTRICTED, pod=(4000, 0, True), victims=[(2000, 0, -1), (2000, 0, 0)], want=REJ),
    dict(ref="plugin_test.go:1205 restricted, preempt from reservation and node", requested=38000,
         **_RESTRICTED, pod=(4000, 4 * GI, False), victims=[(0, 32 * GI, -1), (4000, 0, 0)], want=0),
]


def golden_cluster(case):
    """One node whose NodeInfo holds `requested` cpu: the reserve pod plus a filler pod (and, for the restore's
    matched / unmatched split, nothing else); the victims are further pods on it."""
    node = F.make_node({"cpu": "32", "memory": "32Gi"}, allowed_pods=100)
    metric = F.make_node_metric(present=False, node_usage=None)
    vic, slots = _victims(case["victims"])
    others = case["requested"] - int(vic["requests"][:, abi.RES_CPU].sum())
    filler = F.make_pod(requests={"cpu": f"{others}m"})
    existing = np.concatenate([filler, vic]) if len(vic) else filler
    cluster = synth.Cluster(node, metric, existing, np.zeros(len(existing), dtype=np.int32), 10**18)
    return cluster, _rsv(*case["rsv"]), _pod(*case["pod"]), vic, slots


def oracle_verdict(cfg, cluster, rsv, pod, vic, slots, node=0):
    st = oracle.states(cluster.n)
    oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
    return oracle.filter_preemption(cfg, cluster.nodes[node], cluster.metrics[node], st[node:node + 1],
                                    rsv[node] if rsv is not None else None, pod, vic, slots, cluster.now_ns)


@pytest.mark.parametrize("case", CASES, ids=[c["ref"].split(" ", 1)[0] for c in CASES])
def test_oracle_reference_tables(case):
    cluster, rsv, pod, vic, slots = golden_cluster(case)
    cfg = F.build_config(profile=RSV_ONLY)
    assert oracle_verdict(cfg, cluster, rsv, pod, vic, slots) == case["want"], case["ref"]


def test_oracle_restore_reproduces_the_tables_state():
    """The restore of the golden NodeInfo gives the state the reference tests write: podRequested 32 (unmatched) /
    36 / 38 cpu and rAllocated 6 cpu with the one matched reservation."""
    by = {c["ref"].split(" ", 1)[0]: c for c in CASES}
    for case in (by["plugin_test.go:594"], by["plugin_test.go:867"], by["plugin_test.go:912"]):
        cluster, rsv, pod, _, _ = golden_cluster(case)
        st = oracle.states(1)
        oracle.add_pods(F.build_config(profile=RSV_ONLY), st, cluster.existing_pods, cluster.existing_node)
        s = oracle.rsv_restore(rsv[0], st, pod)
        assert s["has_state"] == 1
        assert s["pod_requested_cpu"] == (32000 if case is CASES[0] else case["requested"])
        assert s["r_allocated_cpu"] == (0 if case is CASES[0] else 6000)
        assert s["matched"] == (0 if case is CASES[0] else 1)


def test_oracle_victims_free_fit():
    """NodeResourcesFit on the victim-free NodeInfo: a node full by the victims passes once they leave."""
    node = F.make_node({"cpu": "8", "memory": "8Gi"})
    vic, slots = _victims([(6000, 0, -1)])
    cluster = synth.Cluster(node, F.make_node_metric(present=False, node_usage=None), vic,
                            np.zeros(1, dtype=np.int32), 10**18)
    cfg = F.build_config(profile=F.Profile(filter=(F.NODE_RESOURCES_FIT,), score={F.NODE_RESOURCES_FIT: 1}))
    pod = _pod(4000)
    assert oracle_verdict(cfg, cluster, None, pod, vic[:0], slots[:0]) & abi.REJECT_FIT_CPU
    assert oracle_verdict(cfg, cluster, None, pod, vic, slots) == 0


def device_verdict(cfg, cluster, rsv, pod, vic, slots, node=0):
    with Engine(cfg, cluster.n) as e:
        synth.load_rsv_into(e, cluster, rsv) if rsv is not None else synth.load_into(e, cluster)
        return e.filter_preemption(pod, node, vic, slots)


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=[c["ref"].split(" ", 1)[0] for c in CASES])
def test_device_reference_tables(case):
    cluster, rsv, pod, vic, slots = golden_cluster(case)
    for prof in (RSV_ONLY, PROFILE):
        cfg = F.build_config(profile=prof)
        got = device_verdict(cfg, cluster, rsv, pod, vic, slots)
        assert got == oracle_verdict(cfg, cluster, rsv, pod, vic, slots), (case["ref"], prof)
        if prof is RSV_ONLY:
            assert got == case["want"], case["ref"]


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_device_matches_oracle_random(seed):
    """Random C5-style clusters (reservations of every policy, owned / affinity pods) and random victim sets drawn
    from each node's pods, some attributed to a reservation slot: device verdict == oracle verdict, for the
    Reservation-only profile and Fit + LoadAware + Reservation."""
    cluster, rsv = synth.make_rsv_cluster(64, seed=900 + seed)
    pods = synth.make_rsv_pods(64, seed=950 + seed)
    rng = np.random.default_rng(seed)
    for prof in (RSV_ONLY, PROFILE):
        cfg = F.build_config(profile=prof)
        st = oracle.states(cluster.n)
        oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
        with Engine(cfg, cluster.n) as e:
            synth.load_rsv_into(e, cluster, rsv)
            seen = set()
            for j in range(len(pods)):
                i = int(rng.integers(cluster.n))
                on = np.nonzero(cluster.existing_node == i)[0]
                k = int(rng.integers(0, len(on) + 1))
                pick = rng.choice(on, size=k, replace=False) if k else on[:0]
                vic = cluster.existing_pods[pick]
                slots = np.where(rng.random(k) < 0.4, rng.integers(0, max(int(rsv["n"][i]), 1), k), -1).astype(np.int32)
                pod = pods[j:j + 1]
                want = oracle.filter_preemption(cfg, cluster.nodes[i], cluster.metrics[i], st[i:i + 1], rsv[i], pod,
                                                vic, slots, cluster.now_ns)
                got = e.filter_preemption(pod, i, vic, slots)
                assert got == want, (prof, j, i, k, got, want)
                seen.add(want)
        assert len(seen) > 1  # both verdicts occur
