"""Reservation BeforePreFilter restore and nomination against the reference's transformer_test.go
and nominator_test.go tables (tests/golden/reservation.json "restore" / the nominator cases, written by
tests/golden/make_golden_resv.py with source lines).

The oracle (or_rsv_restore) and the device (kg_pods_evaluate_reservation, the exact pass's per-node evaluation) both
report the restored NodeInfo — Requested, NonZeroRequested, pod count —, the matched slots and the state's podRequested;
nominations run through the device on one-node engines.  TestMultiReservationsOnSameNode (nominator_test.go:353) runs as
a scheduling queue on both sides."""
import numpy as np
import pytest

import golden_cases as G
from koordinator_amd import Engine, abi, framework as F
from koordinator_amd.predicates import PredicateTable
from oracle import oracle

GI = 1 << 30
DOC = G.load("reservation.json")
PROFILE = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.RESERVATION), score={F.NODE_RESOURCES_FIT: 1, F.RESERVATION: 5000})


def _slots(slots):
    r = np.zeros(1, dtype=abi.NODE_RSV_DTYPE)
    r[0]["n"] = len(slots)
    for s, d in enumerate(slots):
        for k, v in d.items():
            r[0][k][s] = v
        r[0]["available"][s] = 1
    return r


def _pods(spec):
    out = []
    for cpu, mem, reserve in spec:
        p = F.make_pod({"cpu": str(cpu), "memory": f"{mem}Gi"}, priority_class="koord-prod")
        if reserve:
            p["flags"] |= abi.POD_RESERVE
        out.append(p)
    return np.concatenate(out) if out else np.zeros(0, dtype=abi.POD_DTYPE)


def _pod(c, table=None):
    p = F.make_pod({})
    p["reservation_owner_mask"] = c["mask"]
    p["reservation_flags"] = abi.POD_RSV_AFFINITY if c["affinity"] else 0
    if table is not None and c.get("rsv_affinity"):
        a = c["rsv_affinity"]
        table.fill_reservation_affinity(p, selector=a.get("selector"), required_terms=a.get("terms"))
    return p


def _case(c):
    """(pod, slots) of a restore case; a case with labels compiles the pod's reservation affinity and then the slots'
    fakeNode predicates through one PredicateTable (ABI 12)."""
    table = PredicateTable() if "slot_labels" in c else None
    pod = _pod(c, table)
    slots = _slots(c["slots"])
    if table is not None:
        for s, labels in enumerate(c["slot_labels"]):
            slots[0]["predicates"][s] = table.reservation_predicates(c.get("node_labels"), labels, f"r{s}")
        slots[0]["predicate_count"] = len(table.preds)
    return pod, slots


def _node(c):
    return F.make_node({"cpu": str(c["node"][0]), "memory": f"{c['node'][1]}Gi"})


@pytest.mark.parametrize("c", DOC["restore"], ids=lambda c: c["ref"].split(" ")[0])
def test_restore_oracle(c):
    cfg = F.build_config(profile=PROFILE)
    st = oracle.states(1)
    pods = _pods(c["pods"])
    oracle.add_pods(cfg, st, pods, np.zeros(len(pods), np.int32))
    pod, slots = _case(c)
    got = oracle.rsv_restore(slots, st, pod)
    for k, v in c["want"].items():
        assert got[k] == v, (c["ref"], k)


@pytest.mark.gpu
@pytest.mark.parametrize("c", DOC["restore"], ids=lambda c: c["ref"].split(" ")[0])
def test_restore_device(c):
    with Engine(F.build_config(profile=PROFILE), 1) as e:
        e.upsert_nodes(_node(c))
        pods = _pods(c["pods"])
        e.add_pods(pods, np.zeros(len(pods), np.int32))
        pod, slots = _case(c)
        e.upsert_reservations(slots)
        ev = e.evaluate_reservation(pod)
    for k, v in c["want"].items():
        assert int(ev[k][0]) == v, (c["ref"], k)


NOMINATOR = [c for c in DOC["cases"] if c["ref"].startswith("nominator_test.go")]


@pytest.mark.gpu
@pytest.mark.parametrize("c", NOMINATOR, ids=lambda c: c["ref"].split(" ")[0])
def test_nominate_device(c):
    """NominateReservation on the device for the nominator_test.go cases: a one-node engine whose NodeInfo holds the
    reserve pods (requests = allocatable), the pod matching every slot's owner group."""
    node = F.make_node({"cpu": "64", "memory": "256Gi"})
    with Engine(F.build_config(profile=PROFILE), 1) as e:
        e.upsert_nodes(node)
        rp = _pods([[s["allocatable_cpu"] // 1000, s["allocatable_mem"] // GI, 1] for s in c["slots"]])
        if len(rp):
            e.add_pods(rp, np.zeros(len(rp), np.int32))
        slots = [dict(s, assigned=1 if s["allocated_cpu"] else 0) for s in c["slots"]]
        e.upsert_reservations(_slots(slots))
        pod = F.make_pod({"cpu": f"{c['pod'][0]}m", "memory": str(c["pod"][1])})
        pod["reservation_owner_mask"] = 1
        if c.get("reserve"):
            pod["flags"] |= abi.POD_RESERVE
        ev = e.evaluate_reservation(pod)
    assert int(ev["nominated"][0]) == c["want_nominated"], c["ref"]


def _multi_case():
    """nominator_test.go:353 TestMultiReservationsOnSameNode: three Restricted, reusable 16C32G reservations with the
    same owner on a 96-cpu node, and three 16C32G pods with a required reservation affinity: every reservation is
    nominated exactly once."""
    cfg = F.build_config(profile=PROFILE)
    node = F.make_node({"cpu": "96", "memory": "1886495404Ki"})
    slots = [dict(allocatable_cpu=16000, allocatable_mem=32 * GI, policy=abi.RSV_POLICY["Restricted"], owner=0,
                  allocate_once=0)] * 3
    reserve = _pods([[16, 32, 1]] * 3)
    pods = np.concatenate([F.make_pod({"cpu": "16", "memory": "32Gi"})] * 3)
    pods["reservation_owner_mask"] = 1
    pods["reservation_flags"] = abi.POD_RSV_AFFINITY
    return cfg, node, _slots(slots), reserve, pods


def test_multi_reservations_same_node_oracle():
    cfg, node, rsv, reserve, pods = _multi_case()
    st = oracle.states(1)
    oracle.add_pods(cfg, st, reserve, np.zeros(len(reserve), np.int32))
    metric = F.make_node_metric(present=False)
    got, _, slot = oracle.schedule_resv(cfg, node, metric, st, rsv, pods, 0)
    assert got.tolist() == [0, 0, 0] and sorted(slot.tolist()) == [0, 1, 2]


@pytest.mark.gpu
def test_multi_reservations_same_node_device():
    cfg, node, rsv, reserve, pods = _multi_case()
    with Engine(cfg, 1) as e:
        e.upsert_nodes(node)
        e.update_metrics(F.make_node_metric(present=False), 0)
        e.add_pods(reserve, np.zeros(len(reserve), np.int32))
        e.upsert_reservations(rsv)
        got, _, _ = e.schedule(pods)
        slot = e.fetch_reservations(0, len(pods))
    assert got.tolist() == [0, 0, 0] and sorted(slot.tolist()) == [0, 1, 2]
