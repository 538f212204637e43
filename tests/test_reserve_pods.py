"""(ABI 12) Scheduling a Reservation's reserve pod, and pods in reservation operating mode (SURVEY §8a A16:
Reservation.Filter's allocate-policy conflict, reservation/plugin.go:324-350).

A staged pod with KG_POD_RESERVE matches no reservation (transformer.go:112), is pinned to the node its reservation
names (GetReservePodNodeName) and is rejected on a node holding an available reservation whose allocate policy conflicts
with its own (Default coexists with no other policy); its Reservation Score is MinNodeScore (scoring.go:104-106).
Pinned by the reserve-pod rows of plugin_test.go TestFilter (:318-520), transcribed below as data, on the oracle and
through the device's per-node evaluation; random queues mixing reserve pods into the C5-Reservation world run
device vs oracle bit-exact."""
import numpy as np
import pytest

from koordinator_amd import Engine, abi, framework as F, synth
from oracle import oracle

PROFILE = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.RESERVATION), score={F.NODE_RESOURCES_FIT: 1, F.RESERVATION: 5000})
POL = abi.RSV_POLICY
# plugin_test.go TestFilter (:318): test-node-0 = node 0 ("other-node" = node 1); the reservations available on node 0
# (alignedReservation / restrictedReservation, :376-420); the reserve pod's reservation policy and node name; want pass
FILTER_CASES = [
    dict(ref="plugin_test.go:452 skip for pod not set node", slots=[], policy="Default", pin=None, want=1),
    dict(ref="plugin_test.go:459 filter pod successfully", slots=[], policy="Default", pin=0, want=1),
    dict(ref="plugin_test.go:466 failed for node does not matches the pod", slots=[], policy="Default", pin=1, want=0),
    dict(ref="plugin_test.go:473 ReservationAllocatePolicyDefault cannot coexist with Aligned policy",
         slots=["Aligned"], policy="Default", pin=0, want=0),
    dict(ref="plugin_test.go:483 ReservationAllocatePolicyDefault cannot coexist with Restricted policy",
         slots=["Restricted"], policy="Default", pin=0, want=0),
    dict(ref="plugin_test.go:493 Aligned policy can coexist with Restricted policy",
         slots=["Aligned", "Restricted"], policy="Aligned", pin=None, want=1),
    dict(ref="plugin_test.go:503 Restricted policy can coexist with Aligned policy",
         slots=["Aligned", "Restricted"], policy="Restricted", pin=None, want=1),
]


def _slots(policies, n_nodes=2):
    r = np.zeros(n_nodes, dtype=abi.NODE_RSV_DTYPE)
    r[0]["n"] = len(policies)
    for s, pol in enumerate(policies):
        r[0]["policy"][s] = POL[pol]
        r[0]["available"][s] = 1
        r[0]["allocatable_cpu"][s] = 4000
        r[0]["owner"][s] = 0
    return r


def _reserve_pod(c):
    p = F.make_pod({"cpu": "4"})
    p["flags"] |= abi.POD_RESERVE
    p["reserve_allocate_policy"] = POL[c["policy"]]
    p["reserve_node"] = 0 if c["pin"] is None else c["pin"] + 1
    return p


@pytest.mark.parametrize("c", FILTER_CASES, ids=lambda c: c["ref"].split(" ")[0])
def test_reserve_pod_filter_oracle(c):
    rsv = _slots(c["slots"])
    got = oracle.lib().or_rsv_policy_filter(oracle.p(_reserve_pod(c)), 0, oracle.p(rsv[0:1]))
    assert got == c["want"], c["ref"]


def test_operating_mode_takes_the_aligned_check():
    """IsReservationOperatingMode pods (not reserve pods) take the conflict check with the Aligned policy."""
    p = F.make_pod({"cpu": "1"})
    p["reservation_flags"] = abi.POD_RSV_OPERATING
    L = oracle.lib()
    assert L.or_rsv_policy_filter(oracle.p(p), 0, oracle.p(_slots(["Default"])[0:1])) == 0
    assert L.or_rsv_policy_filter(oracle.p(p), 0, oracle.p(_slots(["Aligned", "Restricted"])[0:1])) == 1


def _mixed_world(seed, n_nodes=400, n_pods=1200):
    """The C5-Reservation world with 10 % reserve pods (random allocate policy, a third pinned to a random node) and
    5 % in reservation operating mode."""
    cluster, rsv = synth.make_rsv_cluster(n_nodes, seed=seed)
    pods = synth.make_rsv_pods(n_pods, seed=seed + 1)
    rng = np.random.default_rng(seed + 2)
    res = rng.random(n_pods) < 0.10
    pods["flags"] = np.where(res, pods["flags"] | abi.POD_RESERVE, pods["flags"])
    pods["reserve_allocate_policy"] = np.where(res, rng.integers(0, 3, n_pods), 0)
    pin = res & (rng.random(n_pods) < 1 / 3)
    pods["reserve_node"] = np.where(pin, rng.integers(0, n_nodes, n_pods) + 1, 0)
    op = ~res & (rng.random(n_pods) < 0.05)
    pods["reservation_flags"] = np.where(op, pods["reservation_flags"] | abi.POD_RSV_OPERATING, pods["reservation_flags"])
    return cluster, rsv, pods, res


def test_reserve_pods_bite_on_the_oracle():
    cluster, rsv, pods, res = _mixed_world(91)
    from test_reservation_oracle import run
    node, score, slot, _, _ = run(F.build_config(profile=PROFILE), cluster, rsv, pods)
    assert (slot[res] == -1).all()  # a reserve pod is never assumed into a reservation
    pinned = res & (pods["reserve_node"] > 0) & (node >= 0)
    assert pinned.any() and (node[pinned] == pods["reserve_node"][pinned] - 1).all()
    # the conflict rule holds on every node a reserve pod landed on
    for j in np.nonzero(res & (node >= 0))[0]:
        r = rsv[node[j]]
        pol = [int(r["policy"][s]) for s in range(int(r["n"])) if r["available"][s]]
        mine = int(pods["reserve_allocate_policy"][j])
        assert all(not ((mine == POL["Default"] or q == POL["Default"]) and mine != q) for q in pol)


@pytest.mark.gpu
@pytest.mark.parametrize("c", FILTER_CASES, ids=lambda c: c["ref"].split(" ")[0])
def test_reserve_pod_filter_device(c):
    nodes = np.concatenate([F.make_node({"cpu": "8", "memory": "16Gi"}) for _ in range(2)])
    with Engine(F.build_config(profile=PROFILE), 2) as e:
        e.upsert_nodes(nodes)
        e.update_metrics(np.concatenate([F.make_node_metric(present=False) for _ in range(2)]), 0)
        e.upsert_reservations(_slots(c["slots"]))
        ev = e.evaluate_reservation(_reserve_pod(c))
    assert int(ev["pass"][0]) == c["want"], c["ref"]
    assert int(ev["matched"][0]) == 0 and int(ev["score"][0]) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [91, 95])
def test_reserve_pods_device_matches_oracle(seed):
    from test_reservation_gpu import check
    cluster, rsv, pods, res = _mixed_world(seed)
    node, slot = check(F.build_config(profile=PROFILE), cluster, rsv, pods, chunks=2)
    assert (node[res] >= 0).any() and (slot[res] == -1).all()


@pytest.mark.gpu
def test_reservation_affinity_refused_against_older_slots():
    """(ABI 12) A queue whose reservation affinity uses a predicate the slots were not compiled against is refused
    (kg_node_reservations.predicate_count, like the node rows' ABI 11 check)."""
    from koordinator_amd.predicates import PredicateTable
    cluster, rsv = synth.make_rsv_cluster(50, seed=5)
    pods = synth.make_rsv_pods(20, seed=6)
    t = PredicateTable()
    pods["reservation_flags"] = abi.POD_RSV_AFFINITY
    t.fill_reservation_affinity(pods[0:1], selector={"reservation-type": "a"})
    rsv["predicate_count"] = 0  # compiled before the predicate existed
    with Engine(F.build_config(profile=PROFILE), cluster.n) as e:
        synth.load_rsv_into(e, cluster, rsv)
        e.stage(pods)
        with pytest.raises(abi.KoordGPUError, match="re-send the reservations"):
            e.schedule_staged(0, len(pods))
