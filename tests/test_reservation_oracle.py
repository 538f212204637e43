"""Reservation scheduling loop of the oracle (or_schedule_resv) — CPU checks of its composition: with the plugin
off it is the Fit + LoadAware loop; with it on, placements land in reservations and Reserve's bookkeeping adds up."""
import numpy as np

from koordinator_amd import abi, framework as F, synth
from oracle import oracle

PROFILE = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.RESERVATION),
                    score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.RESERVATION: 5000})
BASE = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE), score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1})


def run(cfg, cluster, rsv, pods):
    st = oracle.states(cluster.n)
    oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
    r = rsv.copy()
    node, score, slot = oracle.schedule_resv(cfg, cluster.nodes, cluster.metrics, st, r, pods, cluster.now_ns)
    return node, score, slot, st, r


def test_plugin_off_equals_fit_loadaware_loop():
    cluster, rsv = synth.make_rsv_cluster(300, seed=5)
    pods = synth.make_rsv_pods(400, seed=6)
    cfg = F.build_config(profile=BASE)
    node, score, slot, _, _ = run(cfg, cluster, rsv, pods)
    st = oracle.states(cluster.n)
    oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
    wn, ws, _, _ = oracle.schedule_full(cfg, cluster.nodes, cluster.metrics, st, pods, cluster.now_ns, 1)
    assert np.array_equal(node, wn) and np.array_equal(score, ws)
    assert (slot == -1).all()


def test_reserve_bookkeeping_and_affinity():
    cluster, rsv = synth.make_rsv_cluster(300, seed=7)
    pods = synth.make_rsv_pods(600, seed=8)
    cfg = F.build_config(profile=PROFILE)
    node, score, slot, st, r = run(cfg, cluster, rsv, pods)
    assert (slot >= 0).sum() > 10  # owned pods land in their reservations (weight 5000)
    for j in np.nonzero(slot >= 0)[0]:
        i, s = node[j], slot[j]
        assert (int(pods[j]["reservation_owner_mask"]) >> int(rsv[i]["owner"][s])) & 1
    got = r["allocated_cpu"] - rsv["allocated_cpu"]
    want = np.zeros_like(got)
    np.add.at(want, (node[slot >= 0], slot[slot >= 0]), pods["requests"][slot >= 0, abi.RES_CPU])
    want *= rsv["allocatable_cpu"] > 0  # Allocated += Mask(requests, ResourceNames): memory-only keeps cpu absent
    assert np.array_equal(got, want)
    assert np.array_equal(r["assigned"] - rsv["assigned"],
                          np.bincount(node[slot >= 0] * abi.MAX_RSV_SLOTS + slot[slot >= 0],
                                      minlength=cluster.n * abi.MAX_RSV_SLOTS).reshape(cluster.n, -1))
    aff = (pods["reservation_flags"] & abi.POD_RSV_AFFINITY) != 0
    assert ((slot >= 0) | (node < 0))[aff].all()  # required affinity: placed only through a reservation


def _affinity_ok(pod, pred):
    """RequiredReservationAffinity.Match on a slot's predicate bits (the restatement the engine and oracle share)."""
    if not pod["reservation_flags"] & abi.POD_RSV_AFFINITY:
        return True
    sel = int(pod["reservation_selector"])
    if pred & sel != sel:
        return False
    n = int(pod["n_reservation_terms"])
    return n == 0 or any(int(t) != 0 and pred & int(t) == int(t) for t in pod["reservation_terms"][:n])


def test_reservation_affinity_selectors_bite():
    """(ABI 12) Selectors narrower than the owner groups change the matched reservations: placements differ from the
    owner-only run, and every pod assumed into a slot satisfies its affinity on that slot's fakeNode predicates."""
    cluster, rsv = synth.make_rsv_cluster(300, seed=81)
    pods = synth.make_rsv_pods(900, seed=82)
    pods["reservation_flags"] = np.where(pods["reservation_owner_mask"] != 0, abi.POD_RSV_AFFINITY, 0)
    cfg = F.build_config(profile=PROFILE)
    base_node, _, base_slot, _, _ = run(cfg, cluster, rsv, pods)
    synth.add_reservation_affinity(rsv, pods, seed=83)
    node, _, slot, _, _ = run(cfg, cluster, rsv, pods)
    assert (node != base_node).any() or (slot != base_slot).any()
    placed = np.nonzero(slot >= 0)[0]
    assert len(placed) > 5
    for j in placed:
        assert _affinity_ok(pods[j], int(rsv["predicates"][node[j], slot[j]]))
