"""GPU parity of the Reservation plugin (config C5's Reservation part): the HIP engine through the C ABI against
the oracle (oracle/reservation.c), itself pinned by the reference's test tables (tests/golden/reservation.json).

Bar: bit-exact — placements and weighted totals (Reservation weight 5000 with the PreScore preferred node and
DefaultNormalizeScore), the slot Reserve assumed every pod into, the reservations' Allocated / assigned counts and
the NodeInfo / LoadAware node state after the queue."""
import numpy as np
import pytest

from koordinator_amd import Engine, abi, framework as F, synth
from oracle import oracle
from test_golden_reservation import CASES, rsv_row
from test_reservation_oracle import BASE, PROFILE, run

pytestmark = pytest.mark.gpu


def engine_run(cfg, cluster, rsv, pods, chunks=1):
    with Engine(cfg, cluster.n) as e:
        synth.load_rsv_into(e, cluster, rsv)
        e.stage(pods)
        bounds = np.linspace(0, len(pods), chunks + 1).astype(int)
        for a, b in zip(bounds[:-1], bounds[1:]):
            e.schedule_staged(int(a), int(b - a))
        node, score = e.fetch(0, len(pods))
        slot = e.fetch_reservations(0, len(pods))
        state = e.read_state()
        ac, am, asg = e.read_reservations()
    return node, score, slot, state, (ac, am, asg)


def check(cfg, cluster, rsv, pods, chunks=1):
    wn, ws, wslot, st, r = run(cfg, cluster, rsv, pods)
    node, score, slot, state, (ac, am, asg) = engine_run(cfg, cluster, rsv, pods, chunks)
    bad = np.nonzero((node != wn) | (score != ws) | (slot != wslot))[0]
    assert len(bad) == 0, f"first mismatch at pod {bad[0]}: gpu ({node[bad[0]]}, {score[bad[0]]}, {slot[bad[0]]}) " \
                          f"oracle ({wn[bad[0]]}, {ws[bad[0]]}, {wslot[bad[0]]})"
    on = np.arange(abi.MAX_RSV_SLOTS)[None, :] < r["n"][:, None]
    assert np.array_equal(ac, np.where(on, r["allocated_cpu"], 0))
    assert np.array_equal(am, np.where(on, r["allocated_mem"], 0))
    assert np.array_equal(asg, np.where(on, r["assigned"], 0))
    assert np.array_equal(state["requested_cpu"], st["requested"][:, abi.RES_CPU])
    assert np.array_equal(state["num_pods"], st["num_pods"])
    return node, slot


@pytest.mark.parametrize("n_nodes,n_pods,seed", [(300, 1500, 1), (1000, 2000, 2), (257, 1200, 3), (2000, 1500, 4)])
def test_schedule_parity_synthetic(n_nodes, n_pods, seed):
    cluster, rsv = synth.make_rsv_cluster(n_nodes, seed=300 + seed)
    pods = synth.make_rsv_pods(n_pods, seed=400 + seed)
    node, slot = check(F.build_config(profile=PROFILE), cluster, rsv, pods, chunks=2)
    assert (node >= 0).mean() > 0.5 and (slot >= 0).sum() > 10


def test_schedule_parity_owner_heavy_small_cluster():
    """Few nodes, most pods owned: reservations fill up (Restricted / AllocateOnce stop matching), preferred
    nodes move, required-affinity pods become unschedulable."""
    cluster, rsv = synth.make_rsv_cluster(40, seed=51)
    pods = synth.make_rsv_pods(800, seed=52)
    pods["reservation_owner_mask"] = np.left_shift(1, np.arange(len(pods)) % 8)
    rsv["owner"] = rsv["owner"] % 8
    node, slot = check(F.build_config(profile=PROFILE), cluster, rsv, pods, chunks=3)
    assert (node < 0).any() and (slot >= 0).any()


def test_schedule_parity_reservation_affinity_selectors():
    """(ABI 12) Required reservation affinities narrower than the owner groups: reservationSelector and
    ReservationSelectorTerms over the slots' fakeNode labels (synth.add_reservation_affinity)."""
    cluster, rsv = synth.make_rsv_cluster(600, seed=71)
    pods = synth.make_rsv_pods(1500, seed=72)
    pods["reservation_flags"] = np.where(pods["reservation_owner_mask"] != 0, abi.POD_RSV_AFFINITY, 0)
    synth.add_reservation_affinity(rsv, pods, seed=73)
    assert (pods["reservation_selector"] != 0).any() and (pods["n_reservation_terms"] > 0).any()
    node, slot = check(F.build_config(profile=PROFILE), cluster, rsv, pods, chunks=2)
    assert (slot >= 0).sum() > 10


def test_schedule_parity_filter_only_and_plugin_off():
    cluster, rsv = synth.make_rsv_cluster(500, seed=61)
    pods = synth.make_rsv_pods(800, seed=62)
    for prof in (F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.RESERVATION),
                           score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1}),
                 F.Profile(filter=(F.NODE_RESOURCES_FIT, F.RESERVATION),
                           score={F.NODE_RESOURCES_FIT: 2, F.RESERVATION: 7})):
        check(F.build_config(profile=prof), cluster, rsv, pods)


@pytest.mark.parametrize("case", CASES, ids=[c["ref"] for c in CASES])
def test_golden_cases_place_like_the_oracle(case):
    """Each golden case as a 1-node cluster (NodeInfo holding the reserve pods): the engine's placement, total and
    slot equal the oracle loop's on the same cluster (a case without reservations: the plain Fit + LoadAware
    placement, slot -1)."""
    cluster = synth.make_cluster(1, seed=71)
    cluster.existing_pods = cluster.existing_pods[:0]
    cluster.existing_node = cluster.existing_node[:0]
    cluster.nodes["allocatable"][0, :2] = [64000, 256 << 30]
    rsv = np.zeros(1, dtype=abi.NODE_RSV_DTYPE)
    rsv[0] = rsv_row(case["slots"])
    pod = np.zeros(1, dtype=abi.POD_DTYPE)
    pod["requests"][0, :2] = pod["limits"][0, :2] = pod["nonzero_requests"][0] = case["pod"]
    if not any(case["pod"]):
        pod["nonzero_requests"][0] = [100, 200 << 20]
    pod["priority_class"] = abi.PRIO_PROD
    pod["reservation_owner_mask"] = 1
    pod["reservation_flags"] = abi.POD_RSV_AFFINITY if case.get("affinity") else 0
    if case.get("reserve"):
        pod["flags"] |= abi.POD_RESERVE
    check(F.build_config(profile=PROFILE), cluster, rsv, pod)
