"""(r6) The DeviceShare-reservation golden vectors (tests/golden/deviceshare.json, transcribed from
deviceshare/reservation_test.go:38-693, plugin_test.go:1670-1835, 1905-2047, 2937-3009 and scoring_test.go:579-854) through
the DEVICE: a one-node engine whose node holds the case's GPUs and one reservation (slot 0, owner group 0) holding the
case's minors, a pod of that owner group.  Observed through kg_pods_evaluate_reservation (Filter verdict, nominated
slot = FilterReservation + nomination, raw DeviceShare Score of the nominated reservation) and through scheduling
(Reserve's minors and deviceUsed).  tests/test_golden_deviceshare.py runs the same cases on the oracle."""
import numpy as np
import pytest

import test_golden_deviceshare as TG
from koordinator_amd import Engine, abi, framework as F

pytestmark = pytest.mark.gpu

PROFILE = F.Profile(filter=(F.RESERVATION, F.DEVICE_SHARE), score={F.RESERVATION: 1, F.DEVICE_SHARE: 1})


def engine_case(c, required=False):
    args = F.DeviceShareArgs(scoring_strategy=c.get("strategy") or "LeastAllocated")
    cfg = F.build_config(profile=PROFILE, deviceshare=args)
    dev, r = TG.node_device(c["node"]), TG.node_rsv(c["slot"])
    pod = TG.case_pod(c)
    pod["reservation_owner_mask"] = 1
    if required:
        pod["reservation_flags"] |= abi.POD_RSV_AFFINITY
    e = Engine(cfg, 1)
    e.upsert_nodes(F.make_node({"cpu": "64", "memory": str(256 << 30)}))
    e.update_metrics(np.zeros(1, dtype=abi.METRIC_DTYPE), 0)
    e.upsert_devices(dev)
    e.upsert_reservations(r)
    return e, dev, r, pod


@pytest.mark.parametrize("c", TG._cases(("rsv_filter",)), ids=TG._id)
def test_rsv_filter_device(c):
    e, _, _, pod = engine_case(c)
    with e:
        ev = e.evaluate_reservation(pod)
    assert bool(ev["pass"][0]) == c["want_filter"], c["source"]


@pytest.mark.parametrize("c", TG._cases(("rsv_filter_reservation",)), ids=TG._id)
def test_rsv_filter_reservation_device(c):
    """FilterReservation: the pod is nominated into the GPU-holding reservation exactly when DeviceShare can allocate
    from it (a device pod never nominates one it cannot)."""
    from oracle import oracle
    e, dev, r, pod = engine_case(c)
    with e:
        ev = e.evaluate_reservation(pod)
    # the node-level Filter (the reference test calls FilterReservation alone): device = oracle; an exhausted
    # reservation on a node with nothing else free fails both
    st = oracle.ds_rsv_init(r, matched=[0])
    assert bool(ev["pass"][0]) == oracle.ds_filter_rsv(dev, pod, r, st, False), c["source"]
    if ev["pass"][0]:
        assert (ev["nominated"][0] == 0) == c["want_filter"], c["source"]
    else:
        assert not c["want_filter"], c["source"]


@pytest.mark.parametrize("c", TG._cases(("rsv_score",)), ids=TG._id)
def test_rsv_score_device(c):
    """scoreWithReservation of the nominated reservation is the node's raw DeviceShare Score."""
    e, _, _, pod = engine_case(c)
    with e:
        ev = e.evaluate_reservation(pod)
    assert ev["pass"][0] == 1 and ev["nominated"][0] == 0, c["source"]
    assert int(ev["ds_raw"][0]) == c["want_score"], c["source"]


@pytest.mark.parametrize("c", TG._cases(("rsv_reserve",)), ids=TG._id)
def test_rsv_reserve_device(c):
    e, dev, _, pod = engine_case(c)
    with e:
        e.stage(pod)
        e.schedule_staged(0, 1)
        node, _ = e.fetch(0, 1)
        mask = int(e.fetch_devices(0, 1)[0])
        uc, um, _ = e.read_devices()
    assert node[0] == 0 and mask == TG._mask(c["want_minors"]), c["source"]
    inst = c["want_instance"]
    for m in c["want_minors"]:
        assert uc[0, m] - dev[0]["used_core"][m] == inst["core"], c["source"]
        assert um[0, m] - dev[0]["used_memory"][m] == inst["memory"], c["source"]


@pytest.mark.parametrize("c", TG._cases(("rsv_try",)), ids=TG._id)
def test_rsv_try_device(c):
    """tryAllocateFromReservation: a pod requiring the reservation is Unschedulable exactly when the try fails; a pod
    placed through the reservation gets the minors the reference's allocator (with its scorer, as Reserve runs it)
    picks — the oracle's scored try — which is the table's answer where the table's scorer-less allocator agrees."""
    from oracle import oracle
    e, dev, r, pod = engine_case(c, required=c["required"])
    cfg = TG.case_config(c)
    st = oracle.ds_rsv_init(r, matched=[0] if c["slot"] else [])
    slots = list(st[0]["matched"][:st[0]["n_matched"]])
    s_scored, m_scored = oracle.ds_try_rsv(cfg[0], dev.copy(), pod, r, st, slots, scored=True)
    _, m_plain = oracle.ds_try_rsv(cfg[0], dev.copy(), pod, r, st, slots, scored=False)
    with e:
        ev = e.evaluate_reservation(pod)
        if c["required"] and c["slot"]:
            assert (ev["pass"][0] == 0) == c["want_unschedulable"], c["source"]
        if ev["pass"][0] and ev["nominated"][0] == 0:
            e.stage(pod)
            e.schedule_staged(0, 1)
            mask = int(e.fetch_devices(0, 1)[0])
            assert s_scored == 0 and mask == m_scored, c["source"]
            if m_scored == m_plain:
                assert mask == TG._mask(c["want_minors"]), c["source"]
