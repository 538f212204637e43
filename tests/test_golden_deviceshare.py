"""DeviceShare oracle (oracle/deviceshare.c) against the golden vectors transcribed from the reference's own tests
(tests/golden/deviceshare.json, made by tests/golden/make_golden_ds.py; each case cites its source line), plus
scheduling-loop properties of the oracle's DeviceShare profile (NormalizeScore, Reserve bookkeeping).  CPU only."""
import json
import os

import numpy as np
import pytest

from koordinator_amd import abi, framework, synth
from oracle import oracle

F = framework
HERE = os.path.dirname(os.path.abspath(__file__))
DS_PROFILE = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.DEVICE_SHARE),
                       score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.DEVICE_SHARE: 1})


def _cases(kind=None):
    with open(os.path.join(HERE, "golden", "deviceshare.json")) as f:
        cases = json.load(f)["cases"]
    return [c for c in cases if kind is None or c["kind"] in kind]


def _id(c):
    return c["name"]


def node_device(spec) -> np.ndarray:
    gpus = [{"minor": g["minor"], "healthy": g["healthy"], "total": g["total"], "used": g["used"]}
            for g in spec["gpus"]]
    return F.make_node_device(gpus, has_device=spec["has_device"])


def case_config(c):
    args = F.DeviceShareArgs(scoring_strategy=c.get("strategy") or "LeastAllocated")
    return F.build_config(profile=DS_PROFILE, deviceshare=args)


def case_pod(c):
    return F.make_pod({"cpu": "1", "memory": "1Gi"}, devices=c["pod"])


@pytest.mark.parametrize("c", _cases(("score",)), ids=_id)
def test_golden_score(c):
    cfg = case_config(c)
    dev, pod = node_device(c["node"]), case_pod(c)
    assert oracle.ds_filter(dev, pod) == c["want_filter"], c["source"]
    if c["want_filter"]:
        assert oracle.ds_score(cfg[0], dev, pod) == c["want_score"], c["source"]


@pytest.mark.parametrize("c", _cases(("filter",)), ids=_id)
def test_golden_filter(c):
    dev, pod = node_device(c["node"]), case_pod(c)
    assert oracle.ds_filter(dev, pod) == c["want_filter"], c["source"]


@pytest.mark.parametrize("c", _cases(("reserve",)), ids=_id)
def test_golden_reserve(c):
    cfg = case_config(c)
    if not c.get("strategy"):  # the test runs the allocator without a scorer: every minor scores 0
        cfg[0]["ds_scoring_weights"] = 0
    dev, pod = node_device(c["node"]), case_pod(c)
    before = dev.copy()
    mask = oracle.ds_reserve(cfg[0], dev, pod)
    assert mask == sum(1 << m for m in c["want_minors"]), c["source"]
    inst = c["want_instance"]
    for m in range(abi.MAX_MINORS):
        k = 1 if m in c["want_minors"] else 0
        assert dev[0]["used_core"][m] - before[0]["used_core"][m] == k * inst["core"], c["source"]
        assert dev[0]["used_ratio"][m] - before[0]["used_ratio"][m] == k * inst["ratio"], c["source"]
        assert dev[0]["used_memory"][m] - before[0]["used_memory"][m] == k * inst["memory"], c["source"]


@pytest.mark.parametrize("c", _cases(("instance",)), ids=_id)
def test_golden_instance(c):
    got = oracle.ds_instance(node_device(c["node"]), case_pod(c))
    if c["want"] is None:
        assert got is None, c["source"]
    else:
        w = c["want"]
        assert got == (w["count"], w["core"], w["memory"], w["ratio"]), c["source"]


@pytest.mark.parametrize("c", _cases(("ratio_to_bytes", "bytes_to_ratio")), ids=_id)
def test_golden_memory_conversion(c):
    L = oracle.lib()
    if c["kind"] == "ratio_to_bytes":
        assert L.or_ds_memory_ratio_to_bytes(c["ratio"], c["total"]) == c["want"], c["source"]
    else:
        assert L.or_ds_memory_bytes_to_ratio(c["bytes"], c["total"]) == c["want"], c["source"]


@pytest.mark.parametrize("c", _cases(("validate",)), ids=_id)
def test_golden_validate(c):
    d = oracle.ds_pod(case_pod(c))[0]
    assert bool(d["error"]) == c["want_error"], c["source"]
    if not c["want_error"]:
        w = c["want_request"]
        assert (int(d["core"]), int(d["mem"]), int(d["ratio"])) == (w.get("core", 0), w.get("memory", 0),
                                                                    w.get("ratio", 0)), c["source"]
        assert bool(d["has_mem"]) == ("memory" in w), c["source"]


def test_multi_gpu_request_splits_per_instance():
    """ratio 200 → 2 instances of {core/2, mem/2, ratio/2} (devicehandler_gpu.go:53-63); one free GPU fails."""
    gi = 1 << 30
    one = F.make_node_device([{"minor": 0, "total": {"core": 100, "ratio": 100, "memory": 80 * gi}}])
    two = F.make_node_device([{"minor": m, "total": {"core": 100, "ratio": 100, "memory": 80 * gi}} for m in (0, 1)])
    pod = F.make_pod({"cpu": "1"}, devices={"koordinator.sh/gpu-core": 200, "koordinator.sh/gpu-memory-ratio": 200})
    assert oracle.ds_instance(two, pod) == (2, 100, 80 * gi, 100)
    assert not oracle.ds_filter(one, pod)
    assert oracle.ds_filter(two, pod)
    cfg = F.build_config(profile=DS_PROFILE)
    assert oracle.ds_reserve(cfg[0], two, pod) == 0b11
    assert list(two[0]["used_ratio"][:2]) == [100, 100]


def test_schedule_normalizes_deviceshare_over_feasible_nodes():
    """NormalizeScore: the DeviceShare term of every feasible node is 100·raw/max(raw) (weight 1)."""
    cluster, dev = synth.make_gpu_cluster(300, seed=11)
    pods = synth.make_gpu_pods(400, seed=12)
    cfg = F.build_config(profile=DS_PROFILE)
    st = oracle.states(cluster.n)
    oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
    d = dev.copy()
    node, score, _, minors = oracle.schedule_full(cfg, cluster.nodes, cluster.metrics, st, pods, cluster.now_ns,
                                                  devices=d)
    gpu = pods["device_requests"].any(axis=1)
    assert (node >= 0).mean() > 0.9
    assert np.all(minors[(node >= 0) & ~gpu] == 0)
    assert np.all(minors[(node >= 0) & gpu] != 0)
    # every allocated minor got exactly the pods' per-instance requests
    added = d["used_ratio"].sum() - dev["used_ratio"].sum()
    want = 0
    for i in np.flatnonzero((node >= 0) & gpu):
        inst = oracle.ds_instance(dev[node[i]:node[i] + 1], pods[i])
        want += inst[0] * inst[3]
    assert added == want
    # the same queue without DeviceShare in the profile places the non-GPU pods differently somewhere
    assert score.max() <= 300


def test_oracle_threads_agree():
    cluster, dev = synth.make_gpu_cluster(500, seed=21)
    pods = synth.make_gpu_pods(300, seed=22)
    cfg = F.build_config(profile=DS_PROFILE)
    outs = []
    for th in (1, 4):
        st = oracle.states(cluster.n)
        oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
        d = dev.copy()
        outs.append(oracle.schedule_full(cfg, cluster.nodes, cluster.metrics, st, pods, cluster.now_ns, th,
                                         devices=d) + (d,))
    for a, b in zip(outs[0], outs[1]):
        assert np.array_equal(a, b)


# ---- (ABI 13) reservations holding GPUs ----
def node_rsv(sl) -> np.ndarray:
    """One node's kg_node_reservations with the case's slot in slot 0 (cpu / memory allocatable so the Reservation
    plugin's resource-name intersection holds for the case pod)."""
    r = np.zeros(1, dtype=abi.NODE_RSV_DTYPE)
    if sl is None:
        return r
    r["n"] = 1
    r["allocatable_cpu"][0, 0], r["allocatable_mem"][0, 0] = 4000, 8 << 30
    r["available"][0, 0] = 1
    r["policy"][0, 0] = abi.RSV_POLICY[sl["policy"]]
    for key, field in (("alloc", "gpu_alloc"), ("allocated", "gpu_allocated")):
        for m, (core, ratio, mem) in sl[key].items():
            r[field][0, 0, int(m)] = (core, mem, ratio)
    r["gpu_minors"][0, 0] = sum(1 << int(m) for m in sl["alloc"])
    return r


def _mask(minors):
    return None if minors is None else sum(1 << m for m in minors)


@pytest.mark.parametrize("c", _cases(("rsv_restore",)), ids=_id)
def test_golden_rsv_restore(c):
    r = node_rsv(c["slot"])
    st = oracle.ds_rsv_init(r, matched=[0])[0]
    assert st["n_matched"] == 1 and st["matched"][0] == 0, c["source"]
    w = c["want"]
    for key, field in (("mat_alloc", "mat_alloc"), ("mat_allocd", "mat_allocd")):
        want = np.zeros((abi.MAX_MINORS, 3), dtype=np.int64)
        for m, (core, ratio, mem) in w[key].items():
            want[int(m)] = (core, mem, ratio)
        assert np.array_equal(st[field], want), (c["source"], key)
    for m, (core, ratio, mem) in w["remained"].items():  # remained = allocatable − allocated, non-negative
        got = np.maximum(r["gpu_alloc"][0, 0, int(m)] - r["gpu_allocated"][0, 0, int(m)], 0)
        assert tuple(got) == (core, mem, ratio), c["source"]


@pytest.mark.parametrize("c", _cases(("rsv_try",)), ids=_id)
def test_golden_rsv_try(c):
    cfg = case_config(c)
    dev, pod, r = node_device(c["node"]), case_pod(c), node_rsv(c["slot"])
    st = oracle.ds_rsv_init(r, matched=[0] if c["slot"] else [])
    slots = list(st[0]["matched"][:st[0]["n_matched"]])
    s, mask = oracle.ds_try_rsv(cfg[0], dev, pod, r, st, slots, scored=False)  # the test's allocator has no scorer
    assert (mask if s >= 0 else None) == _mask(c["want_minors"]), c["source"]
    assert (s < 0 and c["required"] and bool(slots)) == c["want_unschedulable"], c["source"]
    if c["slot"] and c["required"]:  # Filter with requiredFromReservation passes exactly when the try does
        assert oracle.ds_filter_rsv(dev, pod, r, st, True) == (s >= 0), c["source"]


@pytest.mark.parametrize("c", _cases(("rsv_filter",)), ids=_id)
def test_golden_rsv_filter(c):
    dev, pod, r = node_device(c["node"]), case_pod(c), node_rsv(c["slot"])
    st = oracle.ds_rsv_init(r, matched=[0])
    assert oracle.ds_filter_rsv(dev, pod, r, st, False) == c["want_filter"], c["source"]


@pytest.mark.parametrize("c", _cases(("rsv_filter_reservation",)), ids=_id)
def test_golden_rsv_filter_reservation(c):
    dev, pod, r = node_device(c["node"]), case_pod(c), node_rsv(c["slot"])
    st = oracle.ds_rsv_init(r, matched=[0])
    L = oracle.lib()
    rr = np.ascontiguousarray(r)
    got = L.or_ds_filter_reservation(oracle.p(np.ascontiguousarray(dev)), oracle.p(oracle.ds_pod(pod)), oracle.p(rr),
                                     oracle.p(st), 0)
    assert bool(got) == c["want_filter"], c["source"]


@pytest.mark.parametrize("c", _cases(("rsv_reserve",)), ids=_id)
def test_golden_rsv_reserve(c):
    cfg = case_config(c)
    dev, pod, r = node_device(c["node"]), case_pod(c), node_rsv(c["slot"])
    st = oracle.ds_rsv_init(r, matched=[0])
    before = dev.copy()
    mask = oracle.ds_reserve_rsv(cfg[0], dev, pod, r, st, 0)
    assert mask == _mask(c["want_minors"]), c["source"]
    inst = c["want_instance"]
    for m in c["want_minors"]:
        assert dev[0]["used_core"][m] - before[0]["used_core"][m] == inst["core"], c["source"]
        assert dev[0]["used_memory"][m] - before[0]["used_memory"][m] == inst["memory"], c["source"]


@pytest.mark.parametrize("c", _cases(("rsv_score",)), ids=_id)
def test_golden_rsv_score(c):
    cfg = case_config(c)
    dev, pod, r = node_device(c["node"]), case_pod(c), node_rsv(c["slot"])
    st = oracle.ds_rsv_init(r, matched=[0])
    assert oracle.ds_score_slot(cfg[0], dev, pod, r, st, 0) == c["want_score"], c["source"]
