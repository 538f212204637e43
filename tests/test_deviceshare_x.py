"""(r6, ABI 17) DeviceShare's RDMA / FPGA device types (deviceshare/devicehandler_default.go, allocated alongside the GPU
type by device_allocator.go:92-129, 333-454; scored per type and summed, :499-522).

Pinned by the reference's own tables (tests/golden/deviceshare_x.json, tests/golden/make_golden_ds_x.py):
Test_Plugin_Filter's FPGA rows (plugin_test.go:985-1360), Test_Plugin_Reserve's RDMA / FPGA rows (:2283-2723), TestScore
"requested multiple resources" (scoring_test.go:274-351) and Test_allocateRDMA (device_allocator_test.go:2259-2340, the
preemptible RDMA minors, rebuilt as a preemption victim holding them) — on the oracle (CPU) and through the C ABI
(GPU).  Device vs oracle on random DeviceShare clusters with RDMA / FPGA devices: placements, totals, the packed minors
(GPU bits 0-7, RDMA 8-15, FPGA 16-23) and every node's deviceUsed, with Unreserve interleaved."""
import json
import os

import numpy as np
import pytest

from koordinator_amd import Engine, abi, framework as F, synth
from oracle import oracle

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "deviceshare_x.json")) as fh:
    CASES = json.load(fh)["cases"]
DS = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.DEVICE_SHARE), score={F.NODE_RESOURCES_FIT: 1, F.DEVICE_SHARE: 1})
C5 = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.RESERVATION, F.DEVICE_SHARE),
               score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.RESERVATION: 5000, F.DEVICE_SHARE: 1})
TYPES = ("gpu", "rdma", "fpga")


def _cases(kind):
    return [c for c in CASES if c["kind"] == kind]


def _id(c):
    return c["name"]


def node_dev(spec):
    return F.make_node_device(spec.get("gpus", []), rdma=spec.get("rdma"), fpga=spec.get("fpga"))


def pod_of(req):
    return F.make_pod({"cpu": "1"}, devices=req)


def pack(minors):
    out = 0
    for k, t in enumerate(TYPES):
        for m in (minors or {}).get(t, []):
            out |= 1 << (8 * k + m)
    return out


def unpack(v, t):
    return (v >> (8 * TYPES.index(t))) & 0xFF


# ---- oracle ------------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("c", _cases("filter"), ids=_id)
def test_oracle_filter(c):
    assert oracle.ds_filter(node_dev(c["node"]), pod_of(c["pod"])) == c["want_filter"], c["source"]


@pytest.mark.parametrize("c", _cases("reserve"), ids=_id)
def test_oracle_reserve(c):
    cfg = F.build_config(profile=DS)
    dev = node_dev(c["node"])
    before = dev.copy()
    got = oracle.ds_reserve(cfg[0], dev, pod_of(c["pod"]))
    if c["want_minors"] is None:
        assert got == -1, c["source"]
        assert np.array_equal(dev, before), c["source"]  # nothing allocated
        return
    assert got == pack(c["want_minors"]), c["source"]
    inst = c["want_instance"]
    for t in ("rdma", "fpga"):
        k = abi.XTYPE_RDMA if t == "rdma" else abi.XTYPE_FPGA
        for m in range(abi.MAX_MINORS):
            want = inst[t] if m in c["want_minors"][t] else 0
            assert dev[0]["x_used"][k, m] - before[0]["x_used"][k, m] == want, c["source"]


@pytest.mark.parametrize("c", _cases("score"), ids=_id)
def test_oracle_score(c):
    cfg = F.build_config(profile=DS)
    dev, pod = node_dev(c["node"]), pod_of(c["pod"])
    assert oracle.ds_filter(dev, pod)
    assert oracle.ds_score(cfg[0], dev, pod) == c["want_score"], c["source"]


def _preempt_world(c):
    node = F.make_node({"cpu": "32", "memory": "64Gi"}, allowed_pods=100)
    vic = pod_of(c["victim"])
    cl = synth.Cluster(node, F.make_node_metric(present=False, node_usage=None), vic, np.zeros(1, np.int32), 10**18)
    return cl, node_dev(c["node"]), vic, np.array([pack(c["victim_minors"])], np.int32)


@pytest.mark.parametrize("c", _cases("preempt"), ids=_id)
def test_oracle_preemptible(c):
    """The victim's RDMA minors become preemptibleDevices in the dry run; once it has left, Reserve takes minor 1."""
    cfg = F.build_config(profile=DS)
    cl, dev, vic, mins = _preempt_world(c)
    st = oracle.states(1)
    oracle.add_pods(cfg, st, cl.existing_pods, cl.existing_node)
    pod = pod_of(c["pod"])
    args = (cfg, cl.nodes[0], cl.metrics[0], st[:1], None, pod)
    assert (oracle.filter_preemption(*args, vic[:0], None, cl.now_ns, dev=dev[0], minors=mins[:0]) == 0) == \
        c["want_filter_without"]
    assert (oracle.filter_preemption(*args, vic, None, cl.now_ns, dev=dev[0], minors=mins) == 0) == c["want_filter_with"]
    freed = dev.copy()
    freed["x_used"] = 0
    assert oracle.ds_reserve(cfg[0], freed, pod) == pack(c["want_minors"]), c["source"]


def test_oracle_invalid_and_absent():
    cfg = F.build_config(profile=DS)
    dev = node_dev({"rdma": [{"minor": 0, "total": 100, "used": 0}]})
    assert not oracle.ds_filter(dev, pod_of({"koordinator.sh/rdma": 150}))   # ValidatePercentageResource
    assert not oracle.ds_filter(dev, pod_of({"koordinator.sh/fpga": 50}))    # no FPGA listed: Insufficient
    assert oracle.ds_filter(dev, pod_of({"koordinator.sh/rdma": 100}))
    unhealthy = dev.copy()
    unhealthy["x_healthy"] = 0                                               # an empty ResourceList
    assert not oracle.ds_filter(unhealthy, pod_of({"koordinator.sh/rdma": 25}))
    nodev = F.make_node_device([], has_device=False)
    assert not oracle.ds_filter(nodev, pod_of({"koordinator.sh/rdma": 25}))
    assert oracle.ds_score(cfg[0], dev, pod_of({"koordinator.sh/rdma": 25})) == 75  # (100 − 25) · 100 / 100


# ---- device ------------------------------------------------------------------------------------------------------
def _engine(profile, dev, n=1):
    e = Engine(F.build_config(profile=profile), n)
    e.upsert_nodes(np.concatenate([F.make_node({"cpu": "64", "memory": str(256 << 30)}) for _ in range(n)]))
    e.update_metrics(np.zeros(n, dtype=abi.METRIC_DTYPE), 0)
    e.upsert_devices(dev)
    return e


@pytest.mark.gpu
@pytest.mark.parametrize("c", _cases("filter") + _cases("score"), ids=_id)
def test_device_filter_score(c):
    dev, pod = node_dev(c["node"]), pod_of(c["pod"])
    with _engine(DS, dev) as e:
        ok, sc = e.evaluate_device(pod)
    want = c.get("want_filter", True)
    assert bool(ok[0]) == want, c["source"]
    if "want_score" in c:
        assert int(sc[0]) == c["want_score"], c["source"]


@pytest.mark.gpu
@pytest.mark.parametrize("profile", [DS, C5], ids=["ds", "c5"])
@pytest.mark.parametrize("c", _cases("reserve"), ids=_id)
def test_device_reserve(c, profile):
    dev = node_dev(c["node"])
    with _engine(profile, dev) as e:
        e.stage(pod_of(c["pod"]))
        e.schedule_staged(0, 1)
        node, _ = e.fetch(0, 1)
        g = int(e.fetch_devices(0, 1)[0])
        x = e.fetch_devices_x(0, 1)[0]
        xu = e.read_devices_x()
    if c["want_minors"] is None:
        assert node[0] == -1 and g == 0 and not x.any(), c["source"]
        assert np.array_equal(xu[0], dev[0]["x_used"]), c["source"]
        return
    assert node[0] == 0, c["source"]
    assert g | (int(x[0]) << 8) | (int(x[1]) << 16) == pack(c["want_minors"]), c["source"]
    for t, k in (("rdma", abi.XTYPE_RDMA), ("fpga", abi.XTYPE_FPGA)):
        for m in range(abi.MAX_MINORS):
            want = c["want_instance"][t] if m in c["want_minors"][t] else 0
            assert xu[0, k, m] - dev[0]["x_used"][k, m] == want, c["source"]


@pytest.mark.gpu
@pytest.mark.parametrize("c", _cases("preempt"), ids=_id)
def test_device_preemptible(c):
    cl, dev, vic, mins = _preempt_world(c)
    pod = pod_of(c["pod"])
    with Engine(F.build_config(profile=DS), 1) as e:
        synth.load_into(e, cl)
        e.upsert_devices(dev)
        assert (e.filter_preemption(pod, 0, vic[:0], None, mins[:0]) == 0) == c["want_filter_without"]
        assert (e.filter_preemption(pod, 0, vic, None, mins) == 0) == c["want_filter_with"]
        rej, kept, _ = e.select_victims(pod, np.zeros(1, np.int32), [vic], None, None, [mins])
        assert rej[0] == 0 and kept[0].tolist() == [True]


def _x_world(n, seed, n_pods):
    cluster, dev = synth.make_gpu_cluster(n, seed=seed)
    synth.add_x_devices(dev, frac=0.6, seed=seed + 1)
    pods = synth.make_gpu_pods(n_pods, seed=seed + 2)
    synth.add_x_requests(pods, frac=0.35, seed=seed + 3)
    return cluster, dev, pods


def _packed(e, n):
    g = e.fetch_devices(0, n).astype(np.int64)
    x = e.fetch_devices_x(0, n).astype(np.int64)
    return g | (x[:, 0] << 8) | (x[:, 1] << 16)


@pytest.mark.gpu
@pytest.mark.parametrize("profile", [DS, C5], ids=["ds-profile", "c5-profile"])
def test_device_matches_oracle_random(profile):
    """A DeviceShare cluster (8 GPUs per node) with RDMA / FPGA on 60 % of the nodes, a queue where 35 % of the pods
    request RDMA (some FPGA too), with and without GPU shares: device == oracle on placements, totals, the packed
    minors and deviceUsed of every type; then Unreserve of a third of the placed pods restores deviceUsed exactly."""
    cluster, dev, pods = _x_world(300, 7100, 600)
    cfg = F.build_config(profile=profile)
    st = oracle.states(cluster.n)
    oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
    dv = dev.copy()
    if profile is DS:
        on, sc, _, om = oracle.schedule_full(cfg, cluster.nodes, cluster.metrics, st, pods, cluster.now_ns, 4, devices=dv)
    else:
        rsv = np.zeros(cluster.n, dtype=abi.NODE_RSV_DTYPE)
        on, sc, _, om = oracle.schedule_resv(cfg, cluster.nodes, cluster.metrics, st, rsv, pods, cluster.now_ns,
                                             devices=dv, n_threads=4, with_minors=True)
    with Engine(cfg, cluster.n) as e:
        synth.load_gpu_into(e, cluster, dev)
        if profile is C5:
            e.upsert_reservations(np.zeros(cluster.n, dtype=abi.NODE_RSV_DTYPE))
        e.stage(pods)
        e.schedule_staged(0, len(pods))
        node, total = e.fetch(0, len(pods))
        packed = _packed(e, len(pods))
        uc, um, ur = e.read_devices()
        xu = e.read_devices_x()
        np.testing.assert_array_equal(node, on)
        np.testing.assert_array_equal(total, sc)
        np.testing.assert_array_equal(packed, np.asarray(om, dtype=np.int64))
        np.testing.assert_array_equal(uc, dv["used_core"])
        np.testing.assert_array_equal(um, dv["used_memory"])
        np.testing.assert_array_equal(xu, dv["x_used"])
        assert ((packed >> 8) != 0).sum() > 20 and (node >= 0).sum() > 300  # RDMA / FPGA minors were allocated
        # Unreserve a third of the placed pods: deviceUsed of every type back to the oracle's release of them
        placed = np.nonzero(node >= 0)[0][::3]
        mask = np.zeros(len(pods), dtype=np.uint8)
        mask[placed] = 1
        e.unreserve(0, len(pods), mask)
        for j in placed:
            oracle.unreserve(cfg, st, pods[j:j + 1], int(on[j]), devices=dv, minors=int(om[j]))
        np.testing.assert_array_equal(e.read_devices_x(), dv["x_used"])
        np.testing.assert_array_equal(e.read_devices()[0], dv["used_core"])
