"""(ABI 13) DeviceShare with reservations that hold GPUs (deviceshare/reservation.go, plugin.go:280-455; SURVEY §8a
rows A20/A22 together): the C5 variant where 30 % of the reservations on GPU nodes also hold GPU shares.

The golden vectors of the reference's own tables (Test_tryAllocateFromReservation, Test_Plugin_Filter "allocate from
reserved", Test_Plugin_FilterReservation, Test_Plugin_Reserve "reserve from reservation", TestScoreReservation) pin
the oracle in tests/test_golden_deviceshare.py.  Here: CPU — the oracle's scheduling loop with GPU reservations
(device pods nominate them, the slots' gpu_allocated follows Reserve / Unreserve exactly); GPU — the engine through
the C ABI against it, bit-exact: placement, weighted total, slot, minor mask, the DeviceShare used table, the
reservations' Allocated / assigned and their gpu_allocated, also with Unreserve interleaved."""
import numpy as np
import pytest

from koordinator_amd import Engine, abi, framework as F, synth
from oracle import oracle

PROFILE = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.RESERVATION, F.DEVICE_SHARE),
                    score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.RESERVATION: 5000, F.DEVICE_SHARE: 1})


def workload(n_nodes, n_pods, seed, frac=0.3, quotas=True):
    cluster, dev, rsv = synth.make_c5_cluster(n_nodes, seed=seed, gpu_rsv_frac=frac)
    pods = synth.make_c5_pods(n_pods, seed=seed + 50)
    q = synth.make_c5_quotas(pods, seed=seed + 60) if quotas else None
    if not quotas:
        pods["quota_id"] = 0
    return cluster, dev, rsv, pods, q


def oracle_run(cfg, cluster, dev, rsv, pods, quotas, n_threads=8):
    st = oracle.states(cluster.n)
    oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
    r, d, q = rsv.copy(), dev.copy(), None if quotas is None else quotas.copy()
    node, score, slot, minors = oracle.schedule_resv(cfg, cluster.nodes, cluster.metrics, st, r, pods, cluster.now_ns,
                                                     devices=d, quotas=q, n_threads=n_threads, with_minors=True)
    return dict(node=node, score=score, slot=slot, minors=minors, st=st, rsv=r, dev=d, quotas=q)


def _gpu_slot(w, rsv):
    """pods assumed into a GPU-holding slot"""
    s = w["slot"]
    node = np.maximum(w["node"], 0)
    return (s >= 0) & (rsv["gpu_minors"][node, np.maximum(s, 0)] != 0)


# ---- CPU: the oracle ---------------------------------------------------------------------------------------------
def test_oracle_device_pods_use_gpu_reservations():
    cluster, dev, rsv, pods, quotas = workload(400, 1600, 11)
    w = oracle_run(F.build_config(profile=PROFILE), cluster, dev, rsv, pods, quotas)
    device_pod = pods["device_requests"].any(axis=1)
    g = _gpu_slot(w, rsv)
    assert (g & device_pod).sum() > 5           # device pods nominate GPU reservations now
    assert not (device_pod & (w["slot"] >= 0) & ~g).any()  # never a cpu/mem-only one (FilterReservation)
    # each such pod's allocation on the reservation's minors is in the slot's gpu_allocated
    want = rsv["gpu_allocated"].copy()
    for j in np.nonzero(g & device_pod)[0]:
        i, s = w["node"][j], w["slot"][j]
        inst = oracle.ds_instance(dev[i:i + 1], pods[j])
        for m in range(abi.MAX_MINORS):
            if (w["minors"][j] >> m) & 1 and (rsv["gpu_minors"][i, s] >> m) & 1:
                want[i, s, m] += (inst[1], inst[2], inst[3])
    assert np.array_equal(w["rsv"]["gpu_allocated"], want)


def test_oracle_gpu_reservations_change_decisions():
    """The same queue with the GPU holdings dropped (the reservations cpu/mem-only, the node usage unchanged) places
    device pods differently: the restore returns the reservations' GPUs to the pods that match them."""
    cluster, dev, rsv, pods, _ = workload(300, 1200, 12, quotas=False)
    cfg = F.build_config(profile=PROFILE)
    a = oracle_run(cfg, cluster, dev, rsv, pods, None)
    r0 = rsv.copy()
    r0["gpu_minors"] = 0
    r0["gpu_alloc"] = 0
    r0["gpu_allocated"] = 0
    b = oracle_run(cfg, cluster, dev, r0, pods, None)
    assert not (np.array_equal(a["node"], b["node"]) and np.array_equal(a["minors"], b["minors"]))


def test_oracle_threads_agree():
    cluster, dev, rsv, pods, quotas = workload(300, 900, 13)
    cfg = F.build_config(profile=PROFILE)
    a = oracle_run(cfg, cluster, dev, rsv, pods, quotas, n_threads=1)
    b = oracle_run(cfg, cluster, dev, rsv, pods, quotas, n_threads=8)
    for k in ("node", "score", "slot", "minors"):
        assert np.array_equal(a[k], b[k]), k
    assert np.array_equal(a["rsv"]["gpu_allocated"], b["rsv"]["gpu_allocated"])


def test_oracle_unreserve_restores_gpu_allocated():
    cfg = F.build_config(profile=PROFILE)
    cluster, dev, rsv, pods, quotas = workload(200, 900, 14)
    w = oracle_run(cfg, cluster, dev, rsv, pods, quotas)
    assert _gpu_slot(w, rsv).any()
    st, d, r, q = w["st"], w["dev"], w["rsv"], w["quotas"]
    for j in np.nonzero(w["node"] >= 0)[0][::-1]:
        oracle.unreserve(cfg, st, pods[j], w["node"][j], devices=d, rsv=r, quotas=q, minors=w["minors"][j],
                         slot=w["slot"][j])
    assert np.array_equal(r["gpu_allocated"], rsv["gpu_allocated"])
    for k in ("used_core", "used_memory", "used_ratio"):
        assert np.array_equal(d[k], dev[k]), k


# ---- GPU: the engine against the oracle -------------------------------------------------------------------------
def engine_run(cfg, cluster, dev, rsv, pods, quotas, chunks=1):
    with Engine(cfg, cluster.n) as e:
        synth.load_c5_into(e, cluster, dev, rsv, quotas)
        e.stage(pods)
        bounds = np.linspace(0, len(pods), chunks + 1).astype(int)
        for a, b in zip(bounds[:-1], bounds[1:]):
            e.schedule_staged(int(a), int(b - a))
        node, score = e.fetch(0, len(pods))
        return dict(node=node, score=score, slot=e.fetch_reservations(0, len(pods)),
                    minors=e.fetch_devices(0, len(pods)), state=e.read_state(), rsv=e.read_reservations(),
                    gpu=e.read_reservation_gpus(), dev=e.read_devices(),
                    quotas=None if quotas is None else e.read_quotas(len(quotas)))


def check(cfg, cluster, dev, rsv, pods, quotas, chunks=1):
    w = oracle_run(cfg, cluster, dev, rsv, pods, quotas)
    g = engine_run(cfg, cluster, dev, rsv, pods, quotas, chunks)
    bad = np.nonzero((g["node"] != w["node"]) | (g["score"] != w["score"]) | (g["slot"] != w["slot"]) |
                     (g["minors"] != w["minors"]))[0]
    assert len(bad) == 0, f"first mismatch at pod {bad[0]}: gpu " \
        f"{[int(g[k][bad[0]]) for k in ('node', 'score', 'slot', 'minors')]} oracle " \
        f"{[int(w[k][bad[0]]) for k in ('node', 'score', 'slot', 'minors')]}"
    r = w["rsv"]
    on = np.arange(abi.MAX_RSV_SLOTS)[None, :] < r["n"][:, None]
    ac, am, asg = g["rsv"]
    assert np.array_equal(ac, np.where(on, r["allocated_cpu"], 0))
    assert np.array_equal(am, np.where(on, r["allocated_mem"], 0))
    assert np.array_equal(asg, np.where(on, r["assigned"], 0))
    want_gpu = np.where((r["gpu_minors"] != 0)[:, :, None, None], r["gpu_allocated"], 0)
    assert np.array_equal(g["gpu"], want_gpu)
    uc, um, ur = g["dev"]
    assert np.array_equal(uc, w["dev"]["used_core"]) and np.array_equal(um, w["dev"]["used_memory"])
    assert np.array_equal(ur, w["dev"]["used_ratio"])
    assert np.array_equal(g["state"]["requested_cpu"], w["st"]["requested"][:, abi.RES_CPU])
    if quotas is not None:
        assert np.array_equal(g["quotas"], w["quotas"])
    return w


@pytest.mark.gpu
@pytest.mark.parametrize("n_nodes,n_pods,seed,chunks", [(300, 1500, 21, 2), (1000, 2500, 22, 1), (257, 1200, 23, 3)])
def test_gpu_reservation_parity(n_nodes, n_pods, seed, chunks):
    cluster, dev, rsv, pods, quotas = workload(n_nodes, n_pods, seed)
    w = check(F.build_config(profile=PROFILE), cluster, dev, rsv, pods, quotas, chunks)
    assert _gpu_slot(w, rsv).sum() > 3


@pytest.mark.gpu
def test_gpu_reservation_parity_filter_only_and_most_allocated():
    cluster, dev, rsv, pods, _ = workload(500, 1200, 31, quotas=False)
    fo = F.Profile(filter=PROFILE.filter, score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1})
    check(F.build_config(profile=fo), cluster, dev, rsv, pods, None)
    cfg = F.build_config(profile=PROFILE, deviceshare=F.DeviceShareArgs(scoring_strategy="MostAllocated"))
    check(cfg, cluster, dev, rsv, pods, None)


@pytest.mark.gpu
def test_gpu_reservation_parity_50k_nodes():
    """The C5 variant at its configuration size: 50k nodes, 30 % of the GPU nodes' reservations holding GPUs."""
    cluster, dev, rsv, pods, quotas = workload(50_000, 3000, 41)
    w = check(F.build_config(profile=PROFILE), cluster, dev, rsv, pods, quotas, chunks=2)
    assert _gpu_slot(w, rsv).sum() > 10


@pytest.mark.gpu
def test_gpu_reservation_unreserve_interleaved():
    cfg = F.build_config(profile=PROFILE)
    cluster, dev, rsv, pods, quotas = workload(600, 2400, 51)
    st = oracle.states(cluster.n)
    oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
    d, r, q = dev.copy(), rsv.copy(), quotas.copy()
    a = 1200
    w1, _, s1, m1 = oracle.schedule_resv(cfg, cluster.nodes, cluster.metrics, st, r, pods[:a], cluster.now_ns,
                                         devices=d, quotas=q, n_threads=8, with_minors=True)
    placed = np.nonzero(w1 >= 0)[0]
    m = np.zeros(a, dtype=bool)
    m[placed[::2]] = True
    for j in np.nonzero(m)[0]:
        oracle.unreserve(cfg, st, pods[j], w1[j], devices=d, rsv=r, quotas=q, minors=m1[j], slot=s1[j])
    gs = (s1 >= 0) & (rsv["gpu_minors"][np.maximum(w1, 0), np.maximum(s1, 0)] != 0)
    assert (m & gs & (m1 != 0)).any()
    mid_gpu = np.where((r["gpu_minors"] != 0)[:, :, None, None], r["gpu_allocated"], 0)  # after the Unreserve
    w2, ws2, s2, m2 = oracle.schedule_resv(cfg, cluster.nodes, cluster.metrics, st, r, pods[a:], cluster.now_ns,
                                           devices=d, quotas=q, n_threads=8, with_minors=True)
    with Engine(cfg, cluster.n) as e:
        synth.load_c5_into(e, cluster, dev, rsv, quotas)
        e.stage(pods)
        e.schedule_staged(0, a)
        g1, _ = e.fetch(0, a)
        assert np.array_equal(g1, w1) and np.array_equal(e.fetch_devices(0, a), m1)
        e.unreserve(0, a, m)
        assert np.array_equal(e.read_reservation_gpus(), mid_gpu)
        e.schedule_staged(a, len(pods) - a)
        g2, gs2 = e.fetch(a, len(pods) - a)
        assert np.array_equal(g2, w2) and np.array_equal(gs2, ws2)
        assert np.array_equal(e.fetch_reservations(a, len(pods) - a), s2)
        assert np.array_equal(e.fetch_devices(a, len(pods) - a), m2)
        assert np.array_equal(e.read_reservation_gpus(),
                              np.where((r["gpu_minors"] != 0)[:, :, None, None], r["gpu_allocated"], 0))
        uc, um, ur = e.read_devices()
        assert np.array_equal(uc, d["used_core"]) and np.array_equal(ur, d["used_ratio"])


@pytest.mark.gpu
def test_gpu_holdings_validated_at_upsert():
    cfg = F.build_config(profile=PROFILE)
    cluster, dev, rsv, pods, _ = workload(50, 10, 61, quotas=False)
    with Engine(cfg, cluster.n) as e:
        synth.load_c5_into(e, cluster, dev, rsv, None)
        bad = rsv[:1].copy()
        bad["n"] = 1
        bad["gpu_minors"][0, 0] = 1 << abi.MAX_MINORS
        with pytest.raises(abi.KoordGPUError):
            e.upsert_reservations(bad, idx=np.array([0], dtype=np.int32))
        bad["gpu_minors"][0, 0] = 1
        bad["gpu_alloc"][0, 0, 0] = (-1, 0, 0)
        with pytest.raises(abi.KoordGPUError):
            e.upsert_reservations(bad, idx=np.array([0], dtype=np.int32))


@pytest.mark.gpu
def test_read_reservation_gpus_zero_after_reupsert_without_gpus():
    """ Re-upserting a node whose reservations no longer hold GPUs zeroes its rows: the read-back is zero
    there; a profile without Reservation refuses the read (KG_E_INVALID, as koordgpu.h documents)."""
    cfg = F.build_config(profile=PROFILE)
    cluster, dev, rsv, pods, _ = workload(60, 10, 62, frac=1.0, quotas=False)
    held = np.flatnonzero((rsv["gpu_minors"] != 0).any(axis=1))
    assert held.size > 0
    with Engine(cfg, cluster.n) as e:
        synth.load_c5_into(e, cluster, dev, rsv, None)
        before = e.read_reservation_gpus()
        i = int(held[0])
        assert before[i].any() or not rsv["gpu_allocated"][i].any()
        row = rsv[i:i + 1].copy()
        row["gpu_minors"] = 0
        row["gpu_alloc"] = 0
        row["gpu_allocated"] = 0
        e.upsert_reservations(row, idx=np.array([i], dtype=np.int32))
        after = e.read_reservation_gpus()
        assert not after[i].any()
        others = np.arange(cluster.n) != i
        assert np.array_equal(after[others], before[others])
    no_rsv = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.DEVICE_SHARE), score={F.NODE_RESOURCES_FIT: 1})
    with Engine(F.build_config(profile=no_rsv), cluster.n) as e:
        with pytest.raises(abi.KoordGPUError):
            e.read_reservation_gpus()
