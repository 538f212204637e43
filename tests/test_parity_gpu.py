"""GPU parity: the HIP engine (through the C ABI) against the oracle and the golden vectors.

Bar: bit-exact placements (node index, ties → lowest index) and total scores, bit-exact per-plugin scores and
filter verdicts, and bit-exact final node state (NodeInfo.Requested/NonZeroRequested/pods + LoadAware
estimates) — all integer work."""
import numpy as np
import pytest

import golden_cases as G
from koordinator_amd import Engine, abi, framework, synth
from oracle import oracle

pytestmark = pytest.mark.gpu


def _engine(cfg, cluster, capacity=None):
    e = Engine(cfg, capacity or max(cluster.n, 1))
    synth.load_into(e, cluster)
    return e


def _assert_state_equal(e, st):
    s = e.read_state()
    np.testing.assert_array_equal(s["requested_cpu"], st["requested"][:, abi.RES_CPU])
    np.testing.assert_array_equal(s["requested_mem"], st["requested"][:, abi.RES_MEMORY])
    np.testing.assert_array_equal(s["nonzero_cpu"], st["nonzero"][:, 0])
    np.testing.assert_array_equal(s["nonzero_mem"], st["nonzero"][:, 1])
    np.testing.assert_array_equal(s["num_pods"], st["num_pods"])
    np.testing.assert_array_equal(s["la_est_cpu"], st["la_est_all"][:, 0])
    np.testing.assert_array_equal(s["la_est_mem"], st["la_est_all"][:, 1])
    np.testing.assert_array_equal(s["la_est_prod_cpu"], st["la_est_prod"][:, 0])
    np.testing.assert_array_equal(s["la_est_prod_mem"], st["la_est_prod"][:, 1])


def _parity(cfg, cluster, pods, threads=4):
    on, os_, st = oracle.schedule_cluster(cfg, cluster, pods, n_threads=threads)
    with _engine(cfg, cluster) as e:
        gn, gs, stats = e.schedule(pods)
        mism = np.nonzero(gn != on)[0]
        assert mism.size == 0, f"first mismatch at pod {mism[:5]}: gpu {gn[mism[:5]]} oracle {on[mism[:5]]}"
        np.testing.assert_array_equal(gs, os_)
        _assert_state_equal(e, st)
        return gn, stats


# ---------------------------------------------------------------------------------------------------
# golden vectors through the device path (one-node clusters, kg_pods_evaluate)
# ---------------------------------------------------------------------------------------------------
def _one_node_engine(doc, case, profile):
    cfg = G.config(doc, case, profile=profile)
    e = Engine(cfg, 1)
    e.upsert_nodes(G.node(doc, case))
    e.update_metrics(G.metric(case), G.NOW_NS)
    a = G.assigned(case)
    if len(a):
        e.add_pods(a, np.zeros(len(a), dtype=np.int32))
    pm = G.pods_metric(case)
    if len(pm):  # NodeMetric.Status.PodsMetric (load_aware_test.go:1203, :1588)
        e.set_pods_metric(0, pm)
    return e


def _golden_filter_cases():
    return G.cases("loadaware_filter.json") + G.cases("loadaware_filter_expired.json")


@pytest.mark.parametrize("dc", _golden_filter_cases(), ids=G.case_id)
def test_golden_loadaware_filter_on_device(dc):
    doc, case = dc
    prof = framework.Profile(filter=(framework.LOAD_AWARE,), score={})
    with _one_node_engine(doc, case, prof) as e:
        rej, _, _ = e.evaluate(G.pod(case.get("pod")))
        got = "Unschedulable" if rej[0] & abi.REJECT_LOADAWARE else "Success"
        assert got == case["want"], case["source_line"]


@pytest.mark.parametrize("dc", G.cases("loadaware_score.json"), ids=G.case_id)
def test_golden_loadaware_score_on_device(dc):
    doc, case = dc
    prof = framework.Profile(filter=(), score={framework.LOAD_AWARE: 1})
    with _one_node_engine(doc, case, prof) as e:
        _, _, la = e.evaluate(G.pod(case.get("pod")))
        assert la[0] == case["want"], case["source_line"]


# ---------------------------------------------------------------------------------------------------
# exactness of the division-free leastRequestedScore
# ---------------------------------------------------------------------------------------------------
def test_least_requested_exact():
    rng = np.random.default_rng(5)
    caps = np.concatenate([rng.integers(1, 1 << 20, 20000), rng.integers(1, 1 << 50, 20000),
                           np.array([1, 2, 3, 7, 96000, 128 << 30, (1 << 50) - 1, 100, 1000])])
    fr = rng.random(len(caps))
    req = np.floor(caps * fr).astype(np.int64)
    # exact boundaries: requested making (cap-req)*100/cap an integer, ±1
    k = rng.integers(0, 101, len(caps))
    req2 = caps - (caps * k) // 100
    reqs = np.concatenate([req, req2, req2 + 1, req2 - 1, caps, caps + 1, np.zeros_like(caps), -np.ones_like(caps)])
    capv = np.tile(caps, 8)
    cfg = framework.build_config()
    with Engine(cfg, 1) as e:
        got = e.debug_least_requested(reqs, capv)
    want = np.array([oracle.least_requested(int(r), int(c)) for r, c in zip(reqs, capv)])
    np.testing.assert_array_equal(got, want)


def _lrs_exact(req, cap):
    # leastRequestedScore (load_aware.go:388-397) in exact integer arithmetic (Python ints)
    return np.array([0 if (c == 0 or r > c) else ((c - r) * 100) // c for r, c in zip(req.tolist(), cap.tolist())])


@pytest.mark.parametrize("cap_hi,name", [(1 << 24, "cpu"), (1 << 45, "mem")])
def test_fast_lrs_exact(cap_hi, name):
    """The wide pass's division-free quotient routines equal the exact quotient on their whole domain: random
    pairs, every exact-integer quotient boundary ±1, the capacity edge, and small capacities."""
    rng = np.random.default_rng(11 if name == "cpu" else 12)
    caps = np.concatenate([rng.integers(1, cap_hi, 30000), rng.integers(1, 4096, 5000),
                           np.array([1, 2, 3, 7, 100, 1000, 96000, cap_hi - 1, cap_hi - 2, (cap_hi - 1) // 3]),
                           # node-sized memory capacities (GiB multiples, a few bytes off them)
                           np.array([g << 30 for g in (1, 3, 16, 255, 256, 1024, 4095)] +
                                    [(g << 30) + d for g in (7, 512) for d in (-1, 1, 4095)], dtype=np.int64)])
    caps = caps[caps < cap_hi]
    k = rng.integers(0, 101, len(caps))
    edge = caps - (caps * k + 99) // 100          # smallest requested with quotient ≥ 100 - k … boundaries
    reqs = np.concatenate([np.floor(caps * rng.random(len(caps))).astype(np.int64), edge, edge + 1, edge - 1,
                           caps, caps - 1, np.zeros_like(caps), caps + 5, caps * 2])
    capv = np.tile(caps, 9)
    with Engine(framework.build_config(), 1) as e:
        oc, om = e.debug_fast_lrs(reqs, capv)
    got = oc if name == "cpu" else om
    free = capv - reqs
    lo = -(1 << 30) if name == "cpu" else -(1 << 52) + 1
    dom = (capv > 0) & (capv < cap_hi) & (free >= lo) & (free <= capv)
    assert dom.sum() > 0.8 * len(dom)
    assert np.all(got[~dom] == -1)
    np.testing.assert_array_equal(got[dom], _lrs_exact(reqs[dom], capv[dom]))


# ---------------------------------------------------------------------------------------------------
# synthetic clusters: placements + final state vs oracle
# ---------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("n_nodes,n_pods,seed", [(500, 5000, 1), (1000, 4000, 2), (3000, 6000, 3), (257, 3000, 4)])
def test_schedule_parity_synthetic(n_nodes, n_pods, seed):
    cfg = framework.build_config()
    cl = synth.make_cluster(n_nodes, seed=seed)
    pods = synth.make_pods(n_pods, seed=seed + 100)
    gn, stats = _parity(cfg, cl, pods)
    assert stats["device_batches"] > 0


@pytest.mark.parametrize("batch,ppw", [(1, 1), (3, 1), (16, 4), (33, 5), (64, 2), (64, 64)])
def test_schedule_parity_round_shapes(batch, ppw):
    cfg = framework.build_config(batch_pods=batch, pods_per_wave=ppw)
    cl = synth.make_cluster(900, seed=21)
    pods = synth.make_pods(2500, seed=22)
    _parity(cfg, cl, pods)


@pytest.mark.parametrize("depth", [1, 2])
def test_fresh_engine_after_destroy_poisoned(depth, monkeypatch):
    """Regression (GPUTEST_r03: round_shapes[16-4] placed pod 0 on node 230 instead of 277 on the driver's box).
    Cause: the engine's zero fill of the node table ran as null-stream hipMemset calls, which the engine's
    non-blocking streams do not order against, so on some boxes the fill landed after the first NodeMetric deltas and
    the node usage vanished from la_used (the box's placements equal the oracle's with NodeUsage = 0).  The fill is now
    stream-ordered and synchronised before kg_engine_create returns.  This runs the failing shape on an engine created
    right after another one was destroyed, with every fresh device buffer poison-filled (KG_DEBUG_POISON), so a read of
    memory the engine never wrote would show as a wrong answer; ingest follows creation with no host delay."""
    cl = synth.make_cluster(900, seed=21)
    pods = synth.make_pods(2500, seed=22)
    cfg = framework.build_config(batch_pods=16, pods_per_wave=4, pipeline_depth=depth)
    on, os_, st = oracle.schedule_cluster(cfg, cl, pods, n_threads=4)
    with _engine(framework.build_config(batch_pods=3, pods_per_wave=1), cl) as e0:
        e0.schedule(pods)
    monkeypatch.setenv("KG_DEBUG_POISON", "1")
    e = Engine(cfg, cl.n)
    try:
        synth.load_into(e, cl)
        gn, gs, _ = e.schedule(pods)
        mism = np.nonzero(gn != on)[0]
        assert mism.size == 0, f"first mismatch at pod {mism[:5]}: gpu {gn[mism[:5]]} oracle {on[mism[:5]]}"
        np.testing.assert_array_equal(gs, os_)
        _assert_state_equal(e, st)
    finally:
        e.close()


@pytest.mark.parametrize("depth,batch", [(1, 32), (2, 32), (3, 32), (4, 32), (2, 64), (3, 48), (4, 13)])
def test_schedule_parity_pipeline_depths(depth, batch):
    """Rounds in flight (eval(r) reads the table right after resolve(r - depth)): every depth and batch shape
    gives the sequential result, including a tie-heavy cluster where most pods take the speculative resolver's
    slow path."""
    cfg = framework.build_config(batch_pods=batch, pods_per_wave=8, pipeline_depth=depth)
    _parity(cfg, synth.make_cluster(1500, seed=23), synth.make_pods(4000, seed=24))
    n = 300
    nodes = np.concatenate([framework.make_node({"cpu": "16", "memory": "64Gi"}) for _ in range(n)])
    metrics = np.concatenate([framework.make_node_metric(update_time_ns=synth.T0_NS,
                                                         node_usage={"cpu": "1", "memory": "1Gi"}) for _ in range(n)])
    cl = synth.Cluster(nodes, metrics, np.zeros(0, dtype=abi.POD_DTYPE), np.zeros(0, dtype=np.int32),
                       synth.T0_NS + 10**9)
    _parity(cfg, cl, synth.make_pods(2500, seed=25))


def test_schedule_parity_profile_variants():
    cl = synth.make_cluster(800, seed=31)
    pods = synth.make_pods(2000, seed=32)
    for la, prof in [
        (framework.LoadAwareSchedulingArgs(), framework.Profile(score={framework.NODE_RESOURCES_FIT: 1})),
        (framework.LoadAwareSchedulingArgs(), framework.Profile(score={framework.LOAD_AWARE: 3})),
        (framework.LoadAwareSchedulingArgs(resource_weights={"cpu": 3, "memory": 1}, usage_thresholds={"cpu": 50}),
         framework.Profile(score={framework.NODE_RESOURCES_FIT: 2, framework.LOAD_AWARE: 5})),
        (framework.LoadAwareSchedulingArgs(prod_usage_thresholds={"cpu": 40}, score_according_prod_usage=True),
         framework.Profile()),
        (framework.LoadAwareSchedulingArgs(node_metric_expiration_seconds=5), framework.Profile()),
    ]:
        _parity(framework.build_config(la=la, profile=prof), cl, pods)


def test_ties_resolve_to_lowest_index():
    n = 600
    nodes = np.concatenate([framework.make_node({"cpu": "16", "memory": "64Gi"}) for _ in range(n)])
    metrics = np.concatenate([framework.make_node_metric(update_time_ns=synth.T0_NS,
                                                         node_usage={"cpu": "1", "memory": "1Gi"}) for _ in range(n)])
    cl = synth.Cluster(nodes, metrics, np.zeros(0, dtype=abi.POD_DTYPE), np.zeros(0, dtype=np.int32),
                       synth.T0_NS + 10**9)
    pods = np.concatenate([framework.make_pod({"cpu": "100m", "memory": "128Mi"}, priority_class="koord-prod")
                           for _ in range(3000)])
    gn, _ = _parity(framework.build_config(), cl, pods)
    assert gn[0] == 0


def test_unschedulable_and_saturation():
    cfg = framework.build_config()
    cl = synth.make_cluster(100, seed=41)
    pods = synth.make_pods(6000, seed=42)  # far more than fits: the tail must be unschedulable
    gn, _ = _parity(cfg, cl, pods)
    assert (gn < 0).sum() > 0


def test_edge_clusters():
    cfg = framework.build_config()
    pods = synth.make_pods(300, seed=5)
    for n in (1, 2, 63, 64, 65, 255, 256):
        _parity(cfg, synth.make_cluster(n, seed=n), pods)
    # deleted nodes, daemonset + zero-request pods
    cl = synth.make_cluster(700, seed=51, invalid_frac=0.2)
    p = synth.make_pods(1500, seed=52)
    p["flags"][::7] = abi.POD_DAEMONSET
    p["requests"][::11] = 0
    p["limits"][::11] = 0
    p["nonzero_requests"][::11] = (100, 200 << 20)
    _parity(cfg, cl, p)


def test_empty_cluster_all_unschedulable():
    cfg = framework.build_config()
    with Engine(cfg, 16) as e:
        gn, gs, _ = e.schedule(synth.make_pods(10, seed=1))
    assert (gn == -1).all() and (gs == 0).all()


def test_incremental_calls_and_unreserve():
    """Two schedule calls + Unreserve deltas == one oracle run with the same deltas."""
    cfg = framework.build_config()
    cl = synth.make_cluster(1200, seed=61)
    pods = synth.make_pods(3000, seed=62)
    on, _, st = oracle.schedule_cluster(cfg, cl, pods[:1500], n_threads=4)
    with _engine(cfg, cl) as e:
        g1, _, _ = e.schedule(pods[:1500])
        np.testing.assert_array_equal(g1, on)
        ok = np.nonzero(g1 >= 0)[0][::3]
        e.remove_pods(pods[ok], g1[ok])  # Unreserve / ForgetPod
        for i in ok:
            oracle.lib().or_apply_pod(oracle.p(cfg), oracle.p(st[g1[i]:g1[i] + 1]), oracle.p(pods[i:i + 1]), -1)
        on2, _ = oracle.schedule(cfg, cl.nodes, cl.metrics, st, pods[1500:], cl.now_ns, n_threads=4)
        g2, _, _ = e.schedule(pods[1500:])
        np.testing.assert_array_equal(g2, on2)
        _assert_state_equal(e, st)


def test_node_updates_between_calls():
    cfg = framework.build_config()
    cl = synth.make_cluster(600, seed=71)
    pods = synth.make_pods(2000, seed=72)
    with _engine(cfg, cl) as e:
        st = oracle.states(cl.n)
        oracle.add_pods(cfg, st, cl.existing_pods, cl.existing_node)
        g1, _, _ = e.schedule(pods[:700])
        o1, _ = oracle.schedule(cfg, cl.nodes, cl.metrics, st, pods[:700], cl.now_ns)
        np.testing.assert_array_equal(g1, o1)
        # informer deltas: resize some nodes, refresh metrics, delete a few
        nodes = cl.nodes.copy()
        metrics = cl.metrics.copy()
        nodes["allocatable"][::5, abi.RES_CPU] += 16000
        metrics["node_usage"][::3, abi.RES_CPU] //= 2
        e.upsert_nodes(nodes[::5], np.arange(0, cl.n, 5))
        e.update_metrics(metrics[::3], cl.now_ns, np.arange(0, cl.n, 3))
        e.delete_nodes([1, 2, 3])
        nodes["flags"][[1, 2, 3]] &= ~abi.NODE_VALID
        g2, _, _ = e.schedule(pods[700:])
        o2, _ = oracle.schedule(cfg, nodes, metrics, st, pods[700:], cl.now_ns)
        np.testing.assert_array_equal(g2, o2)
        _assert_state_equal(e, st)


def test_evaluate_matches_oracle_per_plugin():
    cfg = framework.build_config()
    cl = synth.make_cluster(1000, seed=81)
    st = oracle.states(cl.n)
    oracle.add_pods(cfg, st, cl.existing_pods, cl.existing_node)
    pods = synth.make_pods(20, seed=82)
    with _engine(cfg, cl) as e:
        for k in range(len(pods)):
            rej, fit, la = e.evaluate(pods[k])
            for i in range(0, cl.n, 7):
                of = oracle.fit_filter(cl.nodes[i:i + 1], st[i:i + 1], pods[k:k + 1])
                ol = oracle.loadaware_filter(cfg, cl.nodes[i:i + 1], cl.metrics[i:i + 1], pods[k:k + 1], cl.now_ns)
                assert (rej[i] & 7) == of, (k, i)
                assert bool(rej[i] & abi.REJECT_LOADAWARE) == bool(ol), (k, i)
                assert fit[i] == oracle.fit_score(cfg, cl.nodes[i:i + 1], st[i:i + 1], pods[k:k + 1])
                assert la[i] == oracle.loadaware_score(cfg, cl.nodes[i:i + 1], cl.metrics[i:i + 1], st[i:i + 1],
                                                       pods[k:k + 1], cl.now_ns)


@pytest.mark.slow
def test_c2_scale_properties():
    """BASELINE config 2 (10k nodes × 100k pods): exact vs the oracle on the first 20k pods, and at full size
    the size-independent properties — batch-shape invariance (B=1 is the trivially sequential device path),
    conservation of requested resources, and feasibility of every placement."""
    cfg = framework.build_config()
    cl = synth.make_cluster(10_000, seed=synth.BASE_SEED + 2)
    pods = synth.make_pods(100_000, seed=synth.BASE_SEED + 3)
    on, _, _ = oracle.schedule_cluster(cfg, cl, pods[:20_000], n_threads=8)
    with _engine(cfg, cl) as e:
        g, s, _ = e.schedule(pods)
        np.testing.assert_array_equal(g[:20_000], on)
        st = e.read_state()
    with _engine(framework.build_config(batch_pods=1, pods_per_wave=1), cl) as e1:
        g1, s1, _ = e1.schedule(pods[:30_000])
    np.testing.assert_array_equal(g[:30_000], g1)
    np.testing.assert_array_equal(s[:30_000], s1)
    placed = g >= 0
    base = np.bincount(cl.existing_node, weights=cl.existing_pods["requests"][:, 0], minlength=cl.n)
    add = np.bincount(g[placed], weights=pods["requests"][placed, 0], minlength=cl.n)
    np.testing.assert_array_equal(st["requested_cpu"], (base + add).astype(np.int64))
    assert (st["requested_cpu"] <= cl.nodes["allocatable"][:, 0]).all()
    assert (st["num_pods"] <= 110).all()


def test_eval_paths_agree():
    """The wide pass's hoisted-term evaluation equals the reference-shaped one on every (pod, node)."""
    for la, prof in [(framework.LoadAwareSchedulingArgs(), framework.Profile()),
                     (framework.LoadAwareSchedulingArgs(resource_weights={"cpu": 7, "memory": 3},
                                                        score_according_prod_usage=True),
                      framework.Profile(score={framework.NODE_RESOURCES_FIT: 3, framework.LOAD_AWARE: 11}))]:
        cfg = framework.build_config(la=la, profile=prof)
        cl = synth.make_cluster(3000, seed=91, invalid_frac=0.05)
        cl.nodes["raw_allocatable"][::4, :2] = cl.nodes["allocatable"][::4, :2] // 2
        cl.nodes["raw_allocatable_present"][::4, :2] = 1
        cl.nodes["flags"][::4] |= abi.NODE_HAS_RAW_ALLOCATABLE
        cl.nodes["allocatable"][::17, abi.RES_MEMORY] = 0
        with _engine(cfg, cl) as e:
            e.schedule(synth.make_pods(2000, seed=92))  # mutate the table
            p = synth.make_pods(200, seed=93)
            p["requests"][::9] = 0
            p["flags"][::5] = abi.POD_DAEMONSET
            e.stage(p)
            assert e.debug_eval_paths() == 0


@pytest.mark.slow
def test_c3_full_size():
    """BASELINE config 3 on one GPU at full size: the 100k-node cluster and the 1M-pod queue bench.py times (same
    seeds, same default geometry).  (r6) Every one of the 1M placements and weighted totals, and the final node state,
    are compared bit-exactly with the oracle's sequential schedule of the whole queue — the committed fixture
    tests/golden/c3_queue.npz written by tests/golden/make_c3_fixture.py (oracle/oracle.c or_schedule; the north_star's
    "bit-exact placements for 1M queued pods on a 100k-node synthetic cluster").  The live oracle re-checks the first
    10k pods on this box, and the queue's segment digests prove it is the fixture's queue.  Conservation and
    feasibility are asserted as well."""
    import hashlib
    import json
    import os
    fx = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "c3_queue.npz"))
    meta = json.loads(str(fx["meta"]))
    n_pods = 1_000_000
    assert meta["nodes"] == 100_000 and meta["pods"] >= n_pods and meta["state_at"] == n_pods
    cfg = framework.build_config()
    cl = synth.make_cluster(100_000, seed=meta["cluster_seed"])
    pods = synth.make_pods_stream(n_pods, seed=meta["pods_seed"])
    seg = meta["segment"]
    for s in range(n_pods // seg):
        assert hashlib.sha256(np.ascontiguousarray(pods[s * seg:(s + 1) * seg]).tobytes()).hexdigest() == \
            str(fx["seg_sha"][s]), f"queue segment {s} differs from the fixture's"
    on, osc, _ = oracle.schedule_cluster(cfg, cl, pods[:10_000], n_threads=16)
    np.testing.assert_array_equal(fx["node"][:10_000], on)  # the fixture is the oracle's schedule (live, this box)
    np.testing.assert_array_equal(fx["score"][:10_000].astype(np.int64), osc)
    with _engine(cfg, cl) as e:
        e.stage(pods)
        for s in range(0, len(pods), 100_000):
            e.schedule_staged(s, 100_000)
        g, sc = e.fetch(0, len(pods))
        st = e.read_state()
    mism = np.nonzero(g != fx["node"][:n_pods])[0]
    assert mism.size == 0, f"{mism.size} placements differ from the oracle's; first at pods {mism[:5]}"
    mism = np.nonzero(sc != fx["score"][:n_pods].astype(np.int64))[0]
    assert mism.size == 0, f"{mism.size} totals differ from the oracle's; first at pods {mism[:5]}"
    for k in ("requested_cpu", "requested_mem", "nonzero_cpu", "nonzero_mem", "num_pods", "la_est_cpu", "la_est_mem",
              "la_est_prod_cpu", "la_est_prod_mem"):
        np.testing.assert_array_equal(st[k], fx["st1m_" + k], err_msg=k)
    placed = g >= 0
    assert placed.sum() > 900_000
    for r, col in ((abi.RES_CPU, "requested_cpu"), (abi.RES_MEMORY, "requested_mem")):
        base = np.bincount(cl.existing_node, weights=cl.existing_pods["requests"][:, r].astype(np.float64),
                           minlength=cl.n)
        add = np.bincount(g[placed], weights=pods["requests"][placed, r].astype(np.float64), minlength=cl.n)
        np.testing.assert_array_equal(st[col], (base + add).astype(np.int64))
        assert (st[col] <= cl.nodes["allocatable"][:, r]).all()
    assert (st["num_pods"] <= cl.nodes["allowed_pods"]).all()


def test_lookahead_resolver_parity():
    """The look-ahead resolver (resolve_mw: chain + keeper + helper waves) is not the default; its
    selection is read once per process, so its parity runs in a child process with KG_RESOLVER=mw."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, "-u", os.path.join(here, "resolver_ab.py")], env={**os.environ, "KG_RESOLVER": "mw"},
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "parity: ok" in r.stdout
