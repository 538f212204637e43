"""GPU parity of DeviceShare (config C5's GPU-share part): the HIP engine through the C ABI against the oracle
(oracle/deviceshare.c + the oracle's scheduling loop) and the reference's own test tables
(tests/golden/deviceshare.json).

Bar: bit-exact — Filter verdicts and raw plugin scores, placements and weighted totals (with DeviceShare's
NormalizeScore over the feasible nodes), the GPU minors Reserve allocates to every pod, and the final
deviceUsed plus NodeInfo / LoadAware node state."""
import numpy as np
import pytest

import test_golden_deviceshare as TG
from koordinator_amd import Engine, abi, framework, synth
from koordinator_amd.abi import KoordGPUError
from oracle import oracle

pytestmark = pytest.mark.gpu
F = framework
PROFILE = TG.DS_PROFILE


def _engine_one(cfg, dev):
    e = Engine(cfg, 1)
    e.upsert_nodes(F.make_node({"cpu": "64", "memory": "256Gi"}))
    e.upsert_devices(dev)
    return e


@pytest.mark.parametrize("c", TG._cases(("score",)), ids=TG._id)
def test_golden_score_device(c):
    cfg = TG.case_config(c)
    dev, pod = TG.node_device(c["node"]), TG.case_pod(c)
    with _engine_one(cfg, dev) as e:
        ok, sc = e.evaluate_device(pod)
    assert bool(ok[0]) == c["want_filter"], c["source"]
    if c["want_filter"]:
        assert int(sc[0]) == c["want_score"], c["source"]


@pytest.mark.parametrize("c", TG._cases(("filter",)), ids=TG._id)
def test_golden_filter_device(c):
    dev, pod = TG.node_device(c["node"]), TG.case_pod(c)
    with _engine_one(TG.case_config(c), dev) as e:
        ok, _ = e.evaluate_device(pod)
    assert bool(ok[0]) == c["want_filter"], c["source"]


@pytest.mark.parametrize("c", TG._cases(("reserve",)), ids=TG._id)
def test_golden_reserve_device(c):
    cfg = TG.case_config(c)
    if not c.get("strategy"):
        cfg[0]["ds_scoring_weights"] = 0
    dev, pod = TG.node_device(c["node"]), TG.case_pod(c)
    with _engine_one(cfg, dev) as e:
        node, _, _ = e.schedule(pod)
        assert node[0] == 0
        mask = e.fetch_devices(0, 1)[0]
        uc, um, ur = e.read_devices()
    assert mask == sum(1 << m for m in c["want_minors"]), c["source"]
    inst = c["want_instance"]
    for m in range(abi.MAX_MINORS):
        k = 1 if m in c["want_minors"] else 0
        assert ur[0, m] - dev[0]["used_ratio"][m] == k * inst["ratio"], c["source"]
        assert um[0, m] - dev[0]["used_memory"][m] == k * inst["memory"], c["source"]
        assert uc[0, m] - dev[0]["used_core"][m] == k * inst["core"], c["source"]


def _oracle_run(cfg, cluster, dev, pods):
    st = oracle.states(cluster.n)
    if len(cluster.existing_pods):
        oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
    d = dev.copy()
    node, score, _, minors = oracle.schedule_full(cfg, cluster.nodes, cluster.metrics, st, pods, cluster.now_ns, 8,
                                                  devices=d)
    return node, score, minors, st, d


def _engine_run(cfg, cluster, dev, pods, chunks=1):
    with Engine(cfg, cluster.n) as e:
        synth.load_gpu_into(e, cluster, dev)
        e.stage(pods)
        step = (len(pods) + chunks - 1) // chunks
        for s in range(0, len(pods), step):
            e.schedule_staged(s, min(step, len(pods) - s))
        node, score = e.fetch(0, len(pods))
        minors = e.fetch_devices(0, len(pods))
        state = e.read_state()
        used = e.read_devices()
    return node, score, minors, state, used


def _check(cfg, cluster, dev, pods, chunks=1):
    want_node, want_score, want_minors, st, d = _oracle_run(cfg, cluster, dev, pods)
    node, score, minors, state, used = _engine_run(cfg, cluster, dev, pods, chunks)
    bad = np.flatnonzero((node != want_node) | (score != want_score))
    assert bad.size == 0, f"first mismatch at pod {bad[0]}: gpu ({node[bad[0]]}, {score[bad[0]]}) vs oracle " \
                          f"({want_node[bad[0]]}, {want_score[bad[0]]})"
    assert np.array_equal(minors, want_minors)
    assert np.array_equal(state["requested_cpu"], st["requested"][:, abi.RES_CPU])
    assert np.array_equal(state["requested_mem"], st["requested"][:, abi.RES_MEMORY])
    assert np.array_equal(state["num_pods"], st["num_pods"])
    assert np.array_equal(used[0], d["used_core"]) and np.array_equal(used[1], d["used_memory"])
    assert np.array_equal(used[2], d["used_ratio"])
    return node


@pytest.mark.parametrize("n_nodes,n_pods,batch,ppw,seed", [
    (300, 2000, 32, 8, 1), (1000, 3000, 16, 4, 2), (257, 1500, 1, 1, 3), (700, 2500, 7, 3, 4), (2000, 3000, 32, 1, 5),
])
def test_schedule_parity_synthetic(n_nodes, n_pods, batch, ppw, seed):
    cluster, dev = synth.make_gpu_cluster(n_nodes, seed=100 + seed)
    pods = synth.make_gpu_pods(n_pods, seed=200 + seed)
    cfg = F.build_config(profile=PROFILE, batch_pods=batch, pods_per_wave=ppw)
    node = _check(cfg, cluster, dev, pods)
    assert (node >= 0).mean() > 0.5


def test_schedule_parity_gpu_heavy_small_cluster():
    """Few nodes, every pod asks for GPU share: the normalization max moves constantly (early-stopped rounds),
    GPUs fill up and pods become unschedulable."""
    cluster, dev = synth.make_gpu_cluster(48, seed=31)
    pods = synth.make_gpu_pods(1500, seed=32)
    pods["device_requests"][:, abi.DEV_GPU_MEMORY_RATIO] = np.where(
        pods["device_requests"].any(axis=1), pods["device_requests"][:, abi.DEV_GPU_MEMORY_RATIO], 50)
    pods["device_requests"][:, abi.DEV_GPU_CORE] = np.where(pods["device_requests"][:, abi.DEV_GPU_MEMORY] > 0, 0,
                                                            pods["device_requests"][:, abi.DEV_GPU_CORE])
    cfg = F.build_config(profile=PROFILE, batch_pods=32, pods_per_wave=8)
    node = _check(cfg, cluster, dev, pods, chunks=3)
    assert (node < 0).any() and (node >= 0).any()


def test_schedule_parity_weights_and_filter_only():
    cluster, dev = synth.make_gpu_cluster(600, seed=41)
    pods = synth.make_gpu_pods(1200, seed=42)
    for prof in (F.Profile(filter=(F.NODE_RESOURCES_FIT, F.DEVICE_SHARE), score={F.NODE_RESOURCES_FIT: 1}),
                 F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.DEVICE_SHARE),
                           score={F.NODE_RESOURCES_FIT: 2, F.LOAD_AWARE: 1, F.DEVICE_SHARE: 7})):
        _check(F.build_config(profile=prof), cluster, dev, pods)


@pytest.mark.parametrize("batch,ppw,seed", [(32, 8, 1), (16, 4, 2), (1, 1, 3)])
def test_schedule_parity_most_allocated(batch, ppw, seed):
    """MostAllocated (scoring.go:281-304): an assume raises the node's DeviceShare score, so a modified row can lift
    the normalization max: the resolver re-scores modified rows for every pod and ends the round when it rises."""
    cluster, dev = synth.make_gpu_cluster(400, seed=300 + seed)
    pods = synth.make_gpu_pods(2000, seed=400 + seed)
    args = F.DeviceShareArgs(scoring_strategy="MostAllocated")
    prof = F.Profile(filter=PROFILE.filter, score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.DEVICE_SHARE: 5})
    _check(F.build_config(profile=prof, deviceshare=args, batch_pods=batch, pods_per_wave=ppw), cluster, dev, pods)


def test_scoring_weights_over_core_and_memory():
    cluster, dev = synth.make_gpu_cluster(400, seed=51)
    pods = synth.make_gpu_pods(1000, seed=52)
    args = F.DeviceShareArgs(scoring_resources={"koordinator.sh/gpu-core": 2, "koordinator.sh/gpu-memory": 1,
                                                "koordinator.sh/gpu-memory-ratio": 3})
    _check(F.build_config(profile=PROFILE, deviceshare=args), cluster, dev, pods)


def test_evaluate_device_matches_oracle():
    cluster, dev = synth.make_gpu_cluster(500, seed=61)
    pods = synth.make_gpu_pods(40, seed=62)
    cfg = F.build_config(profile=PROFILE)
    with Engine(cfg, cluster.n) as e:
        synth.load_gpu_into(e, cluster, dev)
        for i in range(len(pods)):
            ok, sc = e.evaluate_device(pods[i])
            want_ok = np.array([oracle.ds_filter(dev[j:j + 1], pods[i]) for j in range(cluster.n)])
            want_sc = np.array([oracle.ds_score(cfg[0], dev[j:j + 1], pods[i]) if want_ok[j] else 0
                                for j in range(cluster.n)])
            assert np.array_equal(ok.astype(bool), want_ok)
            assert np.array_equal(sc, want_sc)


def test_unsupported_requests_fail_loudly():
    cfg = F.build_config(profile=PROFILE)
    with Engine(cfg, 4) as e:
        with pytest.raises(KoordGPUError) as ei:
            # (ABI 17) RDMA / FPGA are accelerated; a request beyond the accelerated range is still refused
            e.stage(F.make_pod({"cpu": "1"}, devices={"koordinator.sh/rdma": 1 << 21}))
        assert ei.value.code == abi.E_UNSUPPORTED
    with Engine(F.build_config(), 4) as e:  # no DeviceShare in the profile: device requests are refused
        with pytest.raises(KoordGPUError):
            e.stage(F.make_pod({"cpu": "1"}, devices={"koordinator.sh/gpu-memory-ratio": 50}))


def test_bench_kernels_run():
    cluster, dev = synth.make_gpu_cluster(3000, seed=71)
    pods = synth.make_gpu_pods(64, seed=72)
    with Engine(F.build_config(profile=PROFILE), cluster.n) as e:
        synth.load_gpu_into(e, cluster, dev)
        e.stage(pods)
        for which in range(5):
            ms, b = e.bench_kernel(which, 3)
            assert ms > 0 and b > 0
