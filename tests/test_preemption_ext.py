"""(r6, ABI 16) The preemption dry run with NodeNUMAResource, DeviceShare and TaintToleration / NodeAffinity in the
profile (kg_pods_filter_preemption / kg_pods_select_victims with victim_minors).

What the reference does on this path:
  - DeviceShare's PreFilterExtensions (deviceshare/plugin.go:163-278): RemovePod appends a victim's GPU allocation
    (nodeDevice.getUsed) to state.preemptibleDevices[node], AddPod subtracts it; reserve pods, state.skip and victims
    allocated from a reservation (preemptibleInRRs) leave it alone.  Filter (:280-330) allocates with free =
    total − max(0, used − preemptible) (calcFreeWithPreemptible, device_cache.go:314-342).
  - NodeNUMAResource has no PreFilterExtensions (nodenumaresource/plugin.go:272-274): the victims' cpusets stay in the
    NodeAllocation; only filterAmplifiedCPUs sees the victim-free NodeInfo.Requested.
  - TaintToleration / NodeAffinity are node-static.

Pinned by the reference's DeviceShare tables: Test_Plugin_PreFilterExtensions (plugin_test.go:215-327: RemovePod of
an allocated pod makes its minor preemptible, AddPod takes it back) and Test_Plugin_Filter "allocate from preemptible"
(plugin_test.go:1595-1668), restated here as a node + victim whose RemovePod builds that preemptible map, so the same
rows run on the oracle (CPU) and through the C ABI (GPU).  The random tests compare device and oracle bit-exactly on
shipped-profile clusters with predicates."""
import numpy as np
import pytest

from koordinator_amd import Engine, abi, framework as F, synth
from oracle import oracle

GI = 1 << 30
DS_FILTER = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.DEVICE_SHARE), score={F.NODE_RESOURCES_FIT: 1})
NUMA_FILTER = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.NODE_NUMA_RESOURCE), score={F.NODE_RESOURCES_FIT: 1})
EXT = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.NODE_NUMA_RESOURCE, F.DEVICE_SHARE, F.RESERVATION,
                        F.TAINT_TOLERATION, F.NODE_AFFINITY),
                score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.NODE_NUMA_RESOURCE: 1, F.DEVICE_SHARE: 1,
                       F.RESERVATION: 1})


def _gpu(minor, mem, used=(0, 0, 0)):
    return {"minor": minor, "healthy": True, "total": {"core": 100, "ratio": 100, "memory": mem},
            "used": {"core": used[0], "ratio": used[1], "memory": used[2]}}


def _one_node(dev, victims):
    node = F.make_node({"cpu": "32", "memory": "64Gi"}, allowed_pods=100)
    metric = F.make_node_metric(present=False, node_usage=None)
    cl = synth.Cluster(node, metric, victims, np.zeros(len(victims), dtype=np.int32), 10**18)
    return cl, dev


def _oracle(cfg, cl, dev, pod, vic, minors, slots=None, select=False, numa=None, pred=None):
    st = oracle.states(cl.n)
    oracle.add_pods(cfg, st, cl.existing_pods, cl.existing_node)
    kw = dict(numa=None if numa is None else numa[0], dev=None if dev is None else dev[0],
              pred=None if pred is None else pred[0], minors=minors)
    if select:
        return oracle.select_victims(cfg, cl.nodes[0], cl.metrics[0], st[:1], None, pod, vic, slots, None, cl.now_ns,
                                     **kw)
    return oracle.filter_preemption(cfg, cl.nodes[0], cl.metrics[0], st[:1], None, pod, vic, slots, cl.now_ns, **kw)


def _device(cfg, cl, dev, pod, vic, minors, slots=None, select=False, numa=None):
    with Engine(cfg, cl.n) as e:
        synth.load_into(e, cl)
        if dev is not None:
            e.upsert_devices(dev)
        if numa is not None:
            e.upsert_numa(numa)
        if select:
            rej, kept, nv = e.select_victims(pod, np.zeros(1, np.int32), [vic], None if slots is None else [slots],
                                             None, [minors])
            return int(rej[0]), kept[0], int(nv[0])
        return e.filter_preemption(pod, 0, vic, slots, minors)


def case_allocate_from_preemptible():
    """plugin_test.go:1595-1668: one 16Gi GPU (minor 0) used 100 / 100 / 16Gi; the pod asks gpu-core 100 +
    gpu-memory-ratio 100; preemptibleDevices[node] = minor 0 whole → Filter nil.  The victim holding minor 0 (the
    same request) builds that map through RemovePod."""
    dev = F.make_node_device([_gpu(0, 16 * GI, (100, 100, 16 * GI))])
    vic = F.make_pod({"cpu": "1"}, devices={"koordinator.sh/gpu-core": 100, "koordinator.sh/gpu-memory-ratio": 100})
    pod = F.make_pod({"cpu": "1"}, devices={"koordinator.sh/gpu-core": 100, "koordinator.sh/gpu-memory-ratio": 100})
    cl, dev = _one_node(dev, vic)
    return cl, dev, pod, vic


def case_prefilter_extensions(other_used):
    """plugin_test.go:215-327: GPUs minors 1 and 2 (100 / 8Gi / 100); allocated-pod-1 holds minor 1 whole; the pod
    asks koordinator.sh/gpu 100.  RemovePod → preemptibleDevices = minor 1 whole; AddPod → empty again.
    other_used: minor 2 fully used by a pod that is not a victim (so the pod fits only through the preemptible minor)."""
    u2 = (100, 100, 8 * GI) if other_used else (0, 0, 0)
    dev = F.make_node_device([_gpu(1, 8 * GI, (100, 100, 8 * GI)), _gpu(2, 8 * GI, u2)])
    vic = F.make_pod({"cpu": "1"}, devices={"koordinator.sh/gpu": 100})
    pod = F.make_pod({"cpu": "1"}, devices={"koordinator.sh/gpu": 100})
    cl, dev = _one_node(dev, vic)
    return cl, dev, pod, vic


MINOR0, MINOR1 = np.array([1], np.int32), np.array([2], np.int32)


def test_oracle_allocate_from_preemptible():
    cfg = F.build_config(profile=DS_FILTER)
    cl, dev, pod, vic = case_allocate_from_preemptible()
    assert _oracle(cfg, cl, dev, pod, vic[:0], MINOR0[:0]) == abi.REJECT_DEVICE  # no victims: deviceFree 0
    assert _oracle(cfg, cl, dev, pod, vic, MINOR0) == 0                           # the reference's want: nil
    # RemovePod returns first for a reserve pod, and a victim allocated from a reservation goes to preemptibleInRRs
    rv = vic.copy()
    rv["flags"] |= abi.POD_RESERVE
    assert _oracle(cfg, cl, dev, pod, rv, MINOR0) == abi.REJECT_DEVICE
    assert _oracle(cfg, cl, dev, pod, vic, MINOR0, slots=np.array([0], np.int32)) == abi.REJECT_DEVICE
    # the victim's minors say where its share is: on a minor the pod cannot use it frees nothing
    assert _oracle(cfg, cl, dev, pod, vic, np.array([2], np.int32)) == abi.REJECT_DEVICE


def test_oracle_prefilter_extensions_remove_then_add():
    cfg = F.build_config(profile=DS_FILTER)
    cl, dev, pod, vic = case_prefilter_extensions(other_used=True)
    # RemovePod: minor 1 preemptible → fits; AddPod (the reprieve) takes it back → no longer fits → kept as a victim
    assert _oracle(cfg, cl, dev, pod, vic, MINOR1) == 0
    rej, kept, _ = _oracle(cfg, cl, dev, pod, vic, MINOR1, select=True)
    assert rej == 0 and kept.tolist() == [True]
    # minor 2 free: the pod fits without the victim, which is reprieved
    cl, dev, pod, vic = case_prefilter_extensions(other_used=False)
    rej, kept, _ = _oracle(cfg, cl, dev, pod, vic, MINOR1, select=True)
    assert rej == 0 and kept.tolist() == [False]


def test_oracle_preemptor_without_devices_ignores_minors():
    """state.skip: a preemptor without device requests neither reads nor builds preemptibleDevices."""
    cfg = F.build_config(profile=DS_FILTER)
    cl, dev, _, vic = case_allocate_from_preemptible()
    pod = F.make_pod({"cpu": "1"})
    assert _oracle(cfg, cl, dev, pod, vic, MINOR0) == 0
    assert _oracle(cfg, cl, dev, pod, vic[:0], MINOR0[:0]) == 0


def _numa_case():
    """A 1-socket 2-NUMA 8-core SMT2 node (16 cpus) whose cpus 0-11 are held by a bound cpuset victim (12 cpus) and
    the pod an LSR FullPCPUs pod of 8 cpus: Fit passes once the victim leaves (16 − 12 + 12 ≥ 8), but the victim's
    cpuset stays allocated in the NodeAllocation (no PreFilterExtensions), so NodeNUMAResource still rejects."""
    numa = F.make_node_numa(sockets=1, nodes_per_socket=2, cores_per_node=4, cpus_per_core=2,
                            numa_resources=[{"cpu": "8", "memory": "8Gi"}, {"cpu": "8", "memory": "8Gi"}],
                            allocated_cpus=range(12), numa_allocated={0: {"cpu": "8"}, 1: {"cpu": "4"}})
    node = F.make_node({"cpu": "16", "memory": "16Gi"}, allowed_pods=100)
    vic = F.make_pod({"cpu": "12", "memory": "1Gi"}, limits={"cpu": "12", "memory": "1Gi"}, qos="LSR",
                     priority_class="koord-prod", required_cpu_bind_policy="FullPCPUs")
    cl = synth.Cluster(node, F.make_node_metric(present=False, node_usage=None), vic, np.zeros(1, np.int32), 10**18)
    pod = F.make_pod({"cpu": "8", "memory": "1Gi"}, limits={"cpu": "8", "memory": "1Gi"}, qos="LSR",
                     priority_class="koord-prod", required_cpu_bind_policy="FullPCPUs")
    return cl, numa, pod, vic


def test_oracle_numa_victims_cpusets_stay_allocated():
    cfg = F.build_config(profile=NUMA_FILTER)
    cl, numa, pod, vic = _numa_case()
    assert _oracle(cfg, cl, None, pod, vic[:0], None, numa=numa) & abi.REJECT_FIT_CPU
    assert _oracle(cfg, cl, None, pod, vic, None, numa=numa) == abi.REJECT_NUMA
    # the same node with the cpuset released (what a Go dry run never sees) fits
    free = numa.copy()
    free["allocated_cpus"] = 0
    for f in free.dtype.names:
        if f.startswith("numa_alloc"):
            free[f] = 0
    assert _oracle(cfg, cl, None, pod, vic, None, numa=free) == 0


@pytest.mark.gpu
def test_device_reference_rows():
    cfg = F.build_config(profile=DS_FILTER)
    cl, dev, pod, vic = case_allocate_from_preemptible()
    assert _device(cfg, cl, dev, pod, vic[:0], MINOR0[:0]) == abi.REJECT_DEVICE
    assert _device(cfg, cl, dev, pod, vic, MINOR0) == 0
    assert _device(cfg, cl, dev, pod, vic, MINOR0, slots=np.array([0], np.int32)) == abi.REJECT_DEVICE
    cl, dev, pod, vic = case_prefilter_extensions(other_used=True)
    rej, kept, _ = _device(cfg, cl, dev, pod, vic, MINOR1, select=True)
    assert rej == 0 and kept.tolist() == [True]
    cl, dev, pod, vic = case_prefilter_extensions(other_used=False)
    rej, kept, _ = _device(cfg, cl, dev, pod, vic, MINOR1, select=True)
    assert rej == 0 and kept.tolist() == [False]
    cfg = F.build_config(profile=NUMA_FILTER)
    cl, numa, pod, vic = _numa_case()
    assert _device(cfg, cl, None, pod, vic, None, numa=numa) == abi.REJECT_NUMA


def _victim_devices(cluster, dev, vic_idx, rng):
    """Half of the victims get a GPU share on one present minor of their node (gpu-core = gpu-memory-ratio ∈ {25, 50,
    100}); returns their minors (0 = none).  The pods are modified in place (cluster.existing_pods)."""
    minors = np.zeros(len(vic_idx), dtype=np.int32)
    for k, j in enumerate(vic_idx):
        i = int(cluster.existing_node[j])
        present = np.flatnonzero(dev["present"][i])
        if len(present) == 0 or rng.random() < 0.5:
            continue
        c = int(rng.choice([25, 50, 100]))
        p = cluster.existing_pods[j:j + 1]
        p["device_requests"][0] = 0
        p["device_requests"][0, abi.DEVICE_RESOURCE_SLOTS["koordinator.sh/gpu-core"]] = c
        p["device_requests"][0, abi.DEVICE_RESOURCE_SLOTS["koordinator.sh/gpu-memory-ratio"]] = c
        cluster.existing_pods[j] = p[0]
        minors[k] = 1 << int(rng.choice(present))
    return minors


def _ext_world(n, seed):
    cluster, numa, dev, rsv = synth.make_shipped_cluster(n, seed=seed)
    pods = synth.make_shipped_pods(24, seed=seed + 50)
    pods["quota_id"] = 0
    _, preds = synth.make_predicates(n, pods, seed=seed + 60)
    # busy GPUs: most of each present minor used, so the victims' shares decide
    rng = np.random.default_rng(seed + 70)
    pres = dev["present"] != 0
    dev["used_core"] = np.where(pres, rng.choice([50, 75, 100], dev["used_core"].shape), 0)
    dev["used_ratio"] = dev["used_core"]
    dev["used_memory"] = dev["total_memory"] * dev["used_ratio"] // 100
    return cluster, numa, dev, rsv, pods, preds, rng


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2])
def test_device_select_victims_ext_matches_oracle(seed):
    """Shipped-profile clusters (NUMA cpuset nodes, 8-GPU nodes, reservations) with taints / labels: one
    kg_pods_select_victims launch per pod over 32 candidates, random victim subsets (half holding a GPU share on one
    minor, some attributed to a reservation slot) in random reprieve order: reject bits, victims kept and
    numViolatingVictim equal the oracle's."""
    cluster, numa, dev, rsv, pods, preds, rng = _ext_world(64, 5100 + seed)
    cfg = F.build_config(profile=EXT)
    stats = {"kept": 0, "reprieved": 0, "rejected": 0, "device": 0, "numa": 0, "taint_aff": 0}
    with Engine(cfg, cluster.n) as e:
        # every victim's device share is decided before anything is loaded (the engine holds the same pods)
        all_minors = _victim_devices(cluster, dev, np.arange(len(cluster.existing_pods)), rng)
        synth.load_shipped_into(e, cluster, numa, dev, rsv)
        e.upsert_predicates(preds)
        st = oracle.states(cluster.n)
        oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
        for j in range(len(pods)):
            nodes = rng.choice(cluster.n, size=32, replace=False).astype(np.int32)
            vics, slots, viol, mins = [], [], [], []
            for i in nodes:
                on = rng.permutation(np.nonzero(cluster.existing_node == i)[0])
                on = on[:int(rng.integers(0, len(on) + 1))]
                vics.append(cluster.existing_pods[on])
                mins.append(all_minors[on])
                ns = int(rsv["n"][i])
                slots.append(np.where((rng.random(len(on)) < 0.3) & (ns > 0), rng.integers(0, max(ns, 1), len(on)),
                                      -1).astype(np.int32))
                viol.append((rng.random(len(on)) < 0.3).astype(np.uint8))
            rej, kept, nvio = e.select_victims(pods[j:j + 1], nodes, vics, slots, viol, mins)
            for c, i in enumerate(nodes):
                w = oracle.select_victims(cfg, cluster.nodes[i], cluster.metrics[i], st[i:i + 1], rsv[i], pods[j:j + 1],
                                          vics[c], slots[c], viol[c], cluster.now_ns, numa=numa[i], dev=dev[i],
                                          pred=preds[i], minors=mins[c])
                assert (int(rej[c]), kept[c].tolist(), int(nvio[c])) == (w[0], w[1].tolist(), w[2]), (j, c, i)
                if w[0] == 0:
                    stats["kept"] += int(w[1].sum())
                    stats["reprieved"] += int((~w[1]).sum())
                elif w[0] != abi.REJECT_NO_VICTIMS:
                    stats["rejected"] += 1
                    stats["device"] += bool(w[0] & abi.REJECT_DEVICE)
                    stats["numa"] += bool(w[0] & abi.REJECT_NUMA)
                    stats["taint_aff"] += bool(w[0] & (abi.REJECT_TAINT | abi.REJECT_NODE_AFFINITY))
    assert all(v > 0 for v in stats.values()), stats


@pytest.mark.gpu
def test_device_filter_preemption_ext_matches_oracle():
    """kg_pods_filter_preemption on the same worlds, one node per call, with and without the victims' minors."""
    cluster, numa, dev, rsv, pods, preds, rng = _ext_world(48, 5200)
    cfg = F.build_config(profile=EXT)
    all_minors = _victim_devices(cluster, dev, np.arange(len(cluster.existing_pods)), rng)
    seen = set()
    with Engine(cfg, cluster.n) as e:
        synth.load_shipped_into(e, cluster, numa, dev, rsv)
        e.upsert_predicates(preds)
        st = oracle.states(cluster.n)
        oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
        for j in range(len(pods)):
            for _ in range(4):
                i = int(rng.integers(cluster.n))
                on = np.nonzero(cluster.existing_node == i)[0]
                vic, mins = cluster.existing_pods[on], all_minors[on]
                for m in (mins, None):
                    got = e.filter_preemption(pods[j:j + 1], i, vic, None, m)
                    want = oracle.filter_preemption(cfg, cluster.nodes[i], cluster.metrics[i], st[i:i + 1], rsv[i],
                                                    pods[j:j + 1], vic, None, cluster.now_ns, numa=numa[i], dev=dev[i],
                                                    pred=preds[i], minors=m)
                    assert got == want, (j, i, got, want)
                    seen.add(want)
    assert len(seen) > 2, seen


@pytest.mark.gpu
def test_device_refuses_spread_and_gpu_reservations():
    cfg = F.build_config(profile=F.Profile(filter=(F.NODE_RESOURCES_FIT, F.POD_TOPOLOGY_SPREAD),
                                           score={F.NODE_RESOURCES_FIT: 1}))
    cl, _, pod, vic = case_allocate_from_preemptible()
    with Engine(cfg, 1) as e:
        synth.load_into(e, cl)
        with pytest.raises(Exception, match="PodTopologySpread"):
            e.filter_preemption(pod, 0, vic)
