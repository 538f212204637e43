"""Seeded synthetic clusters and pod queues, identical for the GPU engine and the oracle.

Nodes: allocatable cpu ∈ {32,64,96,128} cores, memory ∈ {128,256,512,1024} GiB, 110 pods.  Pre-existing
assigned pods fill 0–50 % of cpu/memory requests.  NodeMetric on 95 % of nodes (cpu usage 0–80 %, memory
0–90 %), UpdateTime 10 s before `now` (never expires), PodsMetric empty; 5 % of nodes carry a
custom-usage-thresholds annotation.  Pods: cpu ∈ {250m,500m,1,2,4,8}, memory ∈ {256Mi..32Gi}, limit =
request (50 %) or 2×request, QoS LS 80 % / BE 10 % / LSR 10 % with matching koord priority classes.
All quantities integral (milli-cpu, bytes).  Seeds are recorded by callers (bench.py, tests).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import abi

GI = 1 << 30
MI = 1 << 20
T0_NS = 1_700_000_000 * 10**9  # fixed NodeMetric epoch
BASE_SEED = 20250117


@dataclass
class Cluster:
    nodes: np.ndarray           # NODE_DTYPE[n]
    metrics: np.ndarray         # METRIC_DTYPE[n]
    existing_pods: np.ndarray   # POD_DTYPE[m]
    existing_node: np.ndarray   # int32[m]
    now_ns: int

    @property
    def n(self) -> int:
        return len(self.nodes)


def make_cluster(n_nodes: int, seed: int = BASE_SEED, pods_per_node: float = 6.0, metric_frac: float = 0.95,
                 custom_frac: float = 0.05, invalid_frac: float = 0.0) -> Cluster:
    rng = np.random.default_rng(seed)
    n = n_nodes
    nodes = np.zeros(n, dtype=abi.NODE_DTYPE)
    cpu = rng.choice(np.array([32, 64, 96, 128], dtype=np.int64), n) * 1000
    mem = rng.choice(np.array([128, 256, 512, 1024], dtype=np.int64), n) * GI
    nodes["allocatable"][:, abi.RES_CPU] = cpu
    nodes["allocatable"][:, abi.RES_MEMORY] = mem
    nodes["allowed_pods"] = 110
    flags = np.full(n, abi.NODE_VALID, dtype=np.int64)
    if invalid_frac > 0:
        flags[rng.random(n) < invalid_frac] = 0
    custom = rng.random(n) < custom_frac
    nodes["custom_usage_thresholds"] = -1
    nodes["custom_prod_usage_thresholds"] = -1
    nodes["custom_usage_thresholds"][custom, abi.RES_CPU] = rng.integers(40, 90, custom.sum())
    nodes["custom_usage_thresholds"][custom, abi.RES_MEMORY] = rng.integers(70, 100, custom.sum())
    flags[custom] |= abi.NODE_HAS_CUSTOM_THRESHOLDS
    nodes["flags"] = flags

    # pre-existing assigned pods: k per node, requests sized so totals are ~U(0, 0.5) of allocatable
    k = rng.poisson(pods_per_node, n).clip(0, 60)
    m = int(k.sum())
    owner = np.repeat(np.arange(n, dtype=np.int32), k)
    frac_cpu = rng.random(n) * 0.5
    frac_mem = rng.random(n) * 0.5
    share = rng.random(m) + 0.05
    share_sum = np.bincount(owner, weights=share, minlength=n)
    w = share / np.maximum(share_sum[owner], 1e-9)
    ex = np.zeros(m, dtype=abi.POD_DTYPE)
    ex_cpu = np.maximum(1, np.floor(w * frac_cpu[owner] * cpu[owner])).astype(np.int64)
    ex_mem = np.maximum(1, np.floor(w * frac_mem[owner] * mem[owner] / MI)).astype(np.int64) * MI
    ex["requests"][:, abi.RES_CPU] = ex_cpu
    ex["requests"][:, abi.RES_MEMORY] = ex_mem
    burst = rng.random(m) < 0.5
    ex["limits"][:, abi.RES_CPU] = np.where(burst, 2 * ex_cpu, ex_cpu)
    ex["limits"][:, abi.RES_MEMORY] = np.where(burst, 2 * ex_mem, ex_mem)
    ex["nonzero_requests"][:, 0] = ex_cpu
    ex["nonzero_requests"][:, 1] = ex_mem
    ex["priority_class"] = _priority(rng, m, lsr=0.1)

    now = T0_NS + 10 * 10**9
    metrics = np.zeros(n, dtype=abi.METRIC_DTYPE)
    has = rng.random(n) < metric_frac
    metrics["present"] = has
    metrics["has_update_time"] = has
    metrics["has_node_metric"] = has
    metrics["update_time_unix_nano"] = np.where(has, T0_NS, 0)
    metrics["node_usage"][:, abi.RES_CPU] = np.where(has, np.floor(rng.random(n) * 0.8 * cpu), 0).astype(np.int64)
    metrics["node_usage"][:, abi.RES_MEMORY] = (np.where(has, np.floor(rng.random(n) * 0.9 * mem / MI), 0)
                                                .astype(np.int64) * MI)
    metrics["node_usage_present"][:, abi.RES_CPU] = has
    metrics["node_usage_present"][:, abi.RES_MEMORY] = has
    return Cluster(nodes, metrics, ex, owner, now)


def _priority(rng, m, lsr=0.1):
    """QoS LS 80 % → koord-prod, BE 10 % → koord-batch, LSR `lsr` → koord-prod (labels pin the class)."""
    u = rng.random(m)
    pc = np.full(m, abi.PRIO_PROD, dtype=np.int64)
    pc[(u >= 0.8) & (u < 0.9)] = abi.PRIO_BATCH
    return pc


def make_pods(n_pods: int, seed: int = BASE_SEED + 1) -> np.ndarray:
    rng = np.random.default_rng(seed)
    p = np.zeros(n_pods, dtype=abi.POD_DTYPE)
    cpu = rng.choice(np.array([250, 500, 1000, 2000, 4000, 8000], dtype=np.int64), n_pods)
    mem = rng.choice(np.array([256, 512, 1024, 2048, 4096, 8192, 16384, 32768], dtype=np.int64), n_pods) * MI
    burst = rng.random(n_pods) < 0.5
    p["requests"][:, abi.RES_CPU] = cpu
    p["requests"][:, abi.RES_MEMORY] = mem
    p["limits"][:, abi.RES_CPU] = np.where(burst, 2 * cpu, cpu)
    p["limits"][:, abi.RES_MEMORY] = np.where(burst, 2 * mem, mem)
    p["nonzero_requests"][:, 0] = cpu
    p["nonzero_requests"][:, 1] = mem
    p["priority_class"] = _priority(rng, n_pods)
    return p


POD_STREAM_CHUNK = 1 << 16


def make_pods_stream(n_pods: int, seed: int = BASE_SEED + 1) -> np.ndarray:
    """(r6) The `make_pods` distribution, prefix-stable: chunk k of 65,536 pods is `make_pods(65536)` seeded with
    SeedSequence([seed, k]), so the first m pods are the same whatever `n_pods` is.  The C3 bench and the 1M-pod
    parity test draw their queue here, which lets one committed oracle fixture (tests/golden/c3_queue.npz) cover any
    prefix the bench times."""
    k = -(-n_pods // POD_STREAM_CHUNK)
    parts = [make_pods(POD_STREAM_CHUNK, seed=np.random.SeedSequence([seed, i])) for i in range(k)]
    if not parts:
        return np.zeros(0, dtype=abi.POD_DTYPE)
    return np.concatenate(parts)[:n_pods]


def make_stream(make, n_pods: int, seed: int, chunk: int = POD_STREAM_CHUNK) -> np.ndarray:
    """(r6) Any queue generator made prefix-stable: chunk k of `chunk` pods is make(chunk, seed=s_k) with s_k an int
    drawn from SeedSequence([seed, k]).  The C4 / shipped benches draw their queues here so one committed oracle
    fixture (tests/golden/make_bench_fixture.py) covers every prefix they time."""
    k = -(-n_pods // chunk)
    parts = [make(chunk, seed=int(np.random.SeedSequence([seed, i]).generate_state(1)[0])) for i in range(k)]
    if not parts:
        return np.zeros(0, dtype=abi.POD_DTYPE)
    return np.concatenate(parts)[:n_pods]


def load_into(engine, cluster: Cluster):
    """Informer-order ingest: nodes, NodeMetrics, then the already-assigned pods."""
    engine.upsert_nodes(cluster.nodes)
    engine.update_metrics(cluster.metrics, cluster.now_ns)
    if len(cluster.existing_pods):
        engine.add_pods(cluster.existing_pods, cluster.existing_node)


# ---- config C4: NodeNUMAResource cpuset / NUMA topology (2-socket 256-cpu nodes, LSR/LSE pods) --------------
def make_numa_cluster(n_nodes: int, seed: int = BASE_SEED + 4) -> tuple:
    """(Cluster, kg_node_numa[n]) for config C4.  Every node: 2 sockets, 256 cpus (SMT-2) in buildCPUTopology
    numbering — 80 % as 1 NUMA node per socket × 64 cores, 20 % as 2 NUMA nodes per socket × 32 cores — with
    1 TiB of memory split evenly over the NUMA zones.  NodeAllocation: 0–40 % of the cores held by bound
    cpuset pods (whole cores at random positions) + 0–40 % of each zone's memory; 20 % of nodes reserve cpus
    0-1.  NUMA policy none 50 % / BestEffort 20 % / Restricted 15 % / SingleNUMANode 15 %; node cpu-bind
    policy FullPCPUsOnly 10 % / SpreadByPCPUs 5 %; NUMA allocate strategy label Least 10 % / Most 10 %.
    Bound pods also count in NodeInfo.Requested (plus 0–10 % non-cpuset cpu).  NodeMetric as make_cluster."""
    rng = np.random.default_rng(seed)
    n = n_nodes
    nodes = np.zeros(n, dtype=abi.NODE_DTYPE)
    nodes["allocatable"][:, abi.RES_CPU] = 256_000
    nodes["allocatable"][:, abi.RES_MEMORY] = 1024 * GI
    nodes["allowed_pods"] = 250
    nodes["flags"] = abi.NODE_VALID
    nodes["custom_usage_thresholds"] = -1
    nodes["custom_prod_usage_thresholds"] = -1
    numa = np.zeros(n, dtype=abi.NODE_NUMA_DTYPE)
    four = rng.random(n) < 0.2
    numa["has_topology"] = 1
    numa["sockets"] = 2
    numa["nodes_per_socket"] = np.where(four, 2, 1)
    numa["cores_per_node"] = np.where(four, 32, 64)
    numa["cpus_per_core"] = 2
    u = rng.random(n)
    numa["numa_policy"] = np.select([u < 0.5, u < 0.7, u < 0.85], [abi.NUMA_POLICY[""], abi.NUMA_POLICY["BestEffort"],
                                    abi.NUMA_POLICY["Restricted"]], abi.NUMA_POLICY["SingleNUMANode"])
    u = rng.random(n)
    numa["node_cpu_bind_policy"] = np.select([u < 0.10, u < 0.15], [abi.NODE_BIND["FullPCPUsOnly"],
                                             abi.NODE_BIND["SpreadByPCPUs"]], abi.NODE_BIND[""])
    u = rng.random(n)
    numa["numa_allocate_strategy"] = np.select([u < 0.1, u < 0.2], [abi.STRATEGY["LeastAllocated"],
                                               abi.STRATEGY["MostAllocated"]], -1)
    zones = np.where(four, 4, 2)
    numa["num_numa"] = zones
    req_cpu = np.zeros(n, dtype=np.int64)
    req_mem = np.zeros(n, dtype=np.int64)
    for i in range(n):
        z = int(zones[i])
        zmem = 1024 * GI // z
        numa["numa_cpu"][i, :z] = 256_000 // z
        numa["numa_mem"][i, :z] = zmem
        held = rng.random(128) < rng.random() * 0.4        # cores held by bound cpuset pods
        cpus = np.flatnonzero(np.repeat(held, 2))
        words = np.zeros(4, dtype=np.uint64)
        for c in cpus:
            words[c // 64] |= np.uint64(1) << np.uint64(c % 64)
        numa["allocated_cpus"][i] = words
        per_zone = np.bincount(cpus // (256 // z), minlength=z)[:z] * 1000
        numa["numa_alloc_cpu"][i, :z] = per_zone
        zm = (np.floor(rng.random(z) * 0.4 * zmem / MI).astype(np.int64)) * MI
        numa["numa_alloc_mem"][i, :z] = zm
        if rng.random() < 0.2:
            numa["reserved_cpus"][i, 0] = np.uint64(3) if not (int(words[0]) & 3) else np.uint64(0)
        req_cpu[i] = int(per_zone.sum()) + int(rng.random() * 0.1 * 256_000)
        req_mem[i] = int(zm.sum())
    ex = np.zeros(n, dtype=abi.POD_DTYPE)
    ex["requests"][:, abi.RES_CPU] = req_cpu
    ex["requests"][:, abi.RES_MEMORY] = req_mem
    ex["limits"] = ex["requests"]
    ex["nonzero_requests"][:, 0] = np.maximum(req_cpu, 100)
    ex["nonzero_requests"][:, 1] = np.maximum(req_mem, 200 * MI)
    ex["priority_class"] = abi.PRIO_PROD
    keep = (req_cpu > 0) | (req_mem > 0)
    now = T0_NS + 10 * 10**9
    metrics = np.zeros(n, dtype=abi.METRIC_DTYPE)
    has = rng.random(n) < 0.95
    metrics["present"] = has
    metrics["has_update_time"] = has
    metrics["has_node_metric"] = has
    metrics["update_time_unix_nano"] = np.where(has, T0_NS, 0)
    metrics["node_usage"][:, abi.RES_CPU] = np.where(has, np.floor(rng.random(n) * 0.6 * 256_000), 0).astype(np.int64)
    metrics["node_usage"][:, abi.RES_MEMORY] = (np.where(has, np.floor(rng.random(n) * 0.9 * 1024 * GI / MI), 0)
                                                .astype(np.int64) * MI)
    metrics["node_usage_present"][:, abi.RES_CPU] = has
    metrics["node_usage_present"][:, abi.RES_MEMORY] = has
    cluster = Cluster(nodes, metrics, ex[keep], np.flatnonzero(keep).astype(np.int32), now)
    return cluster, numa


def make_numa_pods(n_pods: int, seed: int = BASE_SEED + 5) -> np.ndarray:
    """Config C4 queue: 60 % LSR and 10 % LSE koord-prod pods with whole-core cpu requests {1,2,3,4,8,16} (cpu
    bind: required FullPCPUs 20 %, preferred SpreadByPCPUs 20 %, else the default FullPCPUs), 25 % LS koord-prod
    and 4 % BE koord-batch pods with fractional cpu, 1 % zero-request pods; memory 256Mi–32Gi."""
    rng = np.random.default_rng(seed)
    p = np.zeros(n_pods, dtype=abi.POD_DTYPE)
    u = rng.random(n_pods)
    cpuset = u < 0.7
    cores = rng.choice(np.array([1, 2, 3, 4, 8, 16], dtype=np.int64), n_pods)
    frac = rng.choice(np.array([250, 500, 1500, 2000, 4000], dtype=np.int64), n_pods)
    cpu = np.where(cpuset, cores * 1000, frac)
    mem = rng.choice(np.array([256, 1024, 4096, 8192, 16384, 32768], dtype=np.int64), n_pods) * MI
    zero = (u >= 0.99)
    cpu[zero] = 0
    mem[zero] = 0
    p["requests"][:, abi.RES_CPU] = cpu
    p["requests"][:, abi.RES_MEMORY] = mem
    p["limits"] = p["requests"]
    p["nonzero_requests"][:, 0] = np.where(cpu > 0, cpu, 100)
    p["nonzero_requests"][:, 1] = np.where(mem > 0, mem, 200 * MI)
    p["priority_class"] = np.where((u >= 0.95) & (u < 0.99), abi.PRIO_BATCH, abi.PRIO_PROD)
    p["qos"] = np.select([u < 0.6, u < 0.7, u < 0.95], [abi.QOS["LSR"], abi.QOS["LSE"], abi.QOS["LS"]], abi.QOS["BE"])
    b = rng.random(n_pods)
    p["required_cpu_bind_policy"] = np.where(cpuset & (b < 0.2), abi.BIND["FullPCPUs"], abi.BIND[""])
    p["preferred_cpu_bind_policy"] = np.where(cpuset & (b >= 0.2) & (b < 0.4), abi.BIND["SpreadByPCPUs"], abi.BIND[""])
    return p


def load_numa_into(engine, cluster: Cluster, numa: np.ndarray):
    load_into(engine, cluster)
    engine.upsert_numa(numa)


# ---- config C5 (DeviceShare part): GPU nodes, GPU-sharing pods ------------------------------------------------
GPU_MEM = 80 * GI


def make_gpu_cluster(n_nodes: int, seed: int = BASE_SEED + 6) -> tuple:
    """(Cluster, kg_node_device[n]) for config C5's DeviceShare part: make_cluster's nodes and NodeMetrics, each
    node with 8 GPUs (gpu-core 100, gpu-memory-ratio 100, gpu-memory 80 GiB) of which 0–60 % (in steps of 5)
    is used per minor; 1 % of the GPUs unhealthy, 1 % of the nodes without a Device object."""
    cluster = make_cluster(n_nodes, seed=seed)
    return cluster, make_node_devices(n_nodes, seed=seed + 1000)


def make_node_devices(n_nodes: int, seed: int) -> np.ndarray:
    """kg_node_device[n]: 8 GPUs per node (gpu-core 100, gpu-memory-ratio 100, gpu-memory 80 GiB), 0–60 % (steps of 5)
    used per minor, 1 % of the GPUs unhealthy, 1 % of the nodes without a Device object."""
    rng = np.random.default_rng(seed)
    n = n_nodes
    dev = np.zeros(n, dtype=abi.NODE_DEVICE_DTYPE)
    dev["has_device"] = rng.random(n) >= 0.01
    dev["present"] = 1
    dev["healthy"] = rng.random((n, abi.MAX_MINORS)) >= 0.01
    dev["total_core"] = 100
    dev["total_ratio"] = 100
    dev["total_memory"] = GPU_MEM
    used = rng.integers(0, 13, size=(n, abi.MAX_MINORS)) * 5
    dev["used_core"] = used
    dev["used_ratio"] = used
    dev["used_memory"] = used * GPU_MEM // 100
    for f in ("present", "healthy", "total_core", "total_ratio", "total_memory", "used_core", "used_ratio", "used_memory"):
        dev[f][dev["has_device"] == 0] = 0  # no Device object: no device state at all
    return dev


def make_gpu_pods(n_pods: int, seed: int = BASE_SEED + 7, base: np.ndarray | None = None) -> np.ndarray:
    """Config C5 queue: make_pods' cpu/memory pods (or `base`), 30 % of them also requesting GPU share —
    gpu-memory-ratio ∈ {25, 50, 100, 200} with the same gpu-core (70 %), gpu-memory-ratio alone (20 %) or gpu-memory
    bytes (10 %)."""
    p = make_pods(n_pods, seed=seed) if base is None else base
    rng = np.random.default_rng(seed + 1000)
    gpu = rng.random(n_pods) < 0.3
    ratio = rng.choice(np.array([25, 50, 100, 200], dtype=np.int64), n_pods)
    kind = rng.random(n_pods)
    dr = p["device_requests"]
    core_ratio = gpu & (kind < 0.7)
    ratio_only = gpu & (kind >= 0.7) & (kind < 0.9)
    mem_only = gpu & (kind >= 0.9)
    dr[:, abi.DEV_GPU_CORE] = np.where(core_ratio, ratio, 0)
    dr[:, abi.DEV_GPU_MEMORY_RATIO] = np.where(core_ratio | ratio_only, ratio, 0)
    dr[:, abi.DEV_GPU_MEMORY] = np.where(mem_only, ratio * GPU_MEM // 100, 0)
    return p


def add_x_devices(dev: np.ndarray, frac: float = 0.5, seed: int = BASE_SEED + 26) -> None:
    """(ABI 17) RDMA / FPGA devices, in place: `frac` of the nodes with a Device object get 1–4 RDMA NICs and, half of
    them, 1–2 FPGAs at minors 0.., each koordinator.sh/rdma / fpga 100 with 0–100 % (steps of 25) used, 2 % unhealthy."""
    rng = np.random.default_rng(seed)
    for i in np.nonzero(dev["has_device"] != 0)[0]:
        if rng.random() >= frac:
            continue
        for t, k in ((abi.XTYPE_RDMA, int(rng.integers(1, 5))), (abi.XTYPE_FPGA, int(rng.integers(1, 3)) * int(rng.random() < 0.5))):
            for m in range(k):
                dev["x_present"][i, t, m] = 1
                dev["x_healthy"][i, t, m] = int(rng.random() >= 0.02)
                dev["x_total"][i, t, m] = 100
                dev["x_used"][i, t, m] = int(rng.integers(0, 5)) * 25


def add_x_requests(pods: np.ndarray, frac: float = 0.3, seed: int = BASE_SEED + 27) -> None:
    """(ABI 17) RDMA / FPGA requests, in place: `frac` of the pods request koordinator.sh/rdma ∈ {25, 50, 100, 200}
    (a fifth of them also koordinator.sh/fpga 50 or 100), with or without a GPU share."""
    rng = np.random.default_rng(seed)
    n = len(pods)
    x = rng.random(n) < frac
    pods["device_requests"][:, abi.DEV_RDMA] = np.where(x, rng.choice([25, 50, 100, 200], n), 0)
    f = x & (rng.random(n) < 0.2)
    pods["device_requests"][:, abi.DEV_FPGA] = np.where(f, rng.choice([50, 100], n), 0)


def load_gpu_into(engine, cluster: Cluster, dev: np.ndarray):
    load_into(engine, cluster)
    engine.upsert_devices(dev)


def amplify_numa_cluster(cluster: Cluster, numa: np.ndarray, frac: float = 0.3, seed: int = BASE_SEED + 5):
    """CPU amplification (node.koordinator.sh/resource-amplification-ratio cpu ∈ {1.5, 2.0, 2.5}) on `frac` of
    make_numa_cluster's nodes, as the NodeResource controller leaves them: node allocatable cpu and each NUMA zone's
    cpu amplified (Amplify: ceil in float64, apis/extension/node_resource_amplification.go:170-175), the bound
    cpuset pods' NUMA allocations unchanged.  In place; returns the ratios."""
    rng = np.random.default_rng(seed)
    n = cluster.n
    on = rng.random(n) < frac
    ratio = np.where(on, rng.choice(np.array([1.5, 2.0, 2.5]), n), 0.0)
    amp = lambda v, r: np.where(r > 1, np.ceil(v.astype(np.float64) * r), v).astype(np.int64)
    cores = cluster.nodes["allocatable"][:, abi.RES_CPU] // 1000
    cluster.nodes["allocatable"][:, abi.RES_CPU] = amp(cores, ratio) * 1000
    zc = numa["numa_cpu"] // 1000
    numa["numa_cpu"] = amp(zc, ratio[:, None]) * 1000
    numa["cpu_amplification_ratio"] = ratio
    return ratio


# ---- config C5: Reservation matching (50k nodes; 0–4 reservations on 30 % of nodes, owner label selectors) -----
N_OWNERS = 64  # owner groups (reservations sharing an owner spec); a pod carries the bitmask of the groups it matches


def make_rsv_cluster(n_nodes: int, seed: int = BASE_SEED + 8, cluster: Cluster | None = None) -> tuple:
    """(Cluster, kg_node_reservations[n]) for config C5's Reservation part: make_cluster's nodes (or `cluster`), 30 %
    of them with 1–4 Available reservations (cpu {2,4,8,16} cores, memory {4..64} GiB — 8 % of them cpu-only and 4 %
    memory-only —, owner group 0..63, 40 % carrying an order label, policy Default 60 % / Aligned 20 % / Restricted
    20 %, 20 % AllocateOnce).  Each reservation's reserve pod sits in NodeInfo (requests = allocatable, an absent key's
    non-zero request = the 100m / 200MiB default, KG_POD_RESERVE) and 0–2 pods are already assigned to it (in NodeInfo
    and the LoadAware assign cache, accounted in Allocated)."""
    cluster = cluster if cluster is not None else make_cluster(n_nodes, seed=seed)
    rng = np.random.default_rng(seed + 1000)
    n = n_nodes
    rsv = np.zeros(n, dtype=abi.NODE_RSV_DTYPE)
    has = rng.random(n) < 0.3
    rsv["n"] = np.where(has, rng.integers(1, abi.MAX_RSV_SLOTS + 1, n), 0)
    S = abi.MAX_RSV_SLOTS
    cpu = rng.choice(np.array([2, 4, 8, 16], dtype=np.int64), (n, S)) * 1000
    mem = rng.choice(np.array([4, 8, 16, 32, 64], dtype=np.int64), (n, S)) * GI
    kind = rng.random((n, S))
    cpu = np.where(kind >= 0.96, 0, cpu)                  # memory-only
    mem = np.where((kind >= 0.88) & (kind < 0.96), 0, mem)  # cpu-only
    on = np.arange(S)[None, :] < rsv["n"][:, None]
    rsv["allocatable_cpu"] = np.where(on, cpu, 0)
    rsv["allocatable_mem"] = np.where(on, mem, 0)
    rsv["owner"] = np.where(on, rng.integers(0, N_OWNERS, (n, S)), 0)
    rsv["order"] = np.where(on & (rng.random((n, S)) < 0.4), rng.integers(1, 1000, (n, S)), 0)
    u = rng.random((n, S))
    rsv["policy"] = np.where(on, np.where(u < 0.6, 0, np.where(u < 0.8, 1, 2)), 0)
    rsv["allocate_once"] = on & (rng.random((n, S)) < 0.2)
    rsv["available"] = on
    # pods already assigned to reservations: 0–2 per reservation, each a quarter of it
    k = np.where(on, rng.integers(0, 3, (n, S)), 0)
    k = np.where(rsv["allocate_once"].astype(bool), np.minimum(k, 1), k)
    rsv["assigned"] = k
    rsv["allocated_cpu"] = k * (cpu // 4) * on
    rsv["allocated_mem"] = k * (mem // 4) * on
    extra_pods, extra_node = [], []
    ii, ss = np.nonzero(on)
    for i, s in zip(ii.tolist(), ss.tolist()):
        rp = np.zeros(1, dtype=abi.POD_DTYPE)[0]
        rp["requests"][abi.RES_CPU] = rp["limits"][abi.RES_CPU] = cpu[i, s]
        rp["requests"][abi.RES_MEMORY] = rp["limits"][abi.RES_MEMORY] = mem[i, s]
        rp["nonzero_requests"][0] = cpu[i, s] if cpu[i, s] else 100
        rp["nonzero_requests"][1] = mem[i, s] if mem[i, s] else 200 * MI
        rp["priority_class"] = abi.PRIO_PROD
        rp["flags"] = abi.POD_RESERVE
        extra_pods.append(rp)
        extra_node.append(i)
        for _ in range(int(k[i, s])):
            ap = np.zeros(1, dtype=abi.POD_DTYPE)[0]
            ac, am = (cpu[i, s] or 4000) // 4, (mem[i, s] or 8 * GI) // 4
            ap["requests"][abi.RES_CPU] = ap["limits"][abi.RES_CPU] = ap["nonzero_requests"][0] = ac
            ap["requests"][abi.RES_MEMORY] = ap["limits"][abi.RES_MEMORY] = ap["nonzero_requests"][1] = am
            ap["priority_class"] = abi.PRIO_PROD
            extra_pods.append(ap)
            extra_node.append(i)
    if extra_pods:
        cluster.existing_pods = np.concatenate([cluster.existing_pods, np.array(extra_pods, dtype=abi.POD_DTYPE)])
        cluster.existing_node = np.concatenate([cluster.existing_node, np.array(extra_node, dtype=np.int32)])
    return cluster, rsv


def owner_masks(rng, n_pods: int, frac: float = 0.2, n_groups: int = N_OWNERS) -> np.ndarray:
    """Owner-group bitmasks for a queue: `frac` of the pods match one group, a quarter of those a second one."""
    owned = rng.random(n_pods) < frac
    g1 = rng.integers(0, n_groups, n_pods)
    g2 = rng.integers(0, n_groups, n_pods)
    two = owned & (rng.random(n_pods) < 0.25)
    m = np.where(owned, np.left_shift(np.int64(1), g1), 0)
    return (m | np.where(two, np.left_shift(np.int64(1), g2), 0)).astype(np.int64)


def make_rsv_pods(n_pods: int, seed: int = BASE_SEED + 9, base: np.ndarray | None = None) -> np.ndarray:
    """Config C5 Reservation queue: make_pods' pods (or `base`), 20 % owned (matching one owner group's label
    selectors, a quarter of them a second group's), a quarter of those with a required reservation affinity."""
    p = make_pods(n_pods, seed=seed) if base is None else base
    rng = np.random.default_rng(seed + 1000)
    p["reservation_owner_mask"] = owner_masks(rng, n_pods)
    owned = p["reservation_owner_mask"] != 0
    p["reservation_flags"] = np.where(owned & (rng.random(n_pods) < 0.25), abi.POD_RSV_AFFINITY, 0)
    return p


def add_reservation_affinity(rsv: np.ndarray, pods: np.ndarray, seed: int = BASE_SEED + 23) -> None:
    """(ABI 12) Labels and required reservation affinities, in place: each node gets topology.kubernetes.io/zone
    z0..z3, each reservation reservation-type ∈ {a, b, c} (a fifth also zone = its own "z-pinned" value, overlaying the
    node's); half of the pods with a required reservation affinity carry a reservationSelector on reservation-type
    and a third of the others ReservationSelectorTerms (type In {a, b} / zone In {z0, z1}, ORed) — compiled through
    PredicateTable as a caller would (affinities interned first, then the slots' fakeNode predicates)."""
    from .predicates import PredicateTable, ZONE
    rng = np.random.default_rng(seed)
    t = PredicateTable()
    aff = np.nonzero(pods["reservation_flags"] & abi.POD_RSV_AFFINITY)[0]
    kind = rng.random(len(aff))
    for j, k in zip(aff, kind):
        if k < 0.5:
            t.fill_reservation_affinity(pods[j:j + 1], selector={"reservation-type": "abc"[rng.integers(3)]})
        elif k < 0.67:
            t.fill_reservation_affinity(pods[j:j + 1], required_terms=[
                {"matchExpressions": [{"key": "reservation-type", "operator": "In", "values": ["a", "b"]}]},
                {"matchExpressions": [{"key": ZONE, "operator": "In", "values": ["z0", "z1"]}]}])
    n = len(rsv)
    zone = rng.integers(0, 4, n)
    for i in np.nonzero(rsv["n"] > 0)[0]:
        node_labels = {ZONE: f"z{zone[i]}"}
        for s in range(int(rsv["n"][i])):
            labels = {"reservation-type": "abc"[rng.integers(3)]}
            if rng.random() < 0.2:
                labels[ZONE] = "z-pinned"
            rsv["predicates"][i, s] = t.reservation_predicates(node_labels, labels, f"r-{i}-{s}")
        rsv["predicate_count"][i] = len(t.preds)  # ABI 12: the predicates the slots were compiled against


def load_rsv_into(engine, cluster: Cluster, rsv: np.ndarray):
    load_into(engine, cluster)
    engine.upsert_reservations(rsv)


# ---- config C5 (one profile): Reservation + DeviceShare + ElasticQuota ------------------------------------------
N_QUOTAS = 16


def make_c5_cluster(n_nodes: int, seed: int = BASE_SEED + 10, gpu_rsv_frac: float = 0.0) -> tuple:
    """(Cluster, kg_node_device[n], kg_node_reservations[n]) for config C5 as one profile: make_gpu_cluster's GPU nodes
    with make_rsv_cluster's reservations on top (cpu / memory reservations; the reserve pods in NodeInfo).
    gpu_rsv_frac > 0 (ABI 13): that fraction of the reservations on nodes with a Device object also hold GPUs
    (add_gpu_reservations)."""
    cluster, dev = make_gpu_cluster(n_nodes, seed=seed)
    cluster, rsv = make_rsv_cluster(n_nodes, seed=seed + 1, cluster=cluster)
    if gpu_rsv_frac > 0:
        add_gpu_reservations(dev, rsv, gpu_rsv_frac, seed=seed + 3)
    return cluster, dev, rsv


def add_gpu_reservations(dev: np.ndarray, rsv: np.ndarray, frac: float, seed: int = BASE_SEED + 24) -> None:
    """(ABI 13) Reservations holding GPUs, in place: `frac` of the reservations on nodes with a Device object get a
    reserve pod allocation of 1–2 healthy minors, gpu-memory-ratio ∈ {25, 50, 100} each (gpu-core the same, gpu-memory
    the ratio's bytes); each of the reservation's assigned pods used a quarter of it on its first minor, half of them
    on the second too (appendAllocatedByHints: the allocations inside the reservation's minors).  Every allocation
    is added to the node's deviceUsed, as the bound reserve pod and assigned pods are in nodeDevice.deviceUsed; a minor
    may end up over-used (used > total), which calcFreeWithPreemptible clamps."""
    rng = np.random.default_rng(seed)
    S = abi.MAX_RSV_SLOTS
    for i in np.nonzero((rsv["n"] > 0) & (dev["has_device"] != 0))[0]:
        ok = np.nonzero(dev["healthy"][i] & dev["present"][i])[0]
        if len(ok) == 0:
            continue
        for s in range(int(rsv["n"][i])):
            if rng.random() >= frac:
                continue
            k = 1 if rng.random() < 0.7 or len(ok) < 2 else 2
            minors = rng.choice(ok, k, replace=False)
            ratio = int(rng.choice([25, 50, 100]))
            for m in minors:
                rsv["gpu_alloc"][i, s, m] = (ratio, ratio * GPU_MEM // 100, ratio)
            rsv["gpu_minors"][i, s] = int(sum(1 << int(m) for m in minors))
            a = rsv["gpu_allocated"][i, s]
            for q in range(int(rsv["assigned"][i, s])):
                share = ratio // 4
                for t, m in enumerate(minors):
                    if t == 0 or q % 2 == 0:
                        a[m] += (share, share * GPU_MEM // 100, share)
            for m in range(abi.MAX_MINORS):
                al, ad = rsv["gpu_alloc"][i, s, m], rsv["gpu_allocated"][i, s, m]
                dev["used_core"][i, m] += al[0] + ad[0]
                dev["used_memory"][i, m] += al[1] + ad[1]
                dev["used_ratio"][i, m] += al[2] + ad[2]


def make_c5_pods(n_pods: int, seed: int = BASE_SEED + 11) -> np.ndarray:
    """Config C5 queue: make_gpu_pods (30 % GPU-share) with make_rsv_pods' owner masks / affinities (20 % owned) and
    N_QUOTAS ElasticQuota groups (80 % of the pods in one)."""
    p = make_rsv_pods(n_pods, seed=seed + 1, base=make_gpu_pods(n_pods, seed=seed))
    rng = np.random.default_rng(seed + 2000)
    p["quota_id"] = np.where(rng.random(n_pods) < 0.8, rng.integers(1, N_QUOTAS + 1, n_pods), 0)
    return p


def make_c5_quotas(pods: np.ndarray, seed: int = BASE_SEED + 12, n_quotas: int = N_QUOTAS,
                   share: float = 1.0) -> np.ndarray:
    """kg_quota[n_quotas] whose limits run out during the queue: used_limit ≈ U(0.3, 1.2) · `share` of each
    quota's total demand on cpu / memory / gpu-core / gpu-memory-ratio (gpu-memory absent 50 %), min = 1/4 of it."""
    rng = np.random.default_rng(seed)
    q = np.zeros(n_quotas, dtype=abi.QUOTA_DTYPE)
    q["used_limit"] = -1
    q["min"] = -1
    req = np.zeros((len(pods), abi.QUOTA_RES), dtype=np.int64)
    req[:, 0] = pods["requests"][:, abi.RES_CPU]
    req[:, 1] = pods["requests"][:, abi.RES_MEMORY]
    req[:, 2:] = pods["device_requests"][:, :abi.QUOTA_RES - 2]
    for k in range(n_quotas):
        mine = pods["quota_id"] == k + 1
        demand = req[mine].sum(axis=0)
        for d in (0, 1, 2 + abi.DEV_GPU_CORE, 2 + abi.DEV_GPU_MEMORY_RATIO, 2 + abi.DEV_GPU_MEMORY):
            if d == 2 + abi.DEV_GPU_MEMORY and rng.random() < 0.5:
                continue
            lim = int(demand[d] * share * rng.uniform(0.3, 1.2))
            q["used_limit"][k, d] = lim
            q["min"][k, d] = lim // 4
    return q


def load_c5_into(engine, cluster: Cluster, dev: np.ndarray, rsv: np.ndarray, quotas: np.ndarray | None = None):
    load_into(engine, cluster)
    engine.upsert_devices(dev)
    engine.upsert_reservations(rsv)
    if quotas is not None:
        engine.set_quotas(quotas)


# ---- the reference's shipped profile (config/manager/scheduler-config.yaml:66-117): LoadAwareScheduling +
# NodeNUMAResource + DeviceShare + Reservation (+ the upstream NodeResourcesFit) with ElasticQuota admission ------------
def make_shipped_cluster(n_nodes: int, seed: int = BASE_SEED + 13) -> tuple:
    """(Cluster, kg_node_numa[n], kg_node_device[n], kg_node_reservations[n]): make_numa_cluster's 2-socket 256-cpu
    nodes (NUMA policies, bound cpuset pods, NodeMetrics), each with make_node_devices' 8 GPUs, and make_rsv_cluster's
    cpu / memory reservations on 30 % of them (reserve pods in NodeInfo, no cpuset)."""
    cluster, numa = make_numa_cluster(n_nodes, seed=seed)
    dev = make_node_devices(n_nodes, seed=seed + 1000)
    cluster, rsv = make_rsv_cluster(n_nodes, seed=seed + 1, cluster=cluster)
    return cluster, numa, dev, rsv


def add_cpuset_reservations(numa: np.ndarray, rsv: np.ndarray, frac: float = 0.3,
                            seed: int = BASE_SEED + 25) -> int:
    """(ABI 15) Reservations holding cpusets, in place: `frac` of the reservations with a whole-core cpu allocatable on
    nodes with a valid topology get a reserve pod cpuset of that many cpus — whole free cores (neither allocated nor
    kubelet-reserved) at random positions — added to the node's NodeAllocation (allocated cpus; allocatedResources cpu
    of their NUMA nodes, as make_numa_cluster accounts bound cpuset pods).  The reservation's assigned pods hold the
    first ⌊assigned·|R|/4⌋ of those cpus (cpus_assigned, RefCount 2 in NodeAllocation), and a tenth of the reservations
    hand one more single cpu to them (a half core stays reserved, the FullPCPUs edge of takePreferredCPUs).  Returns the
    number of cpuset reservations."""
    rng = np.random.default_rng(seed)
    made = 0
    for i in np.nonzero((rsv["n"] > 0) & (numa["has_topology"] != 0))[0]:
        total = int(numa["sockets"][i] * numa["nodes_per_socket"][i] * numa["cores_per_node"][i] *
                    numa["cpus_per_core"][i])
        cpc = int(numa["cpus_per_core"][i])
        per_numa = total // max(int(numa["num_numa"][i]), 1)
        for s in range(int(rsv["n"][i])):
            need = int(rsv["allocatable_cpu"][i, s]) // 1000
            if need == 0 or need * 1000 != rsv["allocatable_cpu"][i, s] or need % cpc or rng.random() >= frac:
                continue
            held = np.zeros(total, dtype=bool)
            for w in range(4):
                a = int(numa["allocated_cpus"][i, w]) | int(numa["reserved_cpus"][i, w])
                for b in range(64):
                    if 64 * w + b < total and (a >> b) & 1:
                        held[64 * w + b] = True
            free_cores = np.flatnonzero(~held.reshape(-1, cpc).any(axis=1))
            if len(free_cores) < need // cpc:
                continue
            cores = np.sort(rng.choice(free_cores, need // cpc, replace=False))
            cpus = (cores[:, None] * cpc + np.arange(cpc)[None, :]).ravel()
            for c in cpus:
                rsv["cpus"][i, s, c // 64] |= np.uint64(1) << np.uint64(c % 64)
                numa["allocated_cpus"][i, c // 64] |= np.uint64(1) << np.uint64(c % 64)
            z = int(numa["num_numa"][i])
            if z > 0:
                numa["numa_alloc_cpu"][i, :z] += np.bincount(cpus // per_numa, minlength=z)[:z] * 1000
            k = int(rsv["assigned"][i, s]) * len(cpus) // 4
            if k > 0 and rng.random() < 0.1:
                k += 1
            for c in cpus[:min(k, len(cpus))]:
                rsv["cpus_assigned"][i, s, c // 64] |= np.uint64(1) << np.uint64(c % 64)
            made += 1
    return made


def make_shipped_pods(n_pods: int, seed: int = BASE_SEED + 14) -> np.ndarray:
    """The shipped profile's queue: make_numa_pods' LSR / LSE cpuset and LS / BE pods, 30 % also requesting GPU share
    (make_gpu_pods), 20 % owned by reservation owner groups (make_rsv_pods) and 80 % in one of N_QUOTAS quotas."""
    p = make_numa_pods(n_pods, seed=seed)
    p = make_gpu_pods(n_pods, seed=seed + 1, base=p)
    p = make_rsv_pods(n_pods, seed=seed + 2, base=p)
    rng = np.random.default_rng(seed + 3000)
    p["quota_id"] = np.where(rng.random(n_pods) < 0.8, rng.integers(1, N_QUOTAS + 1, n_pods), 0)
    return p


def load_shipped_into(engine, cluster: Cluster, numa: np.ndarray, dev: np.ndarray, rsv: np.ndarray,
                      quotas: np.ndarray | None = None):
    load_into(engine, cluster)
    engine.upsert_numa(numa)
    engine.upsert_devices(dev)
    engine.upsert_reservations(rsv)
    if quotas is not None:
        engine.set_quotas(quotas)


def make_predicates(n_nodes: int, pods: np.ndarray, seed: int = BASE_SEED + 15, no_zone: float = 0.0) -> tuple:
    """Node labels / taints and pod tolerations / nodeSelector / node affinity for TaintToleration + NodeAffinity
    (compiled through koordinator_amd.predicates).  Fills `pods` in place; returns (table, NODE_PRED_DTYPE[n_nodes])."""
    from .predicates import PredicateTable, NO_SCHEDULE, NO_EXECUTE, PREFER_NO_SCHEDULE
    rng = np.random.default_rng(seed)
    zones, pools = ["z0", "z1", "z2", "z3"], ["general", "compute", "memory"]
    labels, taints = [], []
    for i in range(n_nodes):
        lb = {"topology.kubernetes.io/zone": zones[rng.integers(4)], "pool": pools[rng.integers(3)],
              "rack": str(int(rng.integers(20)))}
        if no_zone and rng.random() < no_zone:  # (r4) nodes without a zone label: zone spread rejects / ignores them
            del lb["topology.kubernetes.io/zone"]
        if rng.random() < 0.3:
            lb["ssd"] = "true"
        labels.append(lb)
        ts = []
        u = rng.random()
        if u < 0.12:
            ts.append({"key": "dedicated", "value": ["infra", "batch"][rng.integers(2)], "effect": NO_SCHEDULE})
        elif u < 0.16:
            ts.append({"key": "maintenance", "value": "", "effect": NO_EXECUTE})
        for k in ("spot", "noisy", "legacy"):
            if rng.random() < 0.2:
                ts.append({"key": k, "value": "true", "effect": PREFER_NO_SCHEDULE})
        taints.append(ts)
    table = PredicateTable()
    for ts in taints:  # intern the cluster's taints first: pods' tolerated masks cover them
        for t in ts:
            table.taint_id(t["key"], t.get("value", ""), t["effect"])
    expr = lambda k, op, v=None: {"key": k, "operator": op, **({"values": v} if v is not None else {})}
    for j in range(len(pods)):
        tol = []
        u = rng.random()
        if u < 0.15:
            tol.append({"key": "dedicated", "operator": "Equal", "value": "batch", "effect": NO_SCHEDULE})
        elif u < 0.2:
            tol.append({"operator": "Exists"})  # tolerates everything
        if rng.random() < 0.4:
            tol.append({"key": ["spot", "noisy", "legacy"][rng.integers(3)], "operator": "Exists"})
        sel = {"pool": pools[rng.integers(3)]} if rng.random() < 0.2 else None
        req = None
        u = rng.random()
        if u < 0.25:
            req = [{"matchExpressions": [expr("topology.kubernetes.io/zone", "In", list(rng.choice(zones, 2,
                                                                                                  replace=False)))]}]
            if rng.random() < 0.5:
                req.append({"matchExpressions": [expr("rack", "Gt", [["4", "9", "14"][rng.integers(3)]]),
                                                 expr("ssd", "Exists")]})
        elif u < 0.3:
            req = [{"matchExpressions": [expr("pool", "NotIn", ["memory"]), expr("ssd", "DoesNotExist")]}]
        pref = []
        if rng.random() < 0.5:
            for _ in range(int(rng.integers(1, 4))):
                c = rng.integers(4)
                term = ({"matchExpressions": [expr("ssd", "Exists")]} if c == 0 else
                        {"matchExpressions": [expr("topology.kubernetes.io/zone", "In", [zones[rng.integers(4)]])]}
                        if c == 1 else
                        {"matchExpressions": [expr("rack", "Lt", [["5", "10", "15"][rng.integers(3)]])]} if c == 2 else
                        {"matchExpressions": [expr("pool", "In", ["compute"]), expr("ssd", "Exists")]})
                pref.append((int(rng.integers(1, 101)), term))
        table.fill_pod(pods[j:j + 1], tolerations=tol, node_selector=sel, required_terms=req, preferred=pref)
    rows = np.concatenate([table.node_row(labels[i], taints[i], name=f"node-{i}") for i in range(n_nodes)])
    return table, rows


def make_images(n_nodes: int, pods: np.ndarray, preds: np.ndarray, seed: int = BASE_SEED + 16):
    """Node images and pod containers for ImageLocality (compiled through koordinator_amd.predicates.ImageTable):
    a 40-image catalog (50 MiB - 2 GiB, some listed under two names), 5-15 images per node, 1-3 containers per pod
    (untagged names resolve to ':latest'; 5 % name an image no node holds).  Fills `pods` and preds["images"] in
    place; returns the table."""
    from .predicates import ImageTable
    rng = np.random.default_rng(seed)
    mib = 1024 * 1024
    catalog = []
    for k in range(40):
        names = [f"registry.local/app-{k}:v{k % 3}"] + ([f"registry.local/app-{k}:latest"] if k % 4 == 0 else [])
        catalog.append((names, int(rng.integers(50, 2048)) * mib + int(rng.integers(0, mib))))
    node_images = []
    for _ in range(n_nodes):
        pick = rng.choice(len(catalog), int(rng.integers(5, 16)), replace=False)
        node_images.append([catalog[int(c)] for c in pick])
    table = ImageTable(node_images)
    for j in range(len(pods)):
        cont = []
        for _ in range(int(rng.integers(1, 4))):
            if rng.random() < 0.05:
                cont.append("registry.local/unknown:v9")
            else:
                k = int(rng.integers(40))
                cont.append(f"registry.local/app-{k}" if k % 4 == 0 and rng.random() < 0.5 else catalog[k][0][0])
        table.fill_pod(pods[j:j + 1], cont)
    preds["images"] = [table.node_mask(i) for i in range(n_nodes)]
    preds["image_count"] = table.image_count()
    return table


# ---- (ABI 12) PodTopologySpread / InterPodAffinity (hostname key) ------------------------------------------------
def make_pod_groups(pods: np.ndarray, seed: int = BASE_SEED + 17, n_apps: int = 8, zones: bool = False,
                    ipa_zones: bool | None = None, system_default: float = 0.0) -> np.ndarray:
    """Fills the ABI 12 group fields of `pods` in place, as PodGroupTable would compile them for a workload of n_apps
    deployments (groups 1..n_apps: app=k in the namespace) in n_apps / 2 teams (groups n_apps+1..: team=t): every pod
    matches its app and team; 40 % carry a DoNotSchedule hostname spread constraint on their app (maxSkew 1-3), 50 % a
    ScheduleAnyway one (maxSkew 1-5), with `zones` also 15 % a DoNotSchedule zone one (maxSkew 1-39) and 40 % a
    ScheduleAnyway zone one (maxSkew 1-7), in a random order; 15 % a required anti-affinity to their own app (one per
    node), 10 % a required
    affinity to another team, 30 % one or two preferred (anti-)affinity terms (weights ±1..100).  ipa_zones (default:
    `zones`) re-keys InterPodAffinity terms to topology.kubernetes.io/zone: a third of the required anti-affinity pods
    (one per zone, or a node without the label), half of the required affinity pods (a fifth of them with both keys),
    half of the preferred terms."""
    rng = np.random.default_rng(seed)
    n = len(pods)
    n_teams = n_apps // 2
    app = rng.integers(0, n_apps, n)
    team = app // 2
    pods["match_groups"] = (1 << app) | (1 << (n_apps + team))
    # spread constraints (≤ 4, in pod order): hostname / zone × DoNotSchedule / ScheduleAnyway, each with probability
    # p; zone ones only with `zones` (the nodes carry topology.kubernetes.io/zone)
    kinds = [(abi.SPREAD_HARD, 0.4, 1, 4), (0, 0.5, 1, 6)]
    if zones:
        kinds += [(abi.SPREAD_HARD | abi.SPREAD_ZONE, 0.15, 1, 40), (abi.SPREAD_ZONE, 0.4, 1, 8)]
    nsp = np.zeros(n, dtype=np.int64)
    order = np.argsort(rng.random((n, len(kinds))), axis=1)  # a random constraint order per pod
    for kk in range(len(kinds)):
        flag, prob, lo, hi = kinds[kk]
        on = rng.random(n) < prob
        skew = rng.integers(lo, hi, n)
        for j in np.nonzero(on)[0]:
            c = nsp[j]
            pods["spread_group"][j, c] = app[j] + 1
            pods["spread_max_skew"][j, c] = skew[j]
            pods["spread_flags"][j, c] = flag
            nsp[j] += 1
    for j in range(n):  # shuffle each pod's constraints (the raw Score sums them in the pod's order)
        c = nsp[j]
        if c > 1:
            perm = order[j][order[j] < c]
            for f in ("spread_group", "spread_max_skew", "spread_flags"):
                pods[f][j, :c] = pods[f][j, perm]
    # (ABI 13) a fraction of the pods without constraints of their own get the plugin's system defaults on their app
    # (hostname maxSkew 3 + zone maxSkew 5, ScheduleAnyway, flagged KG_SPREAD_SYSTEM_DEFAULT); drawn after everything
    # above so the rest of the workload is unchanged
    if system_default > 0:
        sd = (nsp == 0) & (np.random.default_rng(seed + 991).random(n) < system_default)
        for j in np.nonzero(sd)[0]:
            cons = [(0, 3)] + ([(abi.SPREAD_ZONE, 5)] if zones else [])
            for c, (flag, skew) in enumerate(cons):
                pods["spread_group"][j, c] = app[j] + 1
                pods["spread_max_skew"][j, c] = skew
                pods["spread_flags"][j, c] = flag | abi.SPREAD_SYSTEM_DEFAULT
            nsp[j] = len(cons)
    pods["n_spread"] = nsp
    anti = rng.random(n) < 0.15
    pods["pod_anti_affinity"] = np.where(anti, 1 << app, 0)
    aff = rng.random(n) < 0.10
    other = (team + rng.integers(1, n_teams, n)) % n_teams
    pods["pod_affinity_group"] = np.where(aff, n_apps + other + 1, 0)
    pods["pod_affinity_terms"] = np.where(aff, 1 << (n_apps + other), 0)
    npref = np.where(rng.random(n) < 0.3, rng.integers(1, 3, n), 0)
    pods["n_pod_preferred"] = npref
    for t in range(2):
        on = npref > t
        g = rng.integers(1, n_apps + n_teams + 1, n)
        w = rng.integers(1, 101, n) * np.where(rng.random(n) < 0.4, -1, 1)
        pods["pod_preferred_group"][:, t] = np.where(on, g, 0)
        pods["pod_preferred_weight"][:, t] = np.where(on, w, 0)
    if zones if ipa_zones is None else ipa_zones:
        za = anti & (rng.random(n) < 1 / 3)
        pods["pod_anti_affinity_zone"] = np.where(za, pods["pod_anti_affinity"], 0)
        pods["pod_anti_affinity"] = np.where(za, 0, pods["pod_anti_affinity"])
        kind = rng.random(n)  # < 0.4: zone only, < 0.5: both keys
        terms = pods["pod_affinity_terms"].copy()
        pods["pod_affinity_terms_zone"] = np.where(aff & (kind < 0.5), terms, 0)
        pods["pod_affinity_terms"] = np.where(aff & (kind < 0.4), 0, terms)
        pz = (rng.random((n, 2)) < 0.5) & (npref[:, None] > np.arange(2))
        pods["pod_preferred_zone"] = pz[:, 0] * 1 + pz[:, 1] * 2
    return pods
