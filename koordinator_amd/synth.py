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


def load_into(engine, cluster: Cluster):
    """Informer-order ingest: nodes, NodeMetrics, then the already-assigned pods."""
    engine.upsert_nodes(cluster.nodes)
    engine.update_metrics(cluster.metrics, cluster.now_ns)
    if len(cluster.existing_pods):
        engine.add_pods(cluster.existing_pods, cluster.existing_node)
