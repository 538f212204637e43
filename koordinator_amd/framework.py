"""Host-side mirror of the reference's plugin surface for the accelerated path.

The reference's Go host (koord-scheduler) cannot run here (no Go toolchain); this module is the host layer
above the C ABI with the reference's names and argument meanings, so tests read like the reference's own:

* ``LoadAwareSchedulingArgs`` — pkg/scheduler/apis/config/types.go:30-76, defaults v1beta2/defaults.go:76-99.
* ``NodeResourcesFitArgs`` — upstream NodeResourcesFitArgs, scoringStrategy LeastAllocated.
* ``Profile`` — the score plugin set + weights of a KubeSchedulerConfiguration profile
  (config/manager/scheduler-config.yaml:82-91).
* ``make_node / make_node_metric / make_pod`` — what the Go shim decodes from corev1.Node, NodeMetric and
  corev1.Pod (allocatable, raw-allocatable and custom-usage-threshold annotations, PodRequestsAndLimits,
  GetPodPriorityClassWithDefault).
* ``Scheduler`` — SchedulePod for a FIFO queue (frameworkext SchedulePod interception,
  framework_extender_factory.go:136-185), RunFilterPlugins / RunScorePlugins for one pod
  (framework_extender.go:204-258), Reserve/Unreserve (kg_pods_add / kg_pods_remove).
Status codes mirror framework.Code: Success, Unschedulable.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import abi
from .engine import Engine
from .quantity import resource_value

SUCCESS, UNSCHEDULABLE = "Success", "Unschedulable"
NODE_RESOURCES_FIT, LOAD_AWARE, NODE_NUMA_RESOURCE = "NodeResourcesFit", "LoadAwareScheduling", "NodeNUMAResource"
DEVICE_SHARE = "DeviceShare"
RESERVATION = "Reservation"
# upstream default plugins a stock profile keeps (k8s v1.24.15 v1beta2 defaults: Score weight 1 each)
TAINT_TOLERATION, NODE_AFFINITY = "TaintToleration", "NodeAffinity"
BALANCED_ALLOCATION = "NodeResourcesBalancedAllocation"
IMAGE_LOCALITY = "ImageLocality"
# (ABI 12) hostname-keyed PodTopologySpread (default weight 2) and InterPodAffinity (default weight 1)
POD_TOPOLOGY_SPREAD, INTER_POD_AFFINITY = "PodTopologySpread", "InterPodAffinity"


def _slots(d: dict | None, absent=0) -> np.ndarray:
    out = np.full(abi.RES_MAX, absent, dtype=np.int64)
    for k, v in (d or {}).items():
        out[abi.RESOURCE_SLOTS[k]] = int(v)
    return out


@dataclass
class LoadAwareSchedulingArgs:
    filter_expired_node_metrics: bool = True
    node_metric_expiration_seconds: int | None = 180
    resource_weights: dict = field(default_factory=lambda: {"cpu": 1, "memory": 1})
    usage_thresholds: dict = field(default_factory=lambda: {"cpu": 65, "memory": 95})
    prod_usage_thresholds: dict = field(default_factory=dict)
    score_according_prod_usage: bool = False
    estimated_scaling_factors: dict = field(default_factory=lambda: {"cpu": 85, "memory": 70})
    # Aggregated (config/types.go:56-76): usage_thresholds / usage_type ("p95", ...) / usage_duration_s for Filter,
    # score_type / score_duration_s for Score; duration 0 = the longest period recorded
    aggregated: dict | None = None


@dataclass
class NodeResourcesFitArgs:
    scoring_resources: dict = field(default_factory=lambda: {"cpu": 1, "memory": 1})


@dataclass
class NodeNUMAResourceArgs:
    """pkg/scheduler/apis/config/types.go NodeNUMAResourceArgs; defaults v1beta2/defaults.go:101-137."""
    default_cpu_bind_policy: str = "FullPCPUs"
    scoring_strategy: str = "LeastAllocated"
    scoring_resources: dict = field(default_factory=lambda: {"cpu": 1, "memory": 1})
    numa_scoring_strategy: str = "LeastAllocated"
    numa_scoring_resources: dict = field(default_factory=lambda: {"cpu": 1, "memory": 1})


@dataclass
class DeviceShareArgs:
    """pkg/scheduler/apis/config/types.go DeviceShareArgs; defaults v1beta2/defaults.go:187-208 (LeastAllocated on
    gpu-memory-ratio / rdma / fpga, weight 1 — rdma and fpga weights only touch RDMA / FPGA devices)."""
    scoring_strategy: str = "LeastAllocated"
    scoring_resources: dict = field(default_factory=lambda: {"koordinator.sh/gpu-memory-ratio": 1,
                                                             "koordinator.sh/rdma": 1, "koordinator.sh/fpga": 1})


@dataclass
class Profile:
    filter: tuple = (NODE_RESOURCES_FIT, LOAD_AWARE)
    score: dict = field(default_factory=lambda: {NODE_RESOURCES_FIT: 1, LOAD_AWARE: 1})


def build_config(la: LoadAwareSchedulingArgs | None = None, fit: NodeResourcesFitArgs | None = None,
                 profile: Profile | None = None, batch_pods: int = 32, pods_per_wave: int = 8,
                 device_id: int = -1, numa: NodeNUMAResourceArgs | None = None,
                 deviceshare: DeviceShareArgs | None = None, pipeline_depth: int = 0,
                 balanced_resources: tuple = ("cpu", "memory"), hard_pod_affinity_weight: int = 1,
                 multi_rank: str = "auto") -> np.ndarray:
    """kg_config of a profile.  multi_rank (ABI 15): "shard" / "replica" / "auto" — how an engine of several ranks
    splits the work (kg_config.multi_rank_mode).  balanced_resources: NodeResourcesBalancedAllocationArgs.resources (v1beta2 default
    cpu + memory, weight 1 each; the weights do not enter the two-resource std).  hard_pod_affinity_weight:
    InterPodAffinityArgs.HardPodAffinityWeight (v1beta2 default 1)."""
    la = la or LoadAwareSchedulingArgs()
    fit = fit or NodeResourcesFitArgs()
    profile = profile or Profile()
    numa = numa or NodeNUMAResourceArgs()
    ds = deviceshare or DeviceShareArgs()
    c = np.zeros(1, dtype=abi.CONFIG_DTYPE)
    r = c[0]
    r["abi_version"] = abi.ABI_VERSION
    r["la_filter_expired_node_metrics"] = int(la.filter_expired_node_metrics)
    r["la_node_metric_expiration_seconds"] = -1 if la.node_metric_expiration_seconds is None else la.node_metric_expiration_seconds
    r["la_resource_weights"] = _slots(la.resource_weights)
    r["la_usage_thresholds"] = _slots(la.usage_thresholds)
    r["la_prod_usage_thresholds"] = _slots(la.prod_usage_thresholds)
    r["la_estimated_scaling_factors"] = _slots(la.estimated_scaling_factors)
    r["la_score_according_prod_usage"] = int(la.score_according_prod_usage)
    agg = la.aggregated or {}
    r["la_agg_usage_thresholds"] = _slots(agg.get("usage_thresholds"))
    r["la_agg_usage_type"] = abi.AGG_TYPES[agg.get("usage_type", "")]
    r["la_agg_usage_duration_ns"] = int(agg.get("usage_duration_s", 0) * 10**9)
    r["la_agg_score_type"] = abi.AGG_TYPES[agg.get("score_type", "")]
    r["la_agg_score_duration_ns"] = int(agg.get("score_duration_s", 0) * 10**9)
    r["fit_resource_weights"] = _slots(fit.scoring_resources)
    r["fit_filter"] = int(NODE_RESOURCES_FIT in profile.filter)
    r["la_filter"] = int(LOAD_AWARE in profile.filter)
    r["fit_score"] = int(NODE_RESOURCES_FIT in profile.score)
    r["la_score"] = int(LOAD_AWARE in profile.score)
    r["weight_fit"] = int(profile.score.get(NODE_RESOURCES_FIT, 0))
    r["weight_loadaware"] = int(profile.score.get(LOAD_AWARE, 0))
    r["batch_pods"] = batch_pods
    r["pods_per_wave"] = pods_per_wave
    r["device_id"] = device_id
    r["pipeline_depth"] = pipeline_depth
    r["numa_filter"] = int(NODE_NUMA_RESOURCE in profile.filter)
    r["numa_score"] = int(NODE_NUMA_RESOURCE in profile.score)
    r["weight_numa"] = int(profile.score.get(NODE_NUMA_RESOURCE, 0))
    r["numa_default_cpu_bind_policy"] = abi.BIND[numa.default_cpu_bind_policy]
    r["numa_scoring_strategy"] = abi.STRATEGY[numa.scoring_strategy]
    r["numa_scoring_weights"] = [numa.scoring_resources.get("cpu", 0), numa.scoring_resources.get("memory", 0)]
    r["numa_numa_scoring_strategy"] = abi.STRATEGY[numa.numa_scoring_strategy]
    r["numa_numa_scoring_weights"] = [numa.numa_scoring_resources.get("cpu", 0),
                                      numa.numa_scoring_resources.get("memory", 0)]
    r["ds_filter"] = int(DEVICE_SHARE in profile.filter)
    r["ds_score"] = int(DEVICE_SHARE in profile.score)
    r["weight_deviceshare"] = int(profile.score.get(DEVICE_SHARE, 0))
    r["reservation_filter"] = int(RESERVATION in profile.filter)
    r["reservation_score"] = int(RESERVATION in profile.score)
    r["weight_reservation"] = int(profile.score.get(RESERVATION, 0))
    r["taint_filter"] = int(TAINT_TOLERATION in profile.filter)
    r["taint_score"] = int(TAINT_TOLERATION in profile.score)
    r["weight_taint"] = int(profile.score.get(TAINT_TOLERATION, 0))
    r["affinity_filter"] = int(NODE_AFFINITY in profile.filter)
    r["affinity_score"] = int(NODE_AFFINITY in profile.score)
    r["weight_affinity"] = int(profile.score.get(NODE_AFFINITY, 0))
    r["balanced_score"] = int(BALANCED_ALLOCATION in profile.score)
    r["weight_balanced"] = int(profile.score.get(BALANCED_ALLOCATION, 0))
    r["balanced_resources"] = sum({"cpu": 1, "memory": 2}.get(k, 1 << 8) for k in balanced_resources)
    r["image_score"] = int(IMAGE_LOCALITY in profile.score)
    r["weight_image"] = int(profile.score.get(IMAGE_LOCALITY, 0))
    r["spread_filter"] = int(POD_TOPOLOGY_SPREAD in profile.filter)
    r["spread_score"] = int(POD_TOPOLOGY_SPREAD in profile.score)
    r["weight_spread"] = int(profile.score.get(POD_TOPOLOGY_SPREAD, 0))
    r["interpod_filter"] = int(INTER_POD_AFFINITY in profile.filter)
    r["interpod_score"] = int(INTER_POD_AFFINITY in profile.score)
    r["weight_interpod"] = int(profile.score.get(INTER_POD_AFFINITY, 0))
    r["hard_pod_affinity_weight"] = hard_pod_affinity_weight
    r["multi_rank_mode"] = abi.MULTI_RANK[multi_rank]
    r["ds_scoring_strategy"] = abi.STRATEGY[ds.scoring_strategy]
    r["ds_scoring_weights"] = [ds.scoring_resources.get("koordinator.sh/gpu-core", 0),
                               ds.scoring_resources.get("koordinator.sh/gpu-memory", 0),
                               ds.scoring_resources.get("koordinator.sh/gpu-memory-ratio", 0)]
    r["ds_scoring_weights_x"] = [ds.scoring_resources.get("koordinator.sh/rdma", 0),
                                 ds.scoring_resources.get("koordinator.sh/fpga", 0)]
    return c


def _values(resources: dict | None) -> np.ndarray:
    out = np.zeros(abi.RES_MAX, dtype=np.int64)
    for k, v in (resources or {}).items():
        out[abi.RESOURCE_SLOTS[k]] = resource_value(k, v)
    return out


def make_node(allocatable: dict, allowed_pods: int = 110, raw_allocatable: dict | None = None,
              custom_usage_thresholds: dict | None = None, custom_prod_usage_thresholds: dict | None = None,
              valid: bool = True, custom_aggregated: dict | None = None) -> np.ndarray:
    """custom_aggregated = the annotation's AggregatedUsage {usage_thresholds, usage_type, usage_duration_s}."""
    n = np.zeros(1, dtype=abi.NODE_DTYPE)
    r = n[0]
    r["allocatable"] = _values(allocatable)
    r["allowed_pods"] = allowed_pods
    flags = abi.NODE_VALID if valid else 0
    if raw_allocatable:
        flags |= abi.NODE_HAS_RAW_ALLOCATABLE
        r["raw_allocatable"] = _values(raw_allocatable)
        pres = np.zeros(abi.RES_MAX, dtype=np.int64)
        for k in raw_allocatable:
            pres[abi.RESOURCE_SLOTS[k]] = 1
        r["raw_allocatable_present"] = pres
    r["custom_usage_thresholds"] = _slots(custom_usage_thresholds, absent=-1)
    r["custom_prod_usage_thresholds"] = _slots(custom_prod_usage_thresholds, absent=-1)
    ca = custom_aggregated or {}
    r["custom_agg_thresholds"] = _slots(ca.get("usage_thresholds"), absent=-1)
    r["custom_agg_type"] = abi.AGG_TYPES[ca.get("usage_type", "")]
    r["custom_agg_duration_ns"] = int(ca.get("usage_duration_s", 0) * 10**9)
    if custom_usage_thresholds or custom_prod_usage_thresholds or custom_aggregated:
        flags |= abi.NODE_HAS_CUSTOM_THRESHOLDS
    r["flags"] = flags
    return n


def make_node_metric(present: bool = True, update_time_ns: int | None = 0, node_usage: dict | None = None,
                     prod_pods_usage: dict | None = None, pods_metric_count: int = 0,
                     aggregated: list | None = None, report_interval_ns: int = 0) -> np.ndarray:
    """NodeMetric status summary; node_usage=None means Status.NodeMetric == nil.  aggregated = the
    AggregatedNodeUsages [{"duration_s": .., "p95": {"cpu": .., "memory": ..}, ...}]."""
    m = np.zeros(1, dtype=abi.METRIC_DTYPE)
    r = m[0]
    r["present"] = int(present)
    r["has_update_time"] = int(update_time_ns is not None)
    r["update_time_unix_nano"] = update_time_ns or 0
    if node_usage is not None:
        r["has_node_metric"] = 1
        r["node_usage"] = _values(node_usage)
        pres = np.zeros(abi.RES_MAX, dtype=np.int64)
        for k in node_usage:
            pres[abi.RESOURCE_SLOTS[k]] = 1
        r["node_usage_present"] = pres
    r["pods_metric_count"] = pods_metric_count
    r["report_interval_ns"] = report_interval_ns  # CollectPolicy.ReportIntervalSeconds; 0 = the 60 s default
    r["prod_pods_usage"] = _values(prod_pods_usage)
    aggs = aggregated or []
    if len(aggs) > 4:
        raise ValueError("at most 4 AggregatedNodeUsages")
    r["agg_count"] = len(aggs)
    for i, a in enumerate(aggs):
        r["agg_duration_ns"][i] = int(a.get("duration_s", 0) * 10**9)
        for name, t in abi.AGG_TYPES.items():
            if t == 0 or name not in a:
                continue
            for k, v in a[name].items():
                slot = abi.RESOURCE_SLOTS[k]
                if slot < 2:
                    r["agg_usage"][i, t - 1, slot] = resource_value(k, v)
                    r["agg_present"][i, t - 1] |= 1 << slot
    return m


def make_node_numa(sockets: int = 0, nodes_per_socket: int = 1, cores_per_node: int = 0, cpus_per_core: int = 2,
                   numa_policy: str = "", node_cpu_bind_policy: str = "", numa_allocate_strategy: str | None = None,
                   numa_resources: list | None = None, reserved_cpus=(), allocated_cpus=(),
                   numa_allocated: dict | None = None, cpu_amplification_ratio: float = 0.0,
                   exclusive_pcpu_cpus=(), exclusive_numa_cpus=()) -> np.ndarray:
    """NodeNUMAResource view of a node: the NodeResourceTopology's CPU topology (buildCPUTopology numbering),
    policies and zones, and the NodeAllocation of already-bound pods. numa_resources = [{"cpu": .., "memory": ..}]
    per NUMA zone; numa_allocated = {zone: {"cpu": .., "memory": ..}}; cpu_amplification_ratio = the node's
    node.koordinator.sh/resource-amplification-ratio cpu (≤ 1 none; zone cpu is given amplified);
    exclusive_{pcpu,numa}_cpus = the allocated cpus whose holder's CPUExclusivePolicy is PCPULevel / NUMANodeLevel."""
    n = np.zeros(1, dtype=abi.NODE_NUMA_DTYPE)
    r = n[0]
    r["has_topology"] = int(sockets > 0)
    r["sockets"], r["nodes_per_socket"], r["cores_per_node"], r["cpus_per_core"] = (
        sockets, nodes_per_socket, cores_per_node, cpus_per_core)
    r["numa_policy"] = abi.NUMA_POLICY[numa_policy]
    r["node_cpu_bind_policy"] = abi.NODE_BIND[node_cpu_bind_policy]
    r["numa_allocate_strategy"] = -1 if numa_allocate_strategy is None else abi.STRATEGY[numa_allocate_strategy]
    zones = numa_resources or []
    r["num_numa"] = len(zones)
    for i, z in enumerate(zones):
        r["numa_cpu"][i] = resource_value("cpu", z.get("cpu", 0))
        r["numa_mem"][i] = resource_value("memory", z.get("memory", 0))
    for name, cpus in (("reserved_cpus", reserved_cpus), ("allocated_cpus", allocated_cpus),
                       ("exclusive_pcpu_cpus", exclusive_pcpu_cpus), ("exclusive_numa_cpus", exclusive_numa_cpus)):
        w = np.zeros(abi.MAX_CPUS // 64, dtype=np.uint64)
        for c in cpus:
            w[c // 64] |= np.uint64(1) << np.uint64(c % 64)
        r[name] = w
    for i, res in (numa_allocated or {}).items():
        r["numa_alloc_cpu"][i] = resource_value("cpu", res.get("cpu", 0))
        r["numa_alloc_mem"][i] = resource_value("memory", res.get("memory", 0))
    r["cpu_amplification_ratio"] = cpu_amplification_ratio
    return n


def cpuset_of(words) -> list:
    """The cpu ids of a 256-bit mask (uint64[4])."""
    out = []
    for w, v in enumerate(np.asarray(words, dtype=np.uint64).tolist()):
        for b in range(64):
            if (v >> b) & 1:
                out.append(64 * w + b)
    return out


def make_node_device(gpus: list | None = None, has_device: bool = True, rdma: list | None = None,
                     fpga: list | None = None) -> np.ndarray:
    """DeviceShare view of one node: gpus = [{"minor": m, "healthy": True, "total": {core, memory, ratio},
    "used": {core, memory, ratio}}, ...] in koordinator.sh/gpu-* units (core / ratio percent, memory bytes).
    (ABI 17) rdma / fpga = [{"minor": m, "healthy": True, "total": percent, "used": percent}, ...]."""
    d = np.zeros(1, dtype=abi.NODE_DEVICE_DTYPE)
    r = d[0]
    r["has_device"] = int(has_device)
    for t, devs in ((abi.XTYPE_RDMA, rdma), (abi.XTYPE_FPGA, fpga)):
        for g in devs or []:
            m = int(g["minor"])
            r["x_present"][t, m] = 1
            r["x_healthy"][t, m] = int(g.get("healthy", True))
            r["x_total"][t, m] = int(g.get("total", 0))
            r["x_used"][t, m] = int(g.get("used", 0))
    for g in gpus or []:
        m = int(g["minor"])
        r["present"][m] = 1
        r["healthy"][m] = int(g.get("healthy", True))
        t, u = g.get("total", {}), g.get("used", {})
        r["total_core"][m], r["total_memory"][m], r["total_ratio"][m] = t.get("core", 0), t.get("memory", 0), t.get("ratio", 0)
        r["used_core"][m], r["used_memory"][m], r["used_ratio"][m] = u.get("core", 0), u.get("memory", 0), u.get("ratio", 0)
    return d


QUOTA_RESOURCES = ("cpu", "memory", "nvidia.com/gpu", "dcu.com/gpu", "koordinator.sh/gpu", "koordinator.sh/gpu-core",
                   "koordinator.sh/gpu-memory", "koordinator.sh/gpu-memory-ratio")


def make_quota(used_limit: dict | None = None, used: dict | None = None, min: dict | None = None,
               non_preemptible_used: dict | None = None) -> np.ndarray:
    """One ElasticQuota (kg_quota) over QUOTA_RESOURCES: {"cpu": milli, "memory": bytes, "koordinator.sh/gpu-core":
    .., ...} lists; a key absent from used_limit / min does not constrain (quotav1.LessThanOrEqual compares only the
    limit's keys)."""
    q = np.zeros(1, dtype=abi.QUOTA_DTYPE)
    r = q[0]
    for f, d, absent in (("used", used, 0), ("non_preemptible_used", non_preemptible_used, 0),
                         ("used_limit", used_limit, -1), ("min", min, -1)):
        d = d or {}
        r[f] = [int(d.get(k, absent)) for k in QUOTA_RESOURCES]
    return q


def make_pod(requests: dict | None = None, limits: dict | None = None, priority_class: str = "",
             daemonset: bool = False, nonzero: tuple | None = None, qos: str = "",
             required_cpu_bind_policy: str = "", preferred_cpu_bind_policy: str = "",
             devices: dict | None = None, quota_id: int = 0, non_preemptible: bool = False,
             preferred_cpu_exclusive_policy: str = "") -> np.ndarray:
    """One single-container pod. nonzero = schedutil.GetNonzeroRequests (100m / 200MiB defaults); qos = the
    koordinator.sh/qosClass label; *_cpu_bind_policy / preferred_cpu_exclusive_policy = the
    scheduling.koordinator.sh/resource-spec annotation."""
    p = np.zeros(1, dtype=abi.POD_DTYPE)
    r = p[0]
    req = _values(requests)
    r["requests"] = req
    r["limits"] = _values(limits)
    if nonzero is None:
        nonzero = (req[abi.RES_CPU] or 100, req[abi.RES_MEMORY] or 200 * 1024 * 1024)
    r["nonzero_requests"] = nonzero
    r["priority_class"] = abi.PRIORITY_CLASSES[priority_class]
    r["flags"] = (abi.POD_DAEMONSET if daemonset else 0) | (abi.POD_NON_PREEMPTIBLE if non_preemptible else 0)
    r["quota_id"] = quota_id  # 1 + index into the ElasticQuota table (0: the pod has no quota)
    r["qos"] = abi.QOS[qos]
    r["required_cpu_bind_policy"] = abi.BIND[required_cpu_bind_policy]
    r["preferred_cpu_bind_policy"] = abi.BIND[preferred_cpu_bind_policy]
    r["preferred_cpu_exclusive_policy"] = abi.EXCL[preferred_cpu_exclusive_policy]
    for k, v in (devices or {}).items():  # device resources: PodRequestsAndLimits of e.g. koordinator.sh/gpu-core
        r["device_requests"][abi.DEVICE_RESOURCE_SLOTS[k]] = int(v)
    return p


@dataclass
class ScheduleResult:
    suggested_host: int          # node index, -1 = FitError (unschedulable)
    score: int
    evaluated_nodes: int
    feasible_nodes: int = -1


class Scheduler:
    """SchedulePod / RunFilterPlugins / RunScorePlugins over the GPU engine."""

    def __init__(self, config: np.ndarray, capacity: int, **kw):
        self.config = config
        self.engine = Engine(config, capacity, **kw)

    def close(self):
        self.engine.close()

    def run_filter_plugins(self, pod: np.ndarray) -> dict:
        rej, _, _ = self.engine.evaluate(pod)
        c = self.config[0]
        out = {}
        if c["fit_filter"]:
            out[NODE_RESOURCES_FIT] = np.where(rej & (abi.REJECT_FIT_PODS | abi.REJECT_FIT_CPU | abi.REJECT_FIT_MEMORY),
                                               UNSCHEDULABLE, SUCCESS)
        if c["la_filter"]:
            out[LOAD_AWARE] = np.where(rej & abi.REJECT_LOADAWARE, UNSCHEDULABLE, SUCCESS)
        return out

    def run_score_plugins(self, pod: np.ndarray) -> dict:
        _, fit, la = self.engine.evaluate(pod)
        c = self.config[0]
        out = {}
        if c["fit_score"]:
            out[NODE_RESOURCES_FIT] = fit
        if c["la_score"]:
            out[LOAD_AWARE] = la
        return out

    def schedule_pods(self, pods: np.ndarray):
        return self.engine.schedule(pods)

    def schedule_pod(self, pod: np.ndarray) -> ScheduleResult:
        node, score, _ = self.engine.schedule(np.asarray(pod).reshape(1))
        return ScheduleResult(int(node[0]), int(score[0]), self.engine.num_nodes)

    def reserve(self, pod: np.ndarray, node_idx: int):
        self.engine.add_pods(np.asarray(pod).reshape(1), [node_idx])

    def unreserve(self, pod: np.ndarray, node_idx: int):
        self.engine.remove_pods(np.asarray(pod).reshape(1), [node_idx])
