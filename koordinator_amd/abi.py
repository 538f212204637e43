"""ctypes/numpy mirror of include/koordgpu.h.

Every ABI struct is a run of int64 fields, so a numpy structured dtype with the same field order IS the C
layout; arrays of nodes / metrics / pods are passed to the library as plain pointers (the same memory a
cgo caller would hand over).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

RES_MAX = 8
RES_CPU, RES_MEMORY, RES_EPHEMERAL, RES_BATCH_CPU, RES_BATCH_MEMORY, RES_MID_CPU, RES_MID_MEMORY = range(7)
RESOURCE_SLOTS = {
    "cpu": RES_CPU,
    "memory": RES_MEMORY,
    "ephemeral-storage": RES_EPHEMERAL,
    "kubernetes.io/batch-cpu": RES_BATCH_CPU,
    "kubernetes.io/batch-memory": RES_BATCH_MEMORY,
    "kubernetes.io/mid-cpu": RES_MID_CPU,
    "kubernetes.io/mid-memory": RES_MID_MEMORY,
}

PRIO_NONE, PRIO_PROD, PRIO_MID, PRIO_BATCH, PRIO_FREE = range(5)
PRIORITY_CLASSES = {"": PRIO_NONE, "koord-prod": PRIO_PROD, "koord-mid": PRIO_MID,
                    "koord-batch": PRIO_BATCH, "koord-free": PRIO_FREE}

OK, E_INVALID, E_DEVICE, E_COLLECTIVE, E_NOMEM, E_UNSUPPORTED = 0, -1, -2, -3, -4, -5
REJECT_FIT_PODS, REJECT_FIT_CPU, REJECT_FIT_MEMORY, REJECT_LOADAWARE, REJECT_INVALID_NODE = 1, 2, 4, 8, 16
NODE_VALID, NODE_HAS_RAW_ALLOCATABLE, NODE_HAS_CUSTOM_THRESHOLDS = 1, 2, 4
POD_DAEMONSET, POD_NON_PREEMPTIBLE, POD_RESERVE = 1, 2, 4
POD_REQUEST_KEYS, POD_CPU_KEY, POD_MEM_KEY = 8, 16, 32
POD_TAINT_TABLE = 64
MAX_OWNER_GROUPS = 64
QUOTA_RES = 8
MAX_QUOTAS = 64
ABI_VERSION = 17
MAX_RSV_SLOTS = 4
RSV_POLICY = {"Default": 0, "Aligned": 1, "Restricted": 2}
POD_RSV_AFFINITY, POD_RSV_OPERATING = 1, 2
PROF_KINDS = 16
PROF_NAMES = {0: "eval_round", 1: "merge_round", 2: "resolve_round", 3: "ds_max_round", 4: "ds_norm_reduce",
              5: "rsv_eval", 6: "rsv_select", 7: "rsv_apply"}
MAX_NUMA, MAX_CPUS = 4, 256
MULTI_RANK = {"auto": 0, "shard": 1, "replica": 2}  # (ABI 15) kg_config.multi_rank_mode
QOS = {"": 0, "LSE": 1, "LSR": 2, "LS": 3, "BE": 4, "SYSTEM": 5}
BIND = {"": 0, "Default": 1, "FullPCPUs": 2, "SpreadByPCPUs": 3, "ConstrainedBurst": 4}
EXCL = {"": 0, "None": 0, "PCPULevel": 1, "NUMANodeLevel": 2}  # CPUExclusivePolicy
NODE_BIND = {"": 0, "None": 0, "FullPCPUsOnly": 1, "SpreadByPCPUs": 2}
NUMA_POLICY = {"": 0, "BestEffort": 1, "Restricted": 2, "SingleNUMANode": 3}
STRATEGY = {"LeastAllocated": 0, "MostAllocated": 1}
REJECT_NUMA = 32
REJECT_DEVICE = 64
RSV_EVAL_WORDS = 16  # KG_RSV_EVAL_WORDS: kg_pods_evaluate_reservation per node
DBG_MERGE_WORDS = 32  # KG_DBG_MERGE_WORDS: one kg_debug_numa_merge case
REJECT_FIT_OTHER = 128  # NodeResourcesFit: ephemeral-storage / a scalar resource (RES_EPHEMERAL .. RES_MID_MEMORY)
REJECT_RESERVATION = 256  # Reservation Filter (kg_pods_filter_preemption)
REJECT_SPREAD = 512  # (ABI 12) PodTopologySpread
REJECT_INTERPOD = 1024  # (ABI 12) InterPodAffinity
REJECT_NO_VICTIMS = 2048  # (ABI 14) kg_pods_select_victims: the candidate has no potential victims
REJECT_TAINT = 4096  # (ABI 16) TaintToleration in the preemption dry run
REJECT_NODE_AFFINITY = 8192  # (ABI 16) NodeAffinity in the preemption dry run
# DeviceShare device resources (KG_DEV_*)
DEV_RES_MAX, MAX_MINORS = 8, 8
DEV_XTYPES, XTYPE_RDMA, XTYPE_FPGA = 2, 0, 1  # (ABI 17) the default handler's device types
MAX_AFF_TERMS = 4  # KG_MAX_AFF_TERMS
MAX_CONTAINERS = 8  # KG_MAX_CONTAINERS
MAX_MATCH_GROUPS = 16  # KG_MAX_MATCH_GROUPS (ABI 12)
MAX_POD_PREFERRED = 4  # KG_MAX_POD_PREFERRED (ABI 12)
MAX_SPREAD = 4  # KG_MAX_SPREAD (ABI 12)
MAX_ZONES = 64  # KG_MAX_ZONES (ABI 12)
SPREAD_HARD, SPREAD_ZONE, SPREAD_SYSTEM_DEFAULT = 1, 2, 4  # KG_SPREAD_* (SYSTEM_DEFAULT: ABI 13)
DEV_NVIDIA_GPU, DEV_HYGON_DCU, DEV_KOORD_GPU, DEV_GPU_CORE, DEV_GPU_MEMORY, DEV_GPU_MEMORY_RATIO, DEV_FPGA, DEV_RDMA = \
    range(8)
DEVICE_RESOURCE_SLOTS = {
    "nvidia.com/gpu": DEV_NVIDIA_GPU, "dcu.com/gpu": DEV_HYGON_DCU, "koordinator.sh/gpu": DEV_KOORD_GPU,
    "koordinator.sh/gpu-core": DEV_GPU_CORE, "koordinator.sh/gpu-memory": DEV_GPU_MEMORY,
    "koordinator.sh/gpu-memory-ratio": DEV_GPU_MEMORY_RATIO, "koordinator.sh/fpga": DEV_FPGA,
    "koordinator.sh/rdma": DEV_RDMA,
}


def _i64(name, n=None):
    return (name, np.int64) if n is None else (name, np.int64, n if isinstance(n, tuple) else (n,))


CONFIG_DTYPE = np.dtype([
    _i64("abi_version"),
    _i64("la_filter_expired_node_metrics"),
    _i64("la_node_metric_expiration_seconds"),
    _i64("la_resource_weights", RES_MAX),
    _i64("la_usage_thresholds", RES_MAX),
    _i64("la_prod_usage_thresholds", RES_MAX),
    _i64("la_estimated_scaling_factors", RES_MAX),
    _i64("la_score_according_prod_usage"),
    _i64("fit_resource_weights", RES_MAX),
    _i64("fit_filter"), _i64("fit_score"), _i64("la_filter"), _i64("la_score"),
    _i64("weight_fit"), _i64("weight_loadaware"),
    _i64("numa_filter"), _i64("numa_score"), _i64("weight_numa"), _i64("numa_default_cpu_bind_policy"),
    _i64("numa_scoring_strategy"), _i64("numa_scoring_weights", 2),
    _i64("numa_numa_scoring_strategy"), _i64("numa_numa_scoring_weights", 2),
    _i64("ds_filter"), _i64("ds_score"), _i64("weight_deviceshare"), _i64("ds_scoring_strategy"),
    _i64("ds_scoring_weights", 3),
    _i64("batch_pods"), _i64("pods_per_wave"), _i64("device_id"),
    _i64("reservation_filter"), _i64("reservation_score"), _i64("weight_reservation"),
    _i64("pipeline_depth"),
    _i64("la_agg_usage_thresholds", RES_MAX), _i64("la_agg_usage_type"), _i64("la_agg_usage_duration_ns"),
    _i64("la_agg_score_type"), _i64("la_agg_score_duration_ns"),
    _i64("taint_filter"), _i64("taint_score"), _i64("weight_taint"),
    _i64("affinity_filter"), _i64("affinity_score"), _i64("weight_affinity"),
    _i64("balanced_score"), _i64("weight_balanced"), _i64("balanced_resources"),
    _i64("image_score"), _i64("weight_image"),
    _i64("spread_filter"), _i64("spread_score"), _i64("weight_spread"),
    _i64("interpod_filter"), _i64("interpod_score"), _i64("weight_interpod"), _i64("hard_pod_affinity_weight"),
    _i64("multi_rank_mode"), _i64("ds_scoring_weights_x", 2), _i64("reserved", 1),
])

NODE_DTYPE = np.dtype([
    _i64("allocatable", RES_MAX),
    _i64("allowed_pods"),
    _i64("flags"),
    _i64("raw_allocatable", RES_MAX),
    _i64("raw_allocatable_present", RES_MAX),
    _i64("custom_usage_thresholds", RES_MAX),
    _i64("custom_prod_usage_thresholds", RES_MAX),
    _i64("custom_agg_thresholds", RES_MAX), _i64("custom_agg_type"), _i64("custom_agg_duration_ns"),
])

METRIC_DTYPE = np.dtype([
    _i64("present"), _i64("has_node_metric"), _i64("has_update_time"), _i64("update_time_unix_nano"),
    _i64("node_usage", RES_MAX),
    _i64("node_usage_present", RES_MAX),
    _i64("pods_metric_count"),
    _i64("prod_pods_usage", RES_MAX),
    _i64("agg_count"), _i64("agg_duration_ns", 4), ("agg_usage", np.int64, (4, 5, 2)), ("agg_present", np.int64, (4, 5)),
    _i64("report_interval_ns"),
])
POD_METRIC_DTYPE = np.dtype([_i64("uid"), _i64("usage", 2), _i64("usage_present"), _i64("prod")])
AGG_TYPES = {"": 0, "avg": 1, "p50": 2, "p90": 3, "p95": 4, "p99": 5}

POD_DTYPE = np.dtype([
    _i64("requests", RES_MAX),
    _i64("limits", RES_MAX),
    _i64("nonzero_requests", 2),
    _i64("priority_class"),
    _i64("flags"),
    _i64("qos"), _i64("required_cpu_bind_policy"), _i64("preferred_cpu_bind_policy"),
    _i64("device_requests", DEV_RES_MAX),
    _i64("quota_id"),
    _i64("reservation_owner_mask"), _i64("reservation_flags"),
    _i64("uid"), _i64("assign_time_unix_nano"),
    ("tolerated_taints", np.uint64), ("node_selector", np.uint64),
    _i64("n_required_terms"), ("required_terms", np.uint64, (MAX_AFF_TERMS,)),
    _i64("n_preferred_terms"), ("preferred_terms", np.uint64, (MAX_AFF_TERMS,)), _i64("preferred_weights", MAX_AFF_TERMS),
    _i64("preferred_cpu_exclusive_policy"),
    _i64("n_containers"), _i64("container_image_bit", MAX_CONTAINERS), _i64("container_image_score", MAX_CONTAINERS),
    _i64("taint_count"),
    _i64("match_groups"), _i64("n_spread"), _i64("spread_group", MAX_SPREAD), _i64("spread_max_skew", MAX_SPREAD),
    _i64("spread_flags", MAX_SPREAD), _i64("pod_affinity_group"), _i64("pod_affinity_terms"), _i64("pod_anti_affinity"),
    _i64("n_pod_preferred"), _i64("pod_preferred_group", MAX_POD_PREFERRED),
    _i64("pod_preferred_weight", MAX_POD_PREFERRED),
    _i64("pod_affinity_terms_zone"), _i64("pod_anti_affinity_zone"), _i64("pod_preferred_zone"),
    ("reservation_selector", np.uint64), _i64("n_reservation_terms"), ("reservation_terms", np.uint64, (MAX_AFF_TERMS,)),
    _i64("reserve_allocate_policy"), _i64("reserve_node"),
])
NODE_PRED_DTYPE = np.dtype([("predicates", np.uint64), ("taints_hard", np.uint64), ("taints_soft", np.uint64),
                            ("images", np.uint64), _i64("predicate_count"), _i64("image_count"), _i64("zone")])


NODE_RSV_DTYPE = np.dtype([_i64("n")] + [_i64(f, MAX_RSV_SLOTS) for f in (
    "owner", "allocatable_cpu", "allocatable_mem", "allocated_cpu", "allocated_mem", "assigned", "order", "policy",
    "allocate_once", "available", "unschedulable")] + [("predicates", np.uint64, (MAX_RSV_SLOTS,)),
                                                        _i64("predicate_count"),
                                                        # (ABI 13) GPUs held per reservation
                                                        _i64("gpu_minors", MAX_RSV_SLOTS),
                                                        _i64("gpu_alloc", (MAX_RSV_SLOTS, MAX_MINORS, 3)),
                                                        _i64("gpu_allocated", (MAX_RSV_SLOTS, MAX_MINORS, 3)),
                                                        # (ABI 15) cpusets held per reservation / its assigned pods'
                                                        ("cpus", np.uint64, (MAX_RSV_SLOTS, MAX_CPUS // 64)),
                                                        ("cpus_assigned", np.uint64, (MAX_RSV_SLOTS, MAX_CPUS // 64))])

QUOTA_DTYPE = np.dtype([_i64("used", QUOTA_RES), _i64("non_preemptible_used", QUOTA_RES), _i64("used_limit", QUOTA_RES),
                        _i64("min", QUOTA_RES)])

NODE_DEVICE_DTYPE = np.dtype([
    _i64("has_device"), _i64("present", MAX_MINORS), _i64("healthy", MAX_MINORS),
    _i64("total_core", MAX_MINORS), _i64("total_memory", MAX_MINORS), _i64("total_ratio", MAX_MINORS),
    _i64("used_core", MAX_MINORS), _i64("used_memory", MAX_MINORS), _i64("used_ratio", MAX_MINORS),
    # (ABI 17) RDMA / FPGA DeviceInfos [XTYPE_RDMA, XTYPE_FPGA][minor]
    _i64("x_present", (DEV_XTYPES, MAX_MINORS)), _i64("x_healthy", (DEV_XTYPES, MAX_MINORS)),
    _i64("x_total", (DEV_XTYPES, MAX_MINORS)), _i64("x_used", (DEV_XTYPES, MAX_MINORS)),
])

NODE_NUMA_DTYPE = np.dtype([
    _i64("has_topology"), _i64("sockets"), _i64("nodes_per_socket"), _i64("cores_per_node"), _i64("cpus_per_core"),
    _i64("numa_policy"), _i64("node_cpu_bind_policy"), _i64("numa_allocate_strategy"), _i64("num_numa"),
    _i64("numa_cpu", MAX_NUMA), _i64("numa_mem", MAX_NUMA),
    ("reserved_cpus", np.uint64, (MAX_CPUS // 64,)), ("allocated_cpus", np.uint64, (MAX_CPUS // 64,)),
    _i64("numa_alloc_cpu", MAX_NUMA), _i64("numa_alloc_mem", MAX_NUMA), ("cpu_amplification_ratio", np.float64),
    ("exclusive_pcpu_cpus", np.uint64, (MAX_CPUS // 64,)), ("exclusive_numa_cpus", np.uint64, (MAX_CPUS // 64,)),
])

STATS_DTYPE = np.dtype([
    _i64("pods_scheduled"), _i64("pods_unschedulable"), _i64("device_batches"), _i64("node_evaluations"),
    ("seconds", np.float64), ("reserved", np.float64, (3,)),
])

STRUCT_DTYPES = {0: CONFIG_DTYPE, 1: NODE_DTYPE, 2: METRIC_DTYPE, 3: POD_DTYPE, 4: STATS_DTYPE, 5: NODE_NUMA_DTYPE,
                 6: NODE_DEVICE_DTYPE, 7: QUOTA_DTYPE, 8: NODE_RSV_DTYPE, 9: POD_METRIC_DTYPE, 10: NODE_PRED_DTYPE}

# Every symbol include/koordgpu.h declares (tests check the library exports all of them).
EXPORTED_SYMBOLS = (
    "kg_config_default", "kg_engine_create", "kg_engine_destroy", "kg_nodes_upsert", "kg_nodes_delete",
    "kg_node_metrics_update", "kg_pods_add", "kg_pods_remove", "kg_pods_schedule", "kg_pods_evaluate",
    "kg_pods_stage", "kg_pods_schedule_staged", "kg_results_fetch", "kg_engine_num_nodes",
    "kg_nodes_read_state", "kg_bench_kernel", "kg_debug_least_requested", "kg_last_error", "kg_abi_version",
    "kg_abi_struct_size", "kg_nccl_unique_id", "kg_debug_rccl_selftest", "kg_debug_eval_paths", "kg_debug_stamps",
    "kg_debug_fast_lrs",
    "kg_nodes_numa_upsert", "kg_nodes_read_numa", "kg_results_fetch_cpusets", "kg_pods_evaluate_numa",
    "kg_nodes_device_upsert", "kg_nodes_read_device", "kg_results_fetch_devices", "kg_pods_evaluate_device",
    "kg_results_fetch_devices_x", "kg_nodes_read_device_x",
    "kg_quotas_set", "kg_quotas_read", "kg_nodes_reservation_upsert", "kg_nodes_read_reservations",
    "kg_nodes_read_reservation_gpus", "kg_nodes_read_reservation_cpus", "kg_engine_ranks",
    "kg_results_fetch_reservations", "kg_profile_enable", "kg_profile_read", "kg_loopback_create",
    "kg_loopback_destroy", "kg_engine_create_loopback", "kg_pods_unreserve", "kg_engine_set_clock",
    "kg_node_pods_metric_set", "kg_debug_numa_merge", "kg_pods_evaluate_reservation", "kg_nodes_predicates_upsert",
    "kg_engine_create_hosted", "kg_pods_filter_preemption", "kg_nodes_read_pod_groups",
    "kg_pods_select_victims",
)

# int (*kg_exchange_fn)(void* user, const void* send, void* recv, int64_t bytes)
EXCHANGE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64)

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("KOORDGPU_LIB") or os.path.join(PKG_DIR, "libkoordgpu.so")

_lib = None


class _ArrayPtr(ctypes.c_void_p):
    """A c_void_p that keeps its array alive: `ptr(np.ascontiguousarray(x))` passes a temporary, which would otherwise
    be freed as soon as ptr() returns, leaving the call a dangling pointer."""


def ptr(a):
    """Pointer to a numpy array's data (None for None); the array lives as long as the pointer object."""
    if a is None:
        return None
    q = _ArrayPtr(a.ctypes.data)
    q._array = a
    return q


def load_library(path: str | None = None):
    """Loads the in-tree engine library.  Fails loudly if it is missing: there is no CPU fallback."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise RuntimeError(f"koordgpu engine library not built: {p} (run `make -C koordinator_amd` "
                           f"or __graft_entry__.build())")
    lib = ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)
    vp, i64, i32, i = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int
    sig = {
        "kg_config_default": (None, [vp]),
        "kg_engine_create": (i, [vp, i64, i, i, vp, ctypes.POINTER(vp)]),
        "kg_engine_destroy": (None, [vp]),
        "kg_nodes_upsert": (i, [vp, vp, vp, i64]),
        "kg_nodes_delete": (i, [vp, vp, i64]),
        "kg_node_metrics_update": (i, [vp, vp, vp, i64, i64]),
        "kg_node_pods_metric_set": (i, [vp, i, vp, i64]),
        "kg_pods_add": (i, [vp, vp, vp, i64]),
        "kg_pods_remove": (i, [vp, vp, vp, i64]),
        "kg_pods_schedule": (i, [vp, vp, i64, vp, vp, vp]),
        "kg_pods_evaluate": (i, [vp, vp, vp, vp, vp]),
        "kg_pods_stage": (i, [vp, vp, i64]),
        "kg_pods_schedule_staged": (i, [vp, i64, i64, vp]),
        "kg_results_fetch": (i, [vp, i64, i64, vp, vp]),
        "kg_engine_num_nodes": (i64, [vp]),
        "kg_nodes_read_state": (i, [vp] + [vp] * 9),
        "kg_bench_kernel": (i, [vp, i, i, vp, vp]),
        "kg_debug_least_requested": (i, [vp, vp, vp, vp, i64]),
        "kg_last_error": (ctypes.c_char_p, []),
        "kg_abi_version": (i, []),
        "kg_abi_struct_size": (i64, [i]),
        "kg_nccl_unique_id": (i, [vp]),
        "kg_debug_rccl_selftest": (i, [i, i64]),
        "kg_debug_eval_paths": (i, [vp, vp]),
        "kg_debug_stamps": (i, [vp, vp]),
        "kg_debug_fast_lrs": (i, [vp, vp, vp, vp, vp, i64]),
        "kg_nodes_numa_upsert": (i, [vp, vp, vp, i64]),
        "kg_nodes_read_numa": (i, [vp, vp, vp, vp]),
        "kg_results_fetch_cpusets": (i, [vp, i64, i64, vp]),
        "kg_pods_evaluate_numa": (i, [vp, vp, vp, vp, vp]),
        "kg_nodes_device_upsert": (i, [vp, vp, vp, i64]),
        "kg_nodes_read_device": (i, [vp, vp, vp, vp]),
        "kg_results_fetch_devices": (i, [vp, i64, i64, vp]),
        "kg_results_fetch_devices_x": (i, [vp, i64, i64, vp]),
        "kg_nodes_read_device_x": (i, [vp, vp]),
        "kg_pods_evaluate_device": (i, [vp, vp, vp, vp]),
        "kg_quotas_set": (i, [vp, vp, i64]),
        "kg_quotas_read": (i, [vp, vp, i64]),
        "kg_nodes_reservation_upsert": (i, [vp, vp, vp, i64]),
        "kg_nodes_read_reservations": (i, [vp, vp, vp, vp]),
        "kg_nodes_read_reservation_gpus": (i, [vp, vp]),
        "kg_nodes_read_reservation_cpus": (i, [vp, vp]),
        "kg_engine_ranks": (i, [vp, vp, vp]),
        "kg_results_fetch_reservations": (i, [vp, i64, i64, vp]),
        "kg_profile_enable": (i, [vp, i]),
        "kg_profile_read": (i, [vp, vp, vp]),
        "kg_loopback_create": (i, [i, ctypes.POINTER(vp)]),
        "kg_loopback_destroy": (None, [vp]),
        "kg_engine_create_loopback": (i, [vp, i64, i, i, vp, ctypes.POINTER(vp)]),
        "kg_pods_unreserve": (i, [vp, i64, i64, vp]),
        "kg_engine_set_clock": (i, [vp, i64]),
        "kg_debug_numa_merge": (i, [vp, vp, i64, vp]),
        "kg_pods_evaluate_reservation": (i, [vp, vp, vp]),
        "kg_pods_filter_preemption": (i, [vp, vp, ctypes.c_int32, vp, vp, vp, i64, vp]),
        "kg_pods_select_victims": (i, [vp, vp, i64, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
        "kg_nodes_read_pod_groups": (i, [vp, vp, vp, vp, vp, vp]),
        "kg_nodes_predicates_upsert": (i, [vp, vp, vp, i64]),
        "kg_engine_create_hosted": (i, [vp, i64, i, i, EXCHANGE_FN, vp, ctypes.POINTER(vp)]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    if lib.kg_abi_version() != ABI_VERSION:
        raise RuntimeError("koordgpu ABI version mismatch")
    for which, dt in STRUCT_DTYPES.items():
        if lib.kg_abi_struct_size(which) != dt.itemsize:
            raise RuntimeError(f"ABI struct {which} size mismatch: C {lib.kg_abi_struct_size(which)} vs {dt.itemsize}")
    if path is None:
        _lib = lib
    return lib


class KoordGPUError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"koordgpu error {code}: {msg}")
        self.code = code


def check(lib, rc: int):
    if rc != 0:
        raise KoordGPUError(rc, lib.kg_last_error().decode(errors="replace"))
    return rc
