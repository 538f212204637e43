"""ctypes binding of the CPU restatement (oracle/oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the
checker or the timed CPU baseline — never by koordinator_amd/.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

from koordinator_amd import abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "liboracle.so")

OR_STATE_DTYPE = np.dtype([
    ("requested", np.int64, (abi.RES_MAX,)),
    ("nonzero", np.int64, (2,)),
    ("num_pods", np.int64),
    ("la_est_all", np.int64, (2,)),
    ("la_est_prod", np.int64, (2,)),
    ("la_term", np.int64, (4,)),
    ("has_la_term", np.int64),
])
OR_ASSIGNED_DTYPE = np.dtype([("uid", np.int64), ("time", np.int64), ("est", np.int64, (2,)), ("prod", np.int64)])

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        vp, i64, i = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
        L.or_estimate_pod.argtypes = [vp, vp, vp]
        # (r6) NodeNUMAResource with reservation cpusets
        L.or_numa_available_pref_flat.argtypes = [vp, vp, vp]
        L.or_numa_available_pref_flat.restype = None
        L.or_take_preferred_flat.argtypes = [i, i, i, i, vp, vp, i, i, i, vp]
        L.or_take_preferred_flat.restype = i
        L.or_numa_reserve_rsv_flat.argtypes = [vp, vp, vp, vp, vp]
        L.or_numa_reserve_rsv_flat.restype = i
        L.or_numa_rsv_reserved_flat.argtypes = [vp, i, vp]
        L.or_numa_rsv_reserved_flat.restype = None
        L.or_numa_state_export.argtypes = [vp, i64, vp]
        L.or_numa_state_export.restype = None
        L.or_numa_state_set.argtypes = [vp, i64, vp]
        L.or_numa_state_set.restype = None
        L.or_la_node_terms.argtypes = [vp, vp, vp, ctypes.c_int64, vp, ctypes.c_int64, vp]
        L.or_la_node_terms.restype = None
        L.or_estimate_node.argtypes = [vp, i]
        L.or_estimate_node.restype = i64
        L.or_loadaware_filter.argtypes = [vp, vp, vp, vp, i64]
        L.or_loadaware_filter.restype = i
        L.or_loadaware_score.argtypes = [vp, vp, vp, vp, vp, i64]
        L.or_loadaware_score.restype = i64
        L.or_fit_filter.argtypes = [vp, vp, vp]
        L.or_fit_filter.restype = i
        L.or_fit_score.argtypes = [vp, vp, vp, vp]
        L.or_fit_score.restype = i64
        L.or_least_requested_score.argtypes = [i64, i64]
        L.or_least_requested_score.restype = i64
        L.or_apply_pod.argtypes = [vp, vp, vp, i]
        L.or_states_init.argtypes = [i64, vp]
        L.or_states_add_pods.argtypes = [vp, i64, vp, i64, vp, vp]
        L.or_states_add_pods.restype = i
        L.or_schedule.argtypes = [vp, i64, vp, vp, vp, i64, vp, i64, i, vp, vp]
        L.or_schedule.restype = i
        L.or_node_keys.argtypes = [vp, vp, vp, vp, vp, i64, i64, i64, vp]
        L.or_node_keys.restype = i
        L.or_schedule_numa.argtypes = [vp, i64, vp, vp, vp, vp, i64, vp, i64, i, vp, vp, vp]
        L.or_schedule_numa.restype = i
        L.or_numa_state_size.restype = i64
        L.or_numa_states_init.argtypes = [vp, i64, vp]
        L.or_numa_state_read.argtypes = [vp, i64, vp, vp, vp]
        L.or_take_cpus_flat.argtypes = [i, i, i, i, vp, i, i, i, vp]
        L.or_take_cpus_flat.restype = i
        L.or_take_cpus_excl_flat.argtypes = [i, i, i, i, vp, i, i, i, i, vp, vp]
        L.or_take_cpus_excl_flat.restype = i
        L.or_numa_eval_flat.argtypes = [vp, vp, vp, i64, i64, i64, i64, vp, vp]
        L.or_numa_eval_flat.restype = i
        L.or_numa_reserve_flat.argtypes = [vp, vp, vp, vp]
        L.or_numa_reserve_flat.restype = i
        L.or_schedule_full.argtypes = [vp, i64, vp, vp, vp, vp, vp, vp, i64, i64, vp, i64, i, vp, vp, vp, vp, vp]
        L.or_unreserve.argtypes = [vp, vp, vp, vp, vp, vp, i64, vp, i, vp, vp, i, i]
        L.or_unreserve.restype = i
        L.or_schedule_full.restype = i
        L.or_ds_pod_init.argtypes = [vp, vp]
        L.or_ds_pod_init.restype = i
        L.or_ds_filter.argtypes = [vp, vp]
        L.or_ds_filter.restype = i
        L.or_ds_score.argtypes = [vp, vp, i, vp]
        L.or_ds_score.restype = i64
        L.or_ds_reserve.argtypes = [vp, vp, i, vp]
        L.or_ds_reserve.restype = ctypes.c_int32
        L.or_dsx_filter.argtypes = [vp, vp, vp]
        L.or_dsx_filter.restype = i
        L.or_dsx_score.argtypes = [vp, vp, i, vp]
        L.or_dsx_score.restype = i64
        L.or_dsx_reserve.argtypes = [vp, vp, i, vp]
        L.or_dsx_reserve.restype = ctypes.c_int32
        L.or_ds_release.argtypes = [vp, vp, ctypes.c_int32]
        L.or_ds_release.restype = None
        L.or_ds_memory_bytes_to_ratio.argtypes = [i64, i64]
        L.or_ds_memory_bytes_to_ratio.restype = i64
        L.or_ds_memory_ratio_to_bytes.argtypes = [i64, i64]
        L.or_ds_memory_ratio_to_bytes.restype = i64
        L.or_ds_instance_flat.argtypes = [vp, vp, vp]
        L.or_ds_instance_flat.restype = i
        L.or_ds_rsv_init.argtypes = [vp, vp, i, vp, i, vp]
        L.or_ds_rsv_init.restype = None
        L.or_ds_try_rsv.argtypes = [vp, vp, vp, vp, vp, i, i, i, vp, vp]
        L.or_ds_try_rsv.restype = i
        L.or_ds_filter_rsv.argtypes = [vp, vp, vp, vp, i]
        L.or_ds_filter_rsv.restype = i
        L.or_ds_filter_reservation.argtypes = [vp, vp, vp, vp, i]
        L.or_ds_filter_reservation.restype = i
        L.or_ds_score_slot.argtypes = [vp, vp, vp, vp, i, i, vp]
        L.or_ds_score_slot.restype = i64
        L.or_ds_score_rsv.argtypes = [vp, vp, vp, vp, i, i, vp]
        L.or_ds_score_rsv.restype = i64
        L.or_ds_reserve_rsv.argtypes = [vp, vp, vp, vp, i, i, vp]
        L.or_ds_reserve_rsv.restype = ctypes.c_int32
        L.or_schedule_resv.argtypes = [vp, i64, vp, vp, vp, vp, i64, vp, i64, vp, vp, vp]
        L.or_schedule_resv.restype = i
        L.or_schedule_resv_full.argtypes = [vp, i64, vp, vp, vp, vp, vp, vp, i64, i64, vp, i64, i, vp, vp, vp, vp,
                                            vp, vp, vp, vp, vp]
        L.or_groups_apply.argtypes = [vp, vp, i, i64]
        L.or_groups_apply.restype = None
        L.or_spread_node_ok.argtypes = [vp, vp, i]
        L.or_spread_node_ok.restype = i
        L.or_spread_has_keys.argtypes = [vp, vp, i]
        L.or_spread_has_keys.restype = i
        L.or_spread_raw.argtypes = [vp, vp, vp]
        L.or_spread_raw.restype = i64
        L.or_spread_normalize.argtypes = [i64, i64, i64]
        L.or_spread_normalize.restype = i64
        L.or_ipa_zones_add.argtypes = [vp, vp, ctypes.c_int32, vp]
        L.or_ipa_zones_add.restype = None
        L.or_interpod_filter.argtypes = [vp, vp, ctypes.c_int32, vp]
        L.or_interpod_filter.restype = i
        L.or_interpod_raw.argtypes = [vp, vp, ctypes.c_int32, vp]
        L.or_interpod_raw.restype = i64
        L.or_interpod_normalize.argtypes = [i64, i64, i64]
        L.or_interpod_normalize.restype = i64
        L.or_schedule_resv_full.restype = i
        L.or_quota_admit.argtypes = [vp, vp]
        L.or_quota_admit.restype = i
        L.or_rsv_case_flat.argtypes = [vp, i64, vp, i64, vp, vp, i, vp, vp]
        L.or_rsv_case_flat.restype = None
        L.or_rsv_policy_filter.argtypes = [vp, i64, vp]
        L.or_rsv_policy_filter.restype = i
        L.or_filter_preemption.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, i64, i64, vp]
        L.or_filter_preemption.restype = i64
        L.or_select_victims.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, i64, vp, vp, vp]
        L.or_select_victims.restype = i64
        for f, res in (("or_taint_filter", i), ("or_taint_count", i64), ("or_affinity_filter", i),
                       ("or_affinity_sum", i64), ("or_image_score", i64)):
            getattr(L, f).argtypes = [vp, vp]
            getattr(L, f).restype = res
        L.or_balanced_score.argtypes = [i64] * 7
        L.or_balanced_score.restype = i64
        L.or_normalize_default.argtypes = [i64, i64, i]
        L.or_normalize_default.restype = i64
        _lib = L
    return _lib


DS_POD_DTYPE = np.dtype([("skip", np.int32), ("reserve", np.int32), ("error", np.int32), ("unsupported", np.int32),
                         ("has_mem", np.int32), ("core", np.int64), ("mem", np.int64), ("ratio", np.int64),
                         ("nogpu", np.int32), ("xq", np.int64, (abi.DEV_XTYPES,))], align=True)
# (ABI 13) or_ds_rsv: the DeviceShare restore of one node (oracle/deviceshare.h)
DS_RSV_DTYPE = np.dtype([("n_matched", np.int32), ("matched", np.int32, (abi.MAX_RSV_SLOTS,)),
                         ("unm_used", np.int64, (abi.MAX_MINORS, 3)), ("mat_allocd", np.int64, (abi.MAX_MINORS, 3)),
                         ("mat_alloc", np.int64, (abi.MAX_MINORS, 3))], align=True)


def ds_pod(pod) -> np.ndarray:
    """DeviceShare preFilterState of one kg_pod (or_ds_pod_init)."""
    out = np.zeros(1, dtype=DS_POD_DTYPE)
    lib().or_ds_pod_init(p(np.ascontiguousarray(np.asarray(pod, dtype=abi.POD_DTYPE).reshape(1))), p(out))
    return out


def ds_instance(dev, pod):
    """CalcDesiredRequestsAndCount on one node: None (Insufficient gpu devices) or (count, core, mem, ratio)."""
    out = np.zeros(4, dtype=np.int64)
    ok = lib().or_ds_instance_flat(p(np.ascontiguousarray(dev)), p(ds_pod(pod)), p(out))
    return tuple(int(x) for x in out) if ok else None


def ds_filter(dev, pod) -> bool:
    return bool(lib().or_ds_filter(p(np.ascontiguousarray(dev)), p(ds_pod(pod))))


def _wx(cfg):
    return np.ascontiguousarray(cfg["ds_scoring_weights_x"].reshape(abi.DEV_XTYPES), dtype=np.int64)


def ds_score(cfg, dev, pod) -> int:
    """The plugin's raw Score: the GPU type's + (ABI 17) the RDMA / FPGA types' (AutopilotAllocator.score sums them)."""
    w = np.ascontiguousarray(cfg["ds_scoring_weights"].reshape(3), dtype=np.int64)
    d, dp = p(np.ascontiguousarray(dev)), p(ds_pod(pod))
    return int(lib().or_ds_score(d, dp, int(cfg["ds_scoring_strategy"]), p(w))) + \
        int(lib().or_dsx_score(d, dp, int(cfg["ds_scoring_strategy"]), p(_wx(cfg))))


def ds_reserve(cfg, dev, pod) -> int:
    """Reserve on one node (mutates `dev`, a 1-element NODE_DEVICE array): the packed minor bitmask (GPU bits 0-7,
    (ABI 17) RDMA 8-15, FPGA 16-23), 0 none, -1 failure (nothing allocated)."""
    w = np.ascontiguousarray(cfg["ds_scoring_weights"].reshape(3), dtype=np.int64)
    dp = ds_pod(pod)
    m = int(lib().or_ds_reserve(p(dev), p(dp), int(cfg["ds_scoring_strategy"]), p(w)))
    if m < 0:
        return m
    x = int(lib().or_dsx_reserve(p(dev), p(dp), int(cfg["ds_scoring_strategy"]), p(_wx(cfg))))
    if x < 0:
        lib().or_ds_release(p(dev), p(dp), m)
        return -1
    return m | x


def dsx_filter(dev, pod, pre=None) -> bool:
    """(ABI 17) the RDMA / FPGA part of the Filter; pre = int64[2, 8] preemptible amounts per type and minor."""
    pr = None if pre is None else np.ascontiguousarray(pre, dtype=np.int64).reshape(abi.DEV_XTYPES, abi.MAX_MINORS)
    return bool(lib().or_dsx_filter(p(np.ascontiguousarray(dev)), p(ds_pod(pod)), p(pr) if pr is not None else None))


def _w(cfg):
    return np.ascontiguousarray(cfg["ds_scoring_weights"].reshape(3), dtype=np.int64)


def ds_rsv_init(rsv, matched=(), unmatched=()) -> np.ndarray:
    """(ABI 13) the DeviceShare restore of one node over its GPU-holding slots (or_ds_rsv_init): `matched` /
    `unmatched` are the Reservation restore's slot lists, in order."""
    out = np.zeros(1, dtype=DS_RSV_DTYPE)
    m = np.ascontiguousarray(matched, dtype=np.int32)
    u = np.ascontiguousarray(unmatched, dtype=np.int32)
    r = np.ascontiguousarray(np.asarray(rsv, dtype=abi.NODE_RSV_DTYPE).reshape(1))
    lib().or_ds_rsv_init(p(r), p(m), len(m), p(u), len(u), p(out))
    return out


def ds_try_rsv(cfg, dev, pod, rsv, st, slots, scored=True):
    """tryAllocateFromReservation over `slots` (or_ds_try_rsv): (satisfied slot or -1, minor mask)."""
    mask = np.zeros(1, dtype=np.int32)
    sl = np.ascontiguousarray(slots, dtype=np.int32)
    r = np.ascontiguousarray(np.asarray(rsv, dtype=abi.NODE_RSV_DTYPE).reshape(1))
    s = lib().or_ds_try_rsv(p(np.ascontiguousarray(dev)), p(ds_pod(pod)), p(r), p(st), p(sl), len(sl), int(scored),
                            int(cfg["ds_scoring_strategy"]), p(_w(cfg)), p(mask))
    return int(s), int(mask[0])


def ds_filter_rsv(dev, pod, rsv, st, required_from_rsv=False) -> bool:
    r = np.ascontiguousarray(np.asarray(rsv, dtype=abi.NODE_RSV_DTYPE).reshape(1))
    return bool(lib().or_ds_filter_rsv(p(np.ascontiguousarray(dev)), p(ds_pod(pod)), p(r), p(st),
                                       int(required_from_rsv)))


def ds_score_slot(cfg, dev, pod, rsv, st, s) -> int:
    """ScoreReservation of slot s (or_ds_score_slot, scoreWithReservation)."""
    r = np.ascontiguousarray(np.asarray(rsv, dtype=abi.NODE_RSV_DTYPE).reshape(1))
    return int(lib().or_ds_score_slot(p(np.ascontiguousarray(dev)), p(ds_pod(pod)), p(r), p(st), int(s),
                                      int(cfg["ds_scoring_strategy"]), p(_w(cfg))))


def ds_reserve_rsv(cfg, dev, pod, rsv, st, nominated) -> int:
    """Reserve with the node's GPU reservations (mutates `dev`): minor bitmask, 0 none, -1 failure."""
    r = np.ascontiguousarray(np.asarray(rsv, dtype=abi.NODE_RSV_DTYPE).reshape(1))
    return int(lib().or_ds_reserve_rsv(p(dev), p(ds_pod(pod)), p(r), p(st), int(nominated),
                                       int(cfg["ds_scoring_strategy"]), p(_w(cfg))))


NUMA_ALLOC_WORDS = 1 + 2 * abi.MAX_NUMA  # per-pod NUMA allocation record (oracle/numa.h OR_NUMA_ALLOC_WORDS)


def schedule_full(cfg, nodes, metrics, st, pods, now_ns: int, n_threads: int = 1, numa_buf=None, devices=None,
                  quotas=None, with_numa_alloc: bool = False):
    """Sequential FIFO scheduling with the optional NodeNUMAResource / DeviceShare states and ElasticQuota table
    (all mutated).  Returns (node, score, cpusets uint64[n, 4], GPU minor masks int32[n]) and, with_numa_alloc,
    each pod's NUMA allocation record int64[n, NUMA_ALLOC_WORDS]."""
    pods = np.ascontiguousarray(pods, dtype=abi.POD_DTYPE)
    out_node = np.empty(len(pods), dtype=np.int32)
    out_score = np.empty(len(pods), dtype=np.int64)
    cpus = np.zeros((max(len(pods), 1), abi.MAX_CPUS // 64), dtype=np.uint64)
    minors = np.zeros(max(len(pods), 1), dtype=np.int32)
    nalloc = np.zeros((max(len(pods), 1), NUMA_ALLOC_WORDS), dtype=np.int64)
    nq = 0 if quotas is None else len(quotas)
    rc = lib().or_schedule_full(p(cfg), len(nodes), p(nodes), p(metrics), p(st), p(numa_buf), p(devices), p(quotas), nq,
                                len(pods), p(pods), now_ns, n_threads, p(out_node), p(out_score), p(cpus), p(minors),
                                p(nalloc))
    if rc != 0:
        raise RuntimeError(f"oracle or_schedule_full failed: {rc}")
    out = (out_node, out_score, cpus[:len(pods)], minors[:len(pods)])
    return out + (nalloc[:len(pods)],) if with_numa_alloc else out


def unreserve(cfg, st, pod, node: int, numa_buf=None, devices=None, rsv=None, quotas=None, cpus=None,
              numa_alloc=None, minors: int = 0, slot: int = -1):
    """The framework's Unreserve of one placed pod (or_unreserve; every state given is mutated)."""
    pod = np.ascontiguousarray(np.asarray(pod, dtype=abi.POD_DTYPE).reshape(1))
    cp = None if cpus is None else np.ascontiguousarray(cpus, dtype=np.uint64)
    na = None if numa_alloc is None else np.ascontiguousarray(numa_alloc, dtype=np.int64)
    nq = 0 if quotas is None else len(quotas)
    rc = lib().or_unreserve(p(cfg), p(st), p(numa_buf), p(devices), p(rsv), p(quotas), nq, p(pod), int(node), p(cp),
                            p(na), int(minors), int(slot))
    if rc != 0:
        raise RuntimeError(f"oracle or_unreserve failed: {rc}")


p = abi.ptr


# (ABI 12) or_group_node: per node and match group, pods matching / required anti-affinity terms / symmetric weights
GROUP_DTYPE = np.dtype([(f, np.int32, (abi.MAX_MATCH_GROUPS,)) for f in ("cnt", "anti", "symw", "anti_z", "symw_z")])
# or_ipa_zones: one incoming pod's zone-keyed InterPodAffinity maps (defaults.h)
IPA_ZONES_DTYPE = np.dtype([(f, np.int64, (abi.MAX_ZONES,)) for f in ("aff", "anti_in", "anti_ex", "score")]
                           + [("entries", np.int64)])


def groups_init(n_nodes: int, pods=None, node_idx=None, hard_weight: int = 1) -> np.ndarray:
    """or_group_node[n_nodes] with `pods` on nodes `node_idx` added (or_groups_apply, NodeInfo.AddPod)."""
    g = np.zeros(max(n_nodes, 1), dtype=GROUP_DTYPE)
    if pods is not None:
        pods = np.ascontiguousarray(pods, dtype=abi.POD_DTYPE)
        for k in range(len(pods)):
            groups_apply(g, int(node_idx[k]), pods[k:k + 1], 1, hard_weight)
    return g


def groups_apply(g, node: int, pod, sign: int, hard_weight: int = 1):
    row = g[node:node + 1]
    lib().or_groups_apply(p(row), p(np.ascontiguousarray(pod, dtype=abi.POD_DTYPE)), sign, hard_weight)


def schedule_resv(cfg, nodes, metrics, st, rsv, pods, now_ns: int, devices=None, quotas=None, n_threads: int = 1,
                  with_minors: bool = False, numa_buf=None, with_numa: bool = False, preds=None, groups=None):
    """Sequential FIFO scheduling through the per-pod exact loop: NodeResourcesFit + LoadAware + Reservation
    [+ DeviceShare + NodeNUMAResource + ElasticQuota + TaintToleration / NodeAffinity over `preds` (NODE_PRED_DTYPE
    rows) + BalancedAllocation] (st, rsv, devices, numa_buf, quotas mutated; the node loop of each
    pod on n_threads threads).  Returns (node, score, slot) — slot = the reservation each pod was assumed into (-1 =
    none) — then, with_minors, DeviceShare's minor masks and, with_numa, the cpusets uint64[n, 4] and NUMA allocation
    records int64[n, NUMA_ALLOC_WORDS] NodeNUMAResource Reserve made."""
    pods = np.ascontiguousarray(pods, dtype=abi.POD_DTYPE)
    n = max(len(pods), 1)
    out_node, out_score, out_slot, out_minors = (np.empty(n, dtype=np.int32), np.empty(n, dtype=np.int64),
                                                 np.empty(n, dtype=np.int32), np.zeros(n, dtype=np.int32))
    cpus = np.zeros((n, abi.MAX_CPUS // 64), dtype=np.uint64)
    nalloc = np.zeros((n, NUMA_ALLOC_WORDS), dtype=np.int64)
    nq = 0 if quotas is None else len(quotas)
    rc = lib().or_schedule_resv_full(p(cfg), len(nodes), p(nodes), p(metrics), p(st), p(rsv), p(devices), p(quotas),
                                     nq, len(pods), p(pods), now_ns, n_threads, p(out_node), p(out_score), p(out_slot),
                                     p(out_minors), p(numa_buf), p(cpus), p(nalloc),
                                     p(None if preds is None else np.ascontiguousarray(preds, dtype=abi.NODE_PRED_DTYPE)),
                                     p(groups))
    if rc != 0:
        raise RuntimeError(f"oracle or_schedule_resv_full failed: {rc}")
    out = (out_node[:len(pods)], out_score[:len(pods)], out_slot[:len(pods)])
    if with_minors:
        out = out + (out_minors[:len(pods)],)
    if with_numa:
        out = out + (cpus[:len(pods)], nalloc[:len(pods)])
    return out


def quota_admit(quota, pod) -> bool:
    """ElasticQuota PreFilter admission of one pod against one quota (or_quota_admit)."""
    return bool(lib().or_quota_admit(p(np.ascontiguousarray(np.asarray(quota, dtype=abi.QUOTA_DTYPE).reshape(1))),
                                     p(np.ascontiguousarray(np.asarray(pod, dtype=abi.POD_DTYPE).reshape(1)))))


def rsv_case(pod, allowed_pods, alloc, num_pods, pod_requested, r_allocated, has_state, rsv):
    """One node's Reservation Filter / nomination / Score with an explicit nodeReservationState, every slot in
    `matched` (how reservation/*_test.go build their states).  Returns (filter_pass, nominated_slot, score)."""
    out = np.zeros(3, dtype=np.int64)
    a = lambda v: np.ascontiguousarray(v, dtype=np.int64)
    lib().or_rsv_case_flat(p(np.ascontiguousarray(np.asarray(pod, dtype=abi.POD_DTYPE).reshape(1))), allowed_pods,
                           p(a(alloc)), num_pods, p(a(pod_requested)), p(a(r_allocated)), int(has_state),
                           p(np.ascontiguousarray(np.asarray(rsv, dtype=abi.NODE_RSV_DTYPE).reshape(1))), p(out))
    return int(out[0]), int(out[1]), int(out[2])


def _pre_ext(numa, dev, pred, minors, n):
    """or_pre_ext {numa, dev, pred, victim_minors} (r6): None members = not in the profile / none.  Returns the struct
    (a ctypes array of 4 pointers) and the arrays it points into (kept alive by the caller)."""
    c = lambda a, dt: np.ascontiguousarray(np.asarray(a, dtype=dt).reshape(-1))
    keep = [c(numa, abi.NODE_NUMA_DTYPE) if numa is not None else None,
            c(dev, abi.NODE_DEVICE_DTYPE) if dev is not None else None,
            c(pred, abi.NODE_PRED_DTYPE) if pred is not None else None,
            c(minors, np.int32) if minors is not None and n else None]
    if all(k is None for k in keep):
        return None, keep
    x = (ctypes.c_void_p * 4)(*[k.ctypes.data if k is not None else None for k in keep])
    return x, keep


def filter_preemption(cfg, node, metric, state, rsv, pod, victims, slots, now_ns: int, numa=None, dev=None, pred=None,
                      minors=None) -> int:
    """or_filter_preemption: the preemption dry run's Filter (KG_REJECT_* bits) of one pod on one node; (r6) numa /
    dev / pred = the node's NodeNUMAResource / DeviceShare / predicate rows, minors[k] = victim k's GPU minors."""
    c = lambda a, dt: np.ascontiguousarray(np.asarray(a, dtype=dt).reshape(-1))
    v = c(victims, abi.POD_DTYPE)
    sl = c(slots if slots is not None else -np.ones(len(v)), np.int32)
    x, _keep = _pre_ext(numa, dev, pred, minors, len(v))
    return int(lib().or_filter_preemption(p(cfg), p(c(node, abi.NODE_DTYPE)), p(c(metric, abi.METRIC_DTYPE)),
                                          p(np.ascontiguousarray(state[:1])),
                                          p(c(rsv, abi.NODE_RSV_DTYPE)) if rsv is not None else None,
                                          p(c(pod, abi.POD_DTYPE)), p(v) if len(v) else None, p(sl) if len(v) else None,
                                          len(v), now_ns, ctypes.cast(x, ctypes.c_void_p) if x is not None else None))


def select_victims(cfg, node, metric, state, rsv, pod, victims, slots, violating, now_ns: int, numa=None, dev=None,
                   pred=None, minors=None):
    """or_select_victims: SelectVictimsOnNode of one candidate → (reject bits, bool[k] victim kept, numViolating)."""
    c = lambda a, dt: np.ascontiguousarray(np.asarray(a, dtype=dt).reshape(-1))
    v = c(victims, abi.POD_DTYPE)
    n = len(v)
    sl = c(slots if slots is not None else -np.ones(n), np.int32)
    vio = c(violating if violating is not None else np.zeros(n), np.uint8)
    kept = np.zeros(max(n, 1), dtype=np.uint8)
    nv = np.zeros(1, dtype=np.int32)
    x, _keep = _pre_ext(numa, dev, pred, minors, n)
    rej = int(lib().or_select_victims(p(cfg), p(c(node, abi.NODE_DTYPE)), p(c(metric, abi.METRIC_DTYPE)),
                                      p(np.ascontiguousarray(state[:1])),
                                      p(c(rsv, abi.NODE_RSV_DTYPE)) if rsv is not None else None,
                                      p(c(pod, abi.POD_DTYPE)), p(v) if n else None, p(sl) if n else None,
                                      p(vio) if n else None, n, now_ns, p(kept), p(nv),
                                      ctypes.cast(x, ctypes.c_void_p) if x is not None else None))
    return rej, kept[:n].astype(bool), int(nv[0])


def rsv_restore(rsv, st, pod) -> dict:
    """BeforePreFilter's restore of one node (or_rsv_restore_flat)."""
    out = np.zeros(11, dtype=np.int64)
    lib().or_rsv_restore_flat(p(np.ascontiguousarray(np.asarray(rsv, dtype=abi.NODE_RSV_DTYPE).reshape(1))),
                              p(np.ascontiguousarray(st[:1])),
                              p(np.ascontiguousarray(np.asarray(pod, dtype=abi.POD_DTYPE).reshape(1))), p(out))
    names = ("has_state", "matched", "requested_cpu", "requested_mem", "nonzero_cpu", "nonzero_mem", "num_pods",
             "pod_requested_cpu", "pod_requested_mem", "r_allocated_cpu", "r_allocated_mem")
    return {k: int(v) for k, v in zip(names, out)}


def states(n: int) -> np.ndarray:
    st = np.zeros(n, dtype=OR_STATE_DTYPE)
    lib().or_states_init(n, p(st))
    return st


def add_pods(cfg, st, pods, node_idx):
    pods = np.ascontiguousarray(pods, dtype=abi.POD_DTYPE)
    node_idx = np.ascontiguousarray(node_idx, dtype=np.int32)
    rc = lib().or_states_add_pods(p(cfg), len(st), p(st), len(pods), p(pods), p(node_idx))
    assert rc == 0, rc


def estimate_pod(cfg, pod) -> tuple:
    out = np.zeros(2, dtype=np.int64)
    lib().or_estimate_pod(p(cfg), p(np.ascontiguousarray(pod)), p(out))
    return int(out[0]), int(out[1])


def estimate_node(node, r: int) -> int:
    return int(lib().or_estimate_node(p(np.ascontiguousarray(node)), r))


def loadaware_filter(cfg, node, metric, pod, now_ns: int) -> int:
    return int(lib().or_loadaware_filter(p(cfg), p(node), p(metric), p(pod), now_ns))


def loadaware_score(cfg, node, metric, state, pod, now_ns: int) -> int:
    return int(lib().or_loadaware_score(p(cfg), p(node), p(metric), p(state), p(pod), now_ns))


def la_node_terms(cfg, metric, pods_metric, assigned) -> np.ndarray:
    """or_la_node_terms: the PodsMetric LoadAware Score terms of one node ([0..1] all pods, [2..3] prod view)."""
    pm = np.ascontiguousarray(pods_metric, dtype=abi.POD_METRIC_DTYPE)
    a = np.ascontiguousarray(assigned, dtype=OR_ASSIGNED_DTYPE)
    out = np.zeros(4, dtype=np.int64)
    lib().or_la_node_terms(p(cfg), p(np.ascontiguousarray(np.asarray(metric, dtype=abi.METRIC_DTYPE).reshape(1))),
                           p(pm) if len(pm) else None, len(pm), p(a) if len(a) else None, len(a), p(out))
    return out


def set_la_terms(st, i: int, terms):
    st["la_term"][i] = terms
    st["has_la_term"][i] = 1


def fit_filter(node, state, pod) -> int:
    return int(lib().or_fit_filter(p(node), p(state), p(pod)))


def fit_score(cfg, node, state, pod) -> int:
    return int(lib().or_fit_score(p(cfg), p(node), p(state), p(pod)))


def least_requested(requested: int, capacity: int) -> int:
    return int(lib().or_least_requested_score(requested, capacity))


def schedule(cfg, nodes, metrics, st, pods, now_ns: int, n_threads: int = 1):
    """Sequential FIFO scheduling; mutates `st` (assume). Returns (node_idx, score)."""
    pods = np.ascontiguousarray(pods, dtype=abi.POD_DTYPE)
    out_node = np.empty(len(pods), dtype=np.int32)
    out_score = np.empty(len(pods), dtype=np.int64)
    rc = lib().or_schedule(p(cfg), len(nodes), p(nodes), p(metrics), p(st), len(pods), p(pods), now_ns,
                           n_threads, p(out_node), p(out_score))
    if rc != 0:
        raise RuntimeError(f"oracle or_schedule failed: {rc}")
    return out_node, out_score


def node_keys(cfg, nodes, metrics, st, pod, now_ns: int, lo: int, hi: int) -> np.ndarray:
    """Packed keys (total << 32 | ~idx, 0 = filtered out) of one pod on nodes [lo, hi), current `st`."""
    out = np.zeros(max(hi - lo, 0), dtype=np.uint64)
    pod = np.ascontiguousarray(np.asarray(pod, dtype=abi.POD_DTYPE).reshape(1))
    rc = lib().or_node_keys(p(cfg), p(nodes), p(metrics), p(st), p(pod), now_ns, lo, hi, p(out))
    if rc != 0:
        raise RuntimeError(f"oracle or_node_keys failed: {rc}")
    return out


def apply_pod(cfg, st, pod, node: int, sign: int = 1):
    """assume (+1) / forget (-1) of one pod on node `node` of `st` (or_apply_pod)."""
    pod = np.ascontiguousarray(np.asarray(pod, dtype=abi.POD_DTYPE).reshape(1))
    lib().or_apply_pod(p(cfg), p(st[node:node + 1]), p(pod), sign)


def numa_states(nodes_numa: np.ndarray) -> np.ndarray:
    """Per-node NodeNUMAResource state (numa.c or_numa_node) from kg_node_numa rows."""
    nodes_numa = np.ascontiguousarray(nodes_numa, dtype=abi.NODE_NUMA_DTYPE)
    size = int(lib().or_numa_state_size())
    buf = np.zeros(max(len(nodes_numa), 1) * size, dtype=np.uint8)
    lib().or_numa_states_init(p(nodes_numa), len(nodes_numa), p(buf))
    return buf


def numa_state_export(buf: np.ndarray, i: int, row: np.ndarray) -> np.ndarray:
    """(r6) kg_node_numa row `row` (static fields) with node i's current NodeAllocation from the oracle state."""
    out = np.ascontiguousarray(np.array(row, dtype=abi.NODE_NUMA_DTYPE).reshape(1))
    lib().or_numa_state_export(p(buf), int(i), p(out))
    return out


def numa_state_set(buf: np.ndarray, i: int, row: np.ndarray):
    """(r6) node i's oracle state re-initialised from a kg_node_numa row (an upsert)."""
    lib().or_numa_state_set(p(buf), int(i), p(np.ascontiguousarray(np.array(row, dtype=abi.NODE_NUMA_DTYPE).reshape(1))))


def numa_state_read(buf: np.ndarray, n: int):
    """(allocated cpu masks uint64[n,4], per-NUMA allocated cpu int64[n,4], memory int64[n,4])."""
    alloc = np.zeros((n, abi.MAX_CPUS // 64), dtype=np.uint64)
    cpu = np.zeros((n, abi.MAX_NUMA), dtype=np.int64)
    mem = np.zeros((n, abi.MAX_NUMA), dtype=np.int64)
    for i in range(n):
        lib().or_numa_state_read(p(buf), i, p(alloc[i]), p(cpu[i]), p(mem[i]))
    return alloc, cpu, mem


def schedule_numa(cfg, nodes, metrics, st, numa_buf, pods, now_ns: int, n_threads: int = 1, with_cpusets=False):
    """or_schedule with the NodeNUMAResource plugin; mutates `st` and `numa_buf`.  Returns (node, score) or,
    with_cpusets, (node, score, uint64[n_pods, 4] cpuset Reserve allocated to each pod)."""
    pods = np.ascontiguousarray(pods, dtype=abi.POD_DTYPE)
    out_node = np.empty(len(pods), dtype=np.int32)
    out_score = np.empty(len(pods), dtype=np.int64)
    cpus = np.zeros((max(len(pods), 1), abi.MAX_CPUS // 64), dtype=np.uint64)
    rc = lib().or_schedule_numa(p(cfg), len(nodes), p(nodes), p(metrics), p(st), p(numa_buf), len(pods), p(pods),
                                now_ns, n_threads, p(out_node), p(out_score), p(cpus))
    if rc != 0:
        raise RuntimeError(f"oracle or_schedule_numa failed: {rc}")
    if with_cpusets:
        return out_node, out_score, cpus[:len(pods)]
    return out_node, out_score


def _cpu_words(cpus):
    words = np.zeros(abi.MAX_CPUS // 64, dtype=np.uint64)
    for c in cpus:
        words[c // 64] |= np.uint64(1) << np.uint64(c % 64)
    return words


def take_cpus(topology, available, needed: int, bind_policy: str, strategy: str, exclusive_policy: str = "",
              exclusive_cpus=()):
    """takeCPUs on buildCPUTopologyForTest(*topology); returns the cpu list or None on error.  exclusive_policy =
    the pod's CPUExclusivePolicy, exclusive_cpus = the allocated cpus holding that policy."""
    words = _cpu_words(available)
    out = np.zeros(abi.MAX_CPUS // 64, dtype=np.uint64)
    if exclusive_policy:
        rc = lib().or_take_cpus_excl_flat(*topology, p(words), needed, abi.BIND[bind_policy], abi.STRATEGY[strategy],
                                          abi.EXCL[exclusive_policy], p(_cpu_words(exclusive_cpus)), p(out))
    else:
        rc = lib().or_take_cpus_flat(*topology, p(words), needed, abi.BIND[bind_policy], abi.STRATEGY[strategy],
                                     p(out))
    if rc != 0:
        return None
    return [64 * w + b for w in range(len(out)) for b in range(64) if (int(out[w]) >> b) & 1]


def _cpu_list(words):
    return [64 * w + b for w in range(len(words)) for b in range(64) if (int(words[w]) >> b) & 1]


def numa_available_pref(node_numa, preferred):
    """(r6) getAvailableCPUs with preferred cpus (node_allocation.go:133-153) on a node whose allocated cpus have
    RefCount 1: the available cpu list."""
    out = np.zeros(abi.MAX_CPUS // 64, dtype=np.uint64)
    lib().or_numa_available_pref_flat(p(np.ascontiguousarray(node_numa)), p(_cpu_words(preferred)), p(out))
    return _cpu_list(out)


def take_preferred(topology, available, preferred, needed: int, bind_policy: str, strategy: str):
    """(r6) takePreferredCPUs (cpu_accumulator.go:33-85): the cpu list or None on error."""
    out = np.zeros(abi.MAX_CPUS // 64, dtype=np.uint64)
    rc = lib().or_take_preferred_flat(*topology, p(_cpu_words(available)), p(_cpu_words(preferred)), needed,
                                      abi.BIND[bind_policy], abi.STRATEGY[strategy], p(out))
    return None if rc != 0 else _cpu_list(out)


def numa_rsv_reserved(rsv, slot: int):
    """(r6) RestoreReservation's reservedCPUs of one slot (nodenumaresource/reservation.go:76-113)."""
    out = np.zeros(abi.MAX_CPUS // 64, dtype=np.uint64)
    lib().or_numa_rsv_reserved_flat(p(np.ascontiguousarray(np.asarray(rsv, dtype=abi.NODE_RSV_DTYPE).reshape(1))),
                                    int(slot), p(out))
    return _cpu_list(out)


def numa_reserve_rsv(cfg, node_numa, rsv, pod):
    """(r6) Reserve of a pod nominated into reservation slot 0, which holds cpus: (0 / -1, chosen cpu list)."""
    out = np.zeros(abi.MAX_CPUS // 64, dtype=np.uint64)
    rc = lib().or_numa_reserve_rsv_flat(p(cfg), p(np.ascontiguousarray(node_numa)),
                                        p(np.ascontiguousarray(np.asarray(rsv, dtype=abi.NODE_RSV_DTYPE).reshape(1))),
                                        p(np.ascontiguousarray(pod)), p(out))
    return rc, _cpu_list(out)


def numa_eval(cfg, node_numa, pod, node_requested=(0, 0), node_allocatable=(0, 0)):
    """(passes Filter, Score, stored affinity mask or -1 for nil) of one pod on one node."""
    score = np.zeros(1, dtype=np.int64)
    mask = np.zeros(1, dtype=np.int64)
    ok = lib().or_numa_eval_flat(p(cfg), p(np.ascontiguousarray(node_numa)), p(np.ascontiguousarray(pod)),
                                 int(node_requested[0]), int(node_requested[1]), int(node_allocatable[0]),
                                 int(node_allocatable[1]), p(score), p(mask))
    return bool(ok), int(score[0]), int(mask[0])


def numa_reserve(cfg, node_numa, pod):
    """Reserve of one pod on one node: (0 / -1, chosen cpu list)."""
    out = np.zeros(abi.MAX_CPUS // 64, dtype=np.uint64)
    rc = lib().or_numa_reserve_flat(p(cfg), p(np.ascontiguousarray(node_numa)), p(np.ascontiguousarray(pod)), p(out))
    return rc, [64 * w + b for w in range(len(out)) for b in range(64) if (int(out[w]) >> b) & 1]


def schedule_cluster(cfg, cluster, pods, n_threads: int = 1):
    st = states(cluster.n)
    if len(cluster.existing_pods):
        add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
    node, score = schedule(cfg, cluster.nodes, cluster.metrics, st, pods, cluster.now_ns, n_threads)
    return node, score, st


MERGE_POLICY = {"best-effort": 1, "restricted": 2, "single-numa-node": 3}


def _hint_arrays(lists):
    """Flat (counts int32[nl], hints int64[nl, 16, 4]) of hint lists [[mask bits or None, preferred, score?], ...]."""
    counts = np.zeros(max(len(lists), 1), dtype=np.int32)
    hints = np.zeros((max(len(lists), 1), 16, 4), dtype=np.int64)
    for i, l in enumerate(lists):
        counts[i] = len(l)
        for j, h in enumerate(l):
            bits = h[0]
            hints[i, j] = (1 if bits is None else 0, 0 if bits is None else sum(1 << b for b in bits), int(bool(h[1])),
                           h[2] if len(h) > 2 else 0)
    return counts, hints


def policy_merge(policy: str, num_numa: int, lists):
    """Policy.Merge + canAdmitPodResult on filtered provider lists (or_debug_policy_merge):
    (admit, mask bits or None, preferred, score)."""
    counts, hints = _hint_arrays(lists)
    out = np.zeros(5, dtype=np.int64)
    rc = lib().or_debug_policy_merge(MERGE_POLICY[policy], num_numa, len(lists), p(counts), p(hints), p(out))
    if rc != 0:
        raise RuntimeError("or_debug_policy_merge failed")
    bits = None if out[1] else [b for b in range(8) if (int(out[2]) >> b) & 1]
    return bool(out[0]), bits, bool(out[3]), int(out[4])


def single_numa_filter(lists):
    """filterSingleNumaHints (or_debug_single_numa_filter): the filtered lists."""
    counts, hints = _hint_arrays(lists)
    oc = np.zeros_like(counts)
    oh = np.zeros_like(hints)
    rc = lib().or_debug_single_numa_filter(len(lists), p(counts), p(hints), p(oc), p(oh))
    if rc != 0:
        raise RuntimeError("or_debug_single_numa_filter failed")
    return [[[None if oh[i, j, 0] else [b for b in range(8) if (int(oh[i, j, 1]) >> b) & 1], bool(oh[i, j, 2])]
             for j in range(oc[i])] for i in range(len(lists))]


def _pred_pod(pred, pod):
    n = np.ascontiguousarray(np.asarray(pred, dtype=abi.NODE_PRED_DTYPE).reshape(1))
    q = np.ascontiguousarray(np.asarray(pod, dtype=abi.POD_DTYPE).reshape(1))
    return n, q


def default_plugins(pred, pod) -> dict:
    """TaintToleration / NodeAffinity of one (node, pod) (oracle/defaults.c): filter verdicts and raw Scores."""
    n, q = _pred_pod(pred, pod)
    L = lib()
    return {"taint_filter": bool(L.or_taint_filter(p(n), p(q))), "taint_count": int(L.or_taint_count(p(n), p(q))),
            "affinity_filter": bool(L.or_affinity_filter(p(n), p(q))),
            "affinity_sum": int(L.or_affinity_sum(p(n), p(q))), "image_score": int(L.or_image_score(p(n), p(q)))}


def balanced_score(alloc_cpu, alloc_mem, req_cpu, req_mem, pod_cpu, pod_mem, resources=3) -> int:
    return int(lib().or_balanced_score(alloc_cpu, alloc_mem, req_cpu, req_mem, pod_cpu, pod_mem, resources))


def normalize_default(score, max_count, reverse) -> int:
    return int(lib().or_normalize_default(score, max_count, int(bool(reverse))))
