"""Python handle over the koordgpu C ABI (the same entry points a cgo binding would call)."""
from __future__ import annotations

import ctypes

import numpy as np

from . import abi
from .abi import check, ptr


def default_config() -> np.ndarray:
    """kg_config_default: v1beta2 LoadAwareSchedulingArgs defaults + NodeResourcesFit LeastAllocated cpu/mem."""
    lib = abi.load_library()
    cfg = np.zeros(1, dtype=abi.CONFIG_DTYPE)
    lib.kg_config_default(ptr(cfg))
    return cfg


def nccl_unique_id() -> bytes:
    """ncclGetUniqueId on this rank (rank 0 creates it; the caller broadcasts the 128 bytes)."""
    lib = abi.load_library()
    buf = ctypes.create_string_buffer(128)
    check(lib, lib.kg_nccl_unique_id(ctypes.cast(buf, ctypes.c_void_p)))
    return buf.raw


class Loopback:
    """kg_loopback (test hook): n ranks' engines in one process exchanging their round records by device copies
    instead of RCCL.  Drive each rank's engine from its own thread (ctypes releases the GIL in the calls)."""

    def __init__(self, n_ranks: int):
        self.lib = abi.load_library()
        h = ctypes.c_void_p()
        check(self.lib, self.lib.kg_loopback_create(int(n_ranks), ctypes.byref(h)))
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self.lib.kg_loopback_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class HostExchange:
    """kg_engine_create_hosted's exchange over a caller-side all-gather: `allgather(send: bytes-like uint8 array)`
    returns the n_ranks parts concatenated in rank order — e.g. torch.distributed.all_gather on gloo CPU tensors,
    so that several processes run the engine's multi-rank round path without RCCL."""

    def __init__(self, allgather):
        self.allgather = allgather
        self.error = None

        def _fn(user, send, recv, nbytes):
            try:
                buf = np.ctypeslib.as_array(ctypes.cast(send, ctypes.POINTER(ctypes.c_uint8)), shape=(int(nbytes),))
                out = np.ascontiguousarray(self.allgather(buf.copy()), dtype=np.uint8).reshape(-1)
                ctypes.memmove(recv, out.ctypes.data, out.nbytes)
                return 0
            except Exception as exc:  # reported through the engine's KG_E_COLLECTIVE
                self.error = exc
                return 1

        self.fn = abi.EXCHANGE_FN(_fn)  # kept alive as long as the engine


class Engine:
    """One engine = one rank's GPU-resident node table (replicated) + its evaluation shard."""

    def __init__(self, config: np.ndarray, capacity: int, rank: int = 0, n_ranks: int = 1,
                 nccl_id: bytes | None = None, loopback: Loopback | None = None,
                 exchange: HostExchange | None = None):
        self.lib = abi.load_library()
        self._cfg = np.array(config, dtype=abi.CONFIG_DTYPE).reshape(1)
        h = ctypes.c_void_p()
        idbuf = None
        if nccl_id is not None:
            idbuf = ctypes.create_string_buffer(bytes(nccl_id), 128)
        self._exchange = exchange
        if exchange is not None:
            check(self.lib, self.lib.kg_engine_create_hosted(ptr(self._cfg), int(capacity), int(rank), int(n_ranks),
                                                             exchange.fn, None, ctypes.byref(h)))
        elif loopback is not None:
            check(self.lib, self.lib.kg_engine_create_loopback(ptr(self._cfg), int(capacity), int(rank), int(n_ranks),
                                                               loopback.h, ctypes.byref(h)))
        else:
            check(self.lib, self.lib.kg_engine_create(ptr(self._cfg), int(capacity), int(rank), int(n_ranks),
                                                      ctypes.cast(idbuf, ctypes.c_void_p) if idbuf else None,
                                                      ctypes.byref(h)))
        self.h = h
        self.capacity = capacity

    # -- lifecycle -------------------------------------------------------------------------------------
    def close(self):
        if getattr(self, "h", None):
            self.lib.kg_engine_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- informer-style deltas ------------------------------------------------------------------------
    @staticmethod
    def _idx(idx, n):
        if idx is None:
            idx = np.arange(n, dtype=np.int32)
        return np.ascontiguousarray(idx, dtype=np.int32)

    def upsert_nodes(self, nodes: np.ndarray, idx=None):
        nodes = np.ascontiguousarray(nodes, dtype=abi.NODE_DTYPE)
        idx = self._idx(idx, len(nodes))
        check(self.lib, self.lib.kg_nodes_upsert(self.h, ptr(nodes), ptr(idx), len(nodes)))

    def delete_nodes(self, idx):
        idx = np.ascontiguousarray(idx, dtype=np.int32)
        check(self.lib, self.lib.kg_nodes_delete(self.h, ptr(idx), len(idx)))

    def update_metrics(self, metrics: np.ndarray, now_ns: int, idx=None):
        metrics = np.ascontiguousarray(metrics, dtype=abi.METRIC_DTYPE)
        idx = self._idx(idx, len(metrics))
        check(self.lib, self.lib.kg_node_metrics_update(self.h, ptr(metrics), ptr(idx), len(metrics), int(now_ns)))

    def set_pods_metric(self, node: int, entries: np.ndarray):
        """kg_node_pods_metric_set: NodeMetric.Status.PodsMetric of one node (POD_METRIC_DTYPE rows)."""
        entries = np.ascontiguousarray(entries, dtype=abi.POD_METRIC_DTYPE)
        check(self.lib, self.lib.kg_node_pods_metric_set(self.h, int(node), ptr(entries) if len(entries) else None,
                                                          len(entries)))

    def add_pods(self, pods: np.ndarray, node_idx):
        pods = np.ascontiguousarray(pods, dtype=abi.POD_DTYPE)
        node_idx = np.ascontiguousarray(node_idx, dtype=np.int32)
        check(self.lib, self.lib.kg_pods_add(self.h, ptr(pods), ptr(node_idx), len(pods)))

    def remove_pods(self, pods: np.ndarray, node_idx):
        pods = np.ascontiguousarray(pods, dtype=abi.POD_DTYPE)
        node_idx = np.ascontiguousarray(node_idx, dtype=np.int32)
        check(self.lib, self.lib.kg_pods_remove(self.h, ptr(pods), ptr(node_idx), len(pods)))

    def unreserve(self, first: int, count: int, mask=None):
        """kg_pods_unreserve: the framework's Unreserve of staged pods [first, first+count) (mask selects them)."""
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        if m is not None and len(m) != count:
            raise ValueError("mask length != count")
        check(self.lib, self.lib.kg_pods_unreserve(self.h, int(first), int(count), ptr(m)))

    def set_clock(self, now_ns: int):
        """kg_engine_set_clock: > 0 fixed, 0 real time, < 0 the newest metrics update time."""
        check(self.lib, self.lib.kg_engine_set_clock(self.h, int(now_ns)))

    def upsert_numa(self, node_numa: np.ndarray, idx=None):
        """NodeNUMAResource state (TopologyOptions + NodeAllocation) of nodes `idx` (kg_nodes_numa_upsert)."""
        node_numa = np.ascontiguousarray(node_numa, dtype=abi.NODE_NUMA_DTYPE)
        idx = self._idx(idx, len(node_numa))
        check(self.lib, self.lib.kg_nodes_numa_upsert(self.h, ptr(node_numa), ptr(idx), len(node_numa)))

    def upsert_devices(self, node_device: np.ndarray, idx=None):
        """DeviceShare GPU state (Device object + deviceUsed) of nodes `idx` (kg_nodes_device_upsert)."""
        node_device = np.ascontiguousarray(node_device, dtype=abi.NODE_DEVICE_DTYPE)
        idx = self._idx(idx, len(node_device))
        check(self.lib, self.lib.kg_nodes_device_upsert(self.h, ptr(node_device), ptr(idx), len(node_device)))

    def upsert_reservations(self, node_rsv: np.ndarray, idx=None):
        """Reservation slots of nodes `idx` (kg_nodes_reservation_upsert)."""
        node_rsv = np.ascontiguousarray(node_rsv, dtype=abi.NODE_RSV_DTYPE)
        idx = self._idx(idx, len(node_rsv))
        check(self.lib, self.lib.kg_nodes_reservation_upsert(self.h, ptr(node_rsv), ptr(idx), len(node_rsv)))

    def upsert_predicates(self, preds: np.ndarray, idx=None):
        """TaintToleration / NodeAffinity node rows of nodes `idx` (kg_nodes_predicates_upsert; NODE_PRED_DTYPE, see
        koordinator_amd/predicates.py)."""
        preds = np.ascontiguousarray(preds, dtype=abi.NODE_PRED_DTYPE)
        idx = self._idx(idx, len(preds))
        check(self.lib, self.lib.kg_nodes_predicates_upsert(self.h, ptr(preds), ptr(idx), len(preds)))

    def read_reservations(self):
        """(allocated cpu, allocated memory, assigned), int64[n, KG_MAX_RSV_SLOTS] each, from the device."""
        n = self.num_nodes
        out = [np.zeros((n, abi.MAX_RSV_SLOTS), dtype=np.int64) for _ in range(3)]
        check(self.lib, self.lib.kg_nodes_read_reservations(self.h, *[ptr(o) for o in out]))
        return tuple(out)

    def read_reservation_gpus(self):
        """(ABI 13) the reservation slots' gpu_allocated, int64[n, KG_MAX_RSV_SLOTS, KG_MAX_MINORS, 3], from the device
        (kg_nodes_read_reservation_gpus)."""
        out = np.zeros((self.num_nodes, abi.MAX_RSV_SLOTS, abi.MAX_MINORS, 3), dtype=np.int64)
        check(self.lib, self.lib.kg_nodes_read_reservation_gpus(self.h, ptr(out)))
        return out

    def read_reservation_cpus(self):
        """(ABI 15) the reservation slots' cpus_assigned, uint64[n, KG_MAX_RSV_SLOTS, 4], from the device
        (kg_nodes_read_reservation_cpus)."""
        out = np.zeros((self.num_nodes, abi.MAX_RSV_SLOTS, abi.MAX_CPUS // 64), dtype=np.uint64)
        check(self.lib, self.lib.kg_nodes_read_reservation_cpus(self.h, ptr(out)))
        return out

    def read_pod_groups(self, zone: bool = False):
        """(ABI 12) per node and match group: (pods matching, required anti-affinity terms, symmetric weight) — and,
        with zone, the zone-keyed terms' (anti-affinity, symmetric weight) — int32[n, KG_MAX_MATCH_GROUPS] each, from
        the device (kg_nodes_read_pod_groups)."""
        n = self.num_nodes
        out = [np.zeros((n, abi.MAX_MATCH_GROUPS), dtype=np.int32) for _ in range(5)]
        check(self.lib, self.lib.kg_nodes_read_pod_groups(self.h, *[ptr(o) for o in out]))
        return tuple(out[:3]) if not zone else tuple(out)

    def fetch_reservations(self, first: int, count: int) -> np.ndarray:
        """int32[count]: the reservation slot Reserve assumed each staged pod into (-1 = none)."""
        out = np.zeros(count, dtype=np.int32)
        check(self.lib, self.lib.kg_results_fetch_reservations(self.h, int(first), int(count), ptr(out)))
        return out

    def set_quotas(self, quotas: np.ndarray):
        """ElasticQuota table (kg_quotas_set): pods' quota_id = 1 + index."""
        quotas = np.ascontiguousarray(quotas, dtype=abi.QUOTA_DTYPE)
        check(self.lib, self.lib.kg_quotas_set(self.h, ptr(quotas), len(quotas)))

    def read_quotas(self, n: int) -> np.ndarray:
        out = np.zeros(n, dtype=abi.QUOTA_DTYPE)
        check(self.lib, self.lib.kg_quotas_read(self.h, ptr(out), n))
        return out

    # -- hot path -----------------------------------------------------------------------------------------
    def schedule(self, pods: np.ndarray):
        """Sequential FIFO scheduling with assume; returns (node_idx[-1 = unschedulable], total_score, stats)."""
        pods = np.ascontiguousarray(pods, dtype=abi.POD_DTYPE)
        n = len(pods)
        out_node = np.empty(n, dtype=np.int32)
        out_score = np.empty(n, dtype=np.int64)
        stats = np.zeros(1, dtype=abi.STATS_DTYPE)
        check(self.lib, self.lib.kg_pods_schedule(self.h, ptr(pods), n, ptr(out_node), ptr(out_score), ptr(stats)))
        return out_node, out_score, stats[0]

    def stage(self, pods: np.ndarray):
        pods = np.ascontiguousarray(pods, dtype=abi.POD_DTYPE)
        check(self.lib, self.lib.kg_pods_stage(self.h, ptr(pods), len(pods)))

    def schedule_staged(self, first: int, count: int):
        stats = np.zeros(1, dtype=abi.STATS_DTYPE)
        check(self.lib, self.lib.kg_pods_schedule_staged(self.h, int(first), int(count), ptr(stats)))
        return stats[0]

    def fetch(self, first: int, count: int):
        out_node = np.empty(count, dtype=np.int32)
        out_score = np.empty(count, dtype=np.int64)
        check(self.lib, self.lib.kg_results_fetch(self.h, int(first), int(count), ptr(out_node), ptr(out_score)))
        return out_node, out_score

    def evaluate(self, pod: np.ndarray):
        """Per-node reject bits, NodeResourcesFit score, LoadAwareScheduling score for one pod (no assume)."""
        pod = np.ascontiguousarray(np.asarray(pod, dtype=abi.POD_DTYPE).reshape(1))
        n = self.num_nodes
        rej = np.zeros(n, dtype=np.int32)
        fit = np.zeros(n, dtype=np.int64)
        la = np.zeros(n, dtype=np.int64)
        check(self.lib, self.lib.kg_pods_evaluate(self.h, ptr(pod), ptr(rej), ptr(fit), ptr(la)))
        return rej, fit, la

    def evaluate_numa(self, pod: np.ndarray):
        """NodeNUMAResource alone on every node: (passes Filter, Score, stored affinity mask or -1 for nil)."""
        pod = np.ascontiguousarray(np.asarray(pod, dtype=abi.POD_DTYPE).reshape(1))
        n = self.num_nodes
        ok = np.zeros(n, dtype=np.int32)
        sc = np.zeros(n, dtype=np.int64)
        af = np.zeros(n, dtype=np.int64)
        check(self.lib, self.lib.kg_pods_evaluate_numa(self.h, ptr(pod), ptr(ok), ptr(sc), ptr(af)))
        return ok, sc, af

    def evaluate_device(self, pod: np.ndarray):
        """DeviceShare alone on every node: (passes Filter, raw Score before NormalizeScore)."""
        pod = np.ascontiguousarray(np.asarray(pod, dtype=abi.POD_DTYPE).reshape(1))
        n = self.num_nodes
        ok = np.zeros(n, dtype=np.int32)
        sc = np.zeros(n, dtype=np.int64)
        check(self.lib, self.lib.kg_pods_evaluate_device(self.h, ptr(pod), ptr(ok), ptr(sc)))
        return ok, sc

    def fetch_devices(self, first: int, count: int) -> np.ndarray:
        """int32[count]: the GPU minor bitmask DeviceShare Reserve allocated to each staged pod (0 = none)."""
        out = np.zeros(count, dtype=np.int32)
        check(self.lib, self.lib.kg_results_fetch_devices(self.h, int(first), int(count), ptr(out)))
        return out

    def fetch_devices_x(self, first: int, count: int) -> np.ndarray:
        """int32[count, 2]: the RDMA / FPGA minor bitmasks DeviceShare Reserve allocated to each staged pod (ABI 17)."""
        out = np.zeros((count, abi.DEV_XTYPES), dtype=np.int32)
        check(self.lib, self.lib.kg_results_fetch_devices_x(self.h, int(first), int(count), ptr(out)))
        return out

    def read_devices_x(self) -> np.ndarray:
        """int64[n, 2, 8]: the RDMA / FPGA deviceUsed from the device (ABI 17)."""
        out = np.zeros((self.num_nodes, abi.DEV_XTYPES, abi.MAX_MINORS), dtype=np.int64)
        check(self.lib, self.lib.kg_nodes_read_device_x(self.h, ptr(out)))
        return out

    def read_devices(self):
        """(used core, used memory, used ratio), int64[n, 8] each, from the device."""
        n = self.num_nodes
        out = [np.zeros((n, abi.MAX_MINORS), dtype=np.int64) for _ in range(3)]
        check(self.lib, self.lib.kg_nodes_read_device(self.h, *[ptr(o) for o in out]))
        return tuple(out)

    def fetch_cpusets(self, first: int, count: int) -> np.ndarray:
        """uint64[count, 4]: the cpuset NodeNUMAResource Reserve allocated to each staged pod (empty = none)."""
        out = np.zeros((count, abi.MAX_CPUS // 64), dtype=np.uint64)
        check(self.lib, self.lib.kg_results_fetch_cpusets(self.h, int(first), int(count), ptr(out)))
        return out

    # -- introspection -----------------------------------------------------------------------------------
    @property
    def ranks(self) -> tuple:
        """(ABI 15) (ranks node evaluation is sharded over, ranks this engine replicates) — kg_engine_ranks."""
        s, r = ctypes.c_int64(), ctypes.c_int64()
        check(self.lib, self.lib.kg_engine_ranks(self.h, ctypes.byref(s), ctypes.byref(r)))
        return int(s.value), int(r.value)

    @property
    def num_nodes(self) -> int:
        return int(self.lib.kg_engine_num_nodes(self.h))

    def read_state(self) -> dict:
        n = self.num_nodes
        names = ("requested_cpu", "requested_mem", "nonzero_cpu", "nonzero_mem", "num_pods",
                 "la_est_cpu", "la_est_mem", "la_est_prod_cpu", "la_est_prod_mem")
        out = {k: np.zeros(n, dtype=np.int64) for k in names}
        check(self.lib, self.lib.kg_nodes_read_state(self.h, *[ptr(out[k]) for k in names]))
        return out

    def read_numa(self):
        """(allocated cpus uint64[n,4], per-NUMA allocated cpu int64[n,4], memory int64[n,4]) from the device."""
        n = self.num_nodes
        alloc = np.zeros((n, abi.MAX_CPUS // 64), dtype=np.uint64)
        cpu = np.zeros((n, abi.MAX_NUMA), dtype=np.int64)
        mem = np.zeros((n, abi.MAX_NUMA), dtype=np.int64)
        check(self.lib, self.lib.kg_nodes_read_numa(self.h, ptr(alloc), ptr(cpu), ptr(mem)))
        return alloc, cpu, mem

    def bench_kernel(self, which: int, iters: int):
        ms = ctypes.c_double()
        by = ctypes.c_double()
        check(self.lib, self.lib.kg_bench_kernel(self.h, int(which), int(iters), ctypes.byref(ms), ctypes.byref(by)))
        return ms.value, by.value

    def profile(self, on: bool = True):
        """Live kernel timing of the round runners (kg_profile_enable): resets the accumulators."""
        check(self.lib, self.lib.kg_profile_enable(self.h, int(on)))

    def profile_read(self) -> dict:
        """{kernel name: (summed event ms, launches)} since profile() (kg_profile_read)."""
        ms = np.zeros(abi.PROF_KINDS, dtype=np.float64)
        n = np.zeros(abi.PROF_KINDS, dtype=np.int64)
        check(self.lib, self.lib.kg_profile_read(self.h, ptr(ms), ptr(n)))
        return {name: (float(ms[k]), int(n[k])) for k, name in abi.PROF_NAMES.items() if n[k] > 0}

    def debug_eval_paths(self) -> int:
        out = np.zeros(1, dtype=np.int64)
        check(self.lib, self.lib.kg_debug_eval_paths(self.h, ptr(out)))
        return int(out[0])

    def filter_preemption(self, pod: np.ndarray, node: int, victims: np.ndarray, slots=None, minors=None) -> int:
        """The preemption dry run's Filter of `pod` on node `node` with `victims` removed (kg_pods_filter_preemption):
        KG_REJECT_* bits, 0 = fits.  slots[k]: the node's reservation slot victim k was allocated from (-1 = none);
        minors[k]: the GPU minors (bitmask) its DeviceShare allocation holds on the node (0 = none)."""
        pod = np.ascontiguousarray(np.asarray(pod, dtype=abi.POD_DTYPE).reshape(1))
        victims = np.ascontiguousarray(np.asarray(victims, dtype=abi.POD_DTYPE).reshape(-1))
        sl = None if slots is None else np.ascontiguousarray(slots, dtype=np.int32)
        mi = None if minors is None else np.ascontiguousarray(minors, dtype=np.int32)
        out = np.zeros(1, dtype=np.int32)
        check(self.lib, self.lib.kg_pods_filter_preemption(self.h, ptr(pod), int(node), ptr(victims) if len(victims) else None,
                                                           ptr(sl) if sl is not None else None,
                                                           ptr(mi) if mi is not None else None, len(victims), ptr(out)))
        return int(out[0])

    def select_victims(self, pod: np.ndarray, nodes, victims_per_node, slots_per_node=None, violating_per_node=None,
                       minors_per_node=None):
        """SelectVictimsOnNode on every candidate node in one launch (kg_pods_select_victims).  victims_per_node[c]:
        candidate c's potential victims (POD_DTYPE) in reprieve order; slots / violating / minors: per-victim reservation
        slot (-1 none), PDB-violating flag and GPU minors.  Returns (reject int32[C], victim bool arrays per candidate,
        violating int32[C])."""
        pod = np.ascontiguousarray(np.asarray(pod, dtype=abi.POD_DTYPE).reshape(1))
        nodes = np.ascontiguousarray(nodes, dtype=np.int32)
        counts = np.array([len(v) for v in victims_per_node], dtype=np.int64)
        off = np.zeros(len(nodes) + 1, dtype=np.int64)
        off[1:] = np.cumsum(counts)
        nv = int(off[-1])
        vic = np.zeros(max(nv, 1), dtype=abi.POD_DTYPE)
        if nv:
            vic[:nv] = np.concatenate([np.asarray(v, dtype=abi.POD_DTYPE).reshape(-1) for v in victims_per_node])
        sl = vio = mi = None
        if minors_per_node is not None and nv:
            mi = np.ascontiguousarray(np.concatenate([np.asarray(s, dtype=np.int32).reshape(-1)
                                                      for s in minors_per_node]))
        if slots_per_node is not None and nv:
            sl = np.ascontiguousarray(np.concatenate([np.asarray(s, dtype=np.int32).reshape(-1)
                                                      for s in slots_per_node]))
        if violating_per_node is not None and nv:
            vio = np.ascontiguousarray(np.concatenate([np.asarray(s, dtype=np.uint8).reshape(-1)
                                                       for s in violating_per_node]))
        rej = np.zeros(max(len(nodes), 1), dtype=np.int32)
        kept = np.zeros(max(nv, 1), dtype=np.uint8)
        nvio = np.zeros(max(len(nodes), 1), dtype=np.int32)
        check(self.lib, self.lib.kg_pods_select_victims(self.h, ptr(pod), len(nodes), ptr(nodes), ptr(off), ptr(vic),
                                                        ptr(sl) if sl is not None else None,
                                                        ptr(mi) if mi is not None else None,
                                                        ptr(vio) if vio is not None else None, ptr(rej), ptr(kept),
                                                        ptr(nvio)))
        return (rej[:len(nodes)], [kept[off[c]:off[c + 1]].astype(bool) for c in range(len(nodes))],
                nvio[:len(nodes)])

    def evaluate_reservation(self, pod: np.ndarray) -> dict:
        """The exact pass's evaluation of one pod on every node (kg_pods_evaluate_reservation): per node pass,
        nominated slot, raw Reservation score, restore state (has_state, matched slots, restored Requested /
        NonZeroRequested / pod count, podRequested), the non-normalized weighted total and the raw DeviceShare score."""
        pod = np.ascontiguousarray(np.asarray(pod, dtype=abi.POD_DTYPE).reshape(1))
        n = self.num_nodes
        out = np.zeros((max(n, 1), abi.RSV_EVAL_WORDS), dtype=np.int64)
        check(self.lib, self.lib.kg_pods_evaluate_reservation(self.h, ptr(pod), ptr(out)))
        out = out[:n]
        names = ("pass", "nominated", "score", "has_state", "matched", "requested_cpu", "requested_mem", "nonzero_cpu",
                 "nonzero_mem", "num_pods", "pod_requested_cpu", "pod_requested_mem", "base", "ds_raw", "order")
        return {k: out[:, q] for q, k in enumerate(names)}

    def debug_numa_merge(self, cases: np.ndarray) -> np.ndarray:
        """The device topology-manager policy merge on int64[n, DBG_MERGE_WORDS] cases (kg_debug_numa_merge);
        returns int64[n, 8]: admit, nil, mask, preferred, score."""
        cases = np.ascontiguousarray(cases, dtype=np.int64).reshape(-1, abi.DBG_MERGE_WORDS)
        out = np.zeros((len(cases), 8), dtype=np.int64)
        check(self.lib, self.lib.kg_debug_numa_merge(self.h, ptr(cases), len(cases), ptr(out)))
        return out

    def debug_least_requested(self, requested, capacity):
        requested = np.ascontiguousarray(requested, dtype=np.int64)
        capacity = np.ascontiguousarray(capacity, dtype=np.int64)
        out = np.zeros(len(requested), dtype=np.int64)
        check(self.lib, self.lib.kg_debug_least_requested(self.h, ptr(requested), ptr(capacity), ptr(out),
                                                          len(requested)))
        return out

    def debug_fast_lrs(self, requested, capacity):
        """(cpu-routine, memory-routine) leastRequestedScore of the wide pass; -1 outside a routine's domain."""
        requested = np.ascontiguousarray(requested, dtype=np.int64)
        capacity = np.ascontiguousarray(capacity, dtype=np.int64)
        oc = np.zeros(len(requested), dtype=np.int64)
        om = np.zeros(len(requested), dtype=np.int64)
        check(self.lib, self.lib.kg_debug_fast_lrs(self.h, ptr(requested), ptr(capacity), ptr(oc), ptr(om),
                                                   len(requested)))
        return oc, om
