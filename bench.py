#!/usr/bin/env python3
"""Benchmark: FIFO pod scheduling throughput of the MI355X engine on BASELINE config 3's cluster.

Workload (BASELINE.json metric "at 100k nodes"): a 100k-node synthetic cluster (SURVEY §8d generator,
seed 20250117) and a queue of pods; profile NodeResourcesFit + LoadAwareScheduling (weights 1/1),
percentageOfNodesToScore=100, ties → lowest index.  One step = scheduling `--pods-per-step` queued pods
(each one filtered + scored on every node and assumed before the next).  The default K=10 steps × 100k pods
schedules the whole 1M-pod queue of config 3.  Inputs are resident in HBM before the timed region (nodes
ingested, pod queue staged); PCIe-inclusive timing of kg_pods_schedule is reported separately.

Other workloads (--workload): c1 (500 nodes, 5k pods: the reference's CPU-runnable case), c2 (10k nodes, 100k pods),
c4 (NodeNUMAResource), c5 (Reservation + DeviceShare + ElasticQuota, 50k nodes), c5ds / c5r (its DeviceShare /
Reservation halves), shipped (the reference's shipped profile, config/manager/scheduler-config.yaml:66-117:
LoadAware + NodeNUMAResource + DeviceShare + Reservation + ElasticQuota on 256-cpu NUMA nodes with 8 GPUs), stock / stockz
(the k8s v1.24 default profile + LoadAware with hostname / also zone-keyed PodTopologySpread and InterPodAffinity).

Single-pod calls (the drop-in's scheduleOne, framework_extender_factory.go:156-185): after the timed region
`--single-pod-calls` more queued pods are scheduled one kg_pods_schedule_staged call each, and the same number through
kg_pods_schedule (host pod in, host decision out); p50 / p99 microseconds per call are reported.

After the timed region: (1) `--profile-pods` more queued pods are scheduled with live kernel timing (HIP events
bracketing every launch on its own stream, kg_profile_enable) — the roofline's kernel time; (2) the first
`--check` placements are compared with the oracle (bit-exact), and (r6) for C3 every timed placement and total
with the committed oracle fixture of the whole queue (tests/golden/c3_queue.npz); (3) the CPU baseline (the oracle, the same
algorithm in C) is timed on a bounded sample with 16 threads and with 1 thread.

N>1 (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N): the node table is replicated on every
rank; with --multi-rank shard its evaluation is sharded over ranks and candidate lists are exchanged with an RCCL
all-gather over xGMI each round; with replica every rank schedules the whole queue on its own table; auto (default)
lets the engine choose from the DESIGN §6 model (replicas below 262,144 nodes for the round profiles).  Total work is
fixed as N grows → "scaling": "strong"; (r6) replicas run N independent queues (rank 0's is the reference one) and
report the pods all ranks scheduled → "scaling": "weak".

Prints ONE JSON line on rank 0 (contract in the task statement).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
B_NODE = 76.0          # SURVEY §8d b_node for Fit + LoadAware: bytes of node columns one evaluation reads

# workload → (nodes, pods per step, batch, pods per wave, default check)
WORKLOADS = {
    "c1": (500, 5_000, 32, 8, 5_000),
    "c2": (10_000, 10_000, 32, 8, 10_000),
    "c3": (100_000, 100_000, 38, 8, 10_000),  # (r5) B = 38: the resolver and the eval→merge chain balance
    "c4": (10_000, 10_000, 16, 1, 2_000),
    "c5": (50_000, 10_000, 32, 4, 10_000),    # (r6) the first step's 10k pods checked against the live oracle
    "c5ds": (50_000, 10_000, 32, 4, 10_000),
    "c5r": (50_000, 10_000, 32, 4, 10_000),
    "shipped": (50_000, 5_000, 32, 4, 1_000),
    "stock": (10_000, 2_000, 32, 8, 2_000),
    "stockz": (10_000, 2_000, 32, 8, 500),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c3")
    ap.add_argument("--nodes", type=int, default=None)
    ap.add_argument("--pods-per-step", type=int, default=None)
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--pods-per-wave", type=int, default=None)
    ap.add_argument("--depth", type=int, default=0, help="pipeline depth (rounds in flight; 0 = engine default)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of each CPU baseline sample")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu-nproc", action="store_true", help="also time the oracle with os.cpu_count() threads")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pcie", action="store_true", help="skip the PCIe-inclusive fresh-engine step (profiling runs)")
    ap.add_argument("--kernel-iters", type=int, default=20)
    ap.add_argument("--profile-pods", type=int, default=None, help="pods scheduled with live kernel timing after "
                    "the timed region (default min(pods per step, 20k))")
    ap.add_argument("--traffic-file", default=None,
                    help="PMC summary (scripts/pmc_summary.py) of the same workload: per-launch HBM bytes "
                         "(default profiles/r02/traffic_<workload>.json)")
    ap.add_argument("--check", type=int, default=None, help="verify the first N placements against the oracle")
    ap.add_argument("--multi-rank", choices=("auto", "shard", "replica"), default="auto",
                    help="N>1: node-sharded evaluation with a per-round exchange, every rank a replica of one GPU, or "
                         "the engine's choice from its model (DESIGN §6)")
    ap.add_argument("--single-pod-calls", type=int, default=200, help="single-pod scheduling calls timed one by one "
                    "after the timed region (0 = skip)")
    return ap.parse_args()


class Dist:
    """torch.distributed (gloo, CPU) for rendezvous/barriers/max-reduce only; the data path is RCCL inside
    the engine."""

    def __init__(self, n):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        if n != self.world:
            raise SystemExit(f"--gpus {n} but WORLD_SIZE={self.world}")
        self.pg = None
        if self.world > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
            self.dist = dist
            self.pg = True

    def barrier(self):
        if self.pg:
            self.dist.barrier()

    def max(self, v: float) -> float:
        if not self.pg:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t[0])

    def bcast_bytes(self, b: bytes | None) -> bytes:
        if not self.pg:
            return b
        obj = [b]
        self.dist.broadcast_object_list(obj, src=0)
        return obj[0]

    def close(self):
        if self.pg:
            self.dist.destroy_process_group()


class Work:
    """One workload: cluster, per-plugin node state, queue generator, engine loader and the oracle run."""

    def __init__(self, name, nodes, cfg):
        from koordinator_amd import synth
        self.name, self.cfg = name, cfg
        self.numa = self.devices = self.rsv = self.quotas = self.preds = None
        S = synth
        if name == "c5":
            self.seed = S.BASE_SEED + 10
            self.cluster, self.devices, self.rsv = S.make_c5_cluster(nodes, seed=self.seed)
            self.make_pods = S.make_c5_pods
        elif name == "shipped":
            self.seed = S.BASE_SEED + 13
            self.cluster, self.numa, self.devices, self.rsv = S.make_shipped_cluster(nodes, seed=self.seed)
            # (r6) prefix-stable queues (C4, shipped): the committed oracle fixture covers any prefix --steps times
            self.make_pods = lambda n, seed: S.make_stream(S.make_shipped_pods, n, seed)
        elif name == "c4":
            self.seed = S.BASE_SEED + 4
            self.cluster, self.numa = S.make_numa_cluster(nodes, seed=self.seed)
            self.make_pods = lambda n, seed: S.make_stream(S.make_numa_pods, n, seed)
        elif name == "c5ds":
            self.seed = S.BASE_SEED + 6
            self.cluster, self.devices = S.make_gpu_cluster(nodes, seed=self.seed)
            self.make_pods = S.make_gpu_pods
        elif name == "c5r":
            self.seed = S.BASE_SEED + 8
            self.cluster, self.rsv = S.make_rsv_cluster(nodes, seed=self.seed)
            self.make_pods = S.make_rsv_pods
        elif name in ("stock", "stockz"):  # (r4) the upstream defaults + PodTopologySpread / InterPodAffinity
            z = name == "stockz"  # stockz: zone-keyed constraints and terms too, 5 % of nodes without a zone label
            self.seed = S.BASE_SEED + 19
            self.cluster = S.make_cluster(nodes, seed=self.seed)
            S.make_pod_groups(self.cluster.existing_pods, seed=self.seed + 3, zones=z)
            self.preds = S.make_predicates(nodes, S.make_pods(0), seed=self.seed + 2,
                                           no_zone=0.05 if z else 0.0)[1]  # labels + taints
            self.make_pods = lambda n, seed: S.make_pod_groups(S.make_pods(n, seed=seed), seed=seed + 4, zones=z)
        else:  # c1, c3: Fit + LoadAware
            self.seed = S.BASE_SEED + (1 if name == "c1" else 3)
            self.cluster = S.make_cluster(nodes, seed=self.seed)
            # (r6) C3's queue is prefix-stable, so the committed oracle fixture covers whatever prefix --steps times
            self.make_pods = S.make_pods_stream if name == "c3" else S.make_pods

    QUOTA_BASIS = 25_000  # (r6) shipped: quotas sized on the queue's first 25k pods, whatever --steps (fixture-stable)

    def set_queue(self, pods):
        """ElasticQuota groups sized on the queue's demand (C5: 16 groups whose limits run out mid-queue)."""
        from koordinator_amd import synth
        if self.name == "c5":
            self.quotas = synth.make_c5_quotas(pods, seed=self.seed + 2)
        elif self.name == "shipped":
            self.quotas = synth.make_c5_quotas(pods[:self.QUOTA_BASIS], seed=self.seed + 2)

    def load(self, e):
        from koordinator_amd import synth
        if self.name == "shipped":
            synth.load_shipped_into(e, self.cluster, self.numa, self.devices, self.rsv, self.quotas)
        elif self.name == "c5":
            synth.load_c5_into(e, self.cluster, self.devices, self.rsv, self.quotas)
        elif self.numa is not None:
            synth.load_numa_into(e, self.cluster, self.numa)
        elif self.devices is not None:
            synth.load_gpu_into(e, self.cluster, self.devices)
        elif self.rsv is not None:
            synth.load_rsv_into(e, self.cluster, self.rsv)
        else:
            synth.load_into(e, self.cluster)
        if self.preds is not None:
            e.upsert_predicates(self.preds)

    def oracle_run(self, pods, threads):
        """(node idx, oracle name) of the oracle's sequential FIFO run over `pods` from the initial state."""
        from oracle import oracle
        cl, cfg = self.cluster, self.cfg
        st = oracle.states(cl.n)
        oracle.add_pods(cfg, st, cl.existing_pods, cl.existing_node)
        if self.name in ("stock", "stockz"):
            g = oracle.groups_init(cl.n, cl.existing_pods, cl.existing_node)
            on, _, _ = oracle.schedule_resv(cfg, cl.nodes, cl.metrics, st, None, pods, cl.now_ns, n_threads=threads,
                                            preds=self.preds, groups=g)
            return on, "oracle/reservation.c or_schedule_resv_full with defaults.c pod groups (Parallelizer chunking)"
        if self.rsv is not None:
            on, _, _ = oracle.schedule_resv(cfg, cl.nodes, cl.metrics, st, self.rsv.copy(), pods, cl.now_ns,
                                            devices=None if self.devices is None else self.devices.copy(),
                                            quotas=None if self.quotas is None else self.quotas.copy(),
                                            n_threads=threads,
                                            numa_buf=None if self.numa is None else oracle.numa_states(self.numa))
            return on, "oracle/reservation.c or_schedule_resv_full (Parallelizer chunking)"
        if self.devices is not None:
            on, _, _, _ = oracle.schedule_full(cfg, cl.nodes, cl.metrics, st, pods, cl.now_ns, threads,
                                               devices=self.devices.copy())
            return on, "oracle/oracle.c or_schedule_full (Parallelizer chunking)"
        if self.numa is not None:
            on, _ = oracle.schedule_numa(cfg, cl.nodes, cl.metrics, st, oracle.numa_states(self.numa), pods,
                                         cl.now_ns, threads)
            return on, "oracle/oracle.c or_schedule_numa (Parallelizer chunking)"
        on, _ = oracle.schedule(cfg, cl.nodes, cl.metrics, st, pods, cl.now_ns, threads)
        return on, "oracle/oracle.c or_schedule (Parallelizer chunking)"


# (r6) the oracle's schedule of the whole queue: tests/golden/make_c3_fixture.py, make_bench_fixture.py
FIXTURES = {"c3": "c3_queue.npz", "c4": "c4_queue.npz", "shipped": "shipped_queue.npz"}


def fixture_check(wl, n_nodes, pods, node_idx, score, total):
    """(r6) Compare the first `total` placements and totals with the committed oracle fixture of this workload's queue
    (outside the timed region).  The fixture holds the oracle's sequential schedule of the same seeded queue; its
    per-segment digests prove the queue is the one this run generated.  Returns (ok, pods checked, source, totals
    compared) or None when no fixture covers this run."""
    import hashlib
    name = FIXTURES.get(wl)
    path = os.path.join(ROOT, "tests", "golden", name) if name else None
    if not path or not os.path.exists(path):
        return None
    z = np.load(path)
    meta = json.loads(str(z["meta"]))
    seg = int(meta["segment"])
    if meta["nodes"] != n_nodes or meta["pods"] < total or total % seg != 0:
        return None
    for s in range(total // seg):
        if hashlib.sha256(np.ascontiguousarray(pods[s * seg:(s + 1) * seg]).tobytes()).hexdigest() != str(z["seg_sha"][s]):
            return None
    ok = bool(np.array_equal(z["node"][:total], node_idx[:total]))
    if "score" in z.files:  # C3: the totals too; C4 / shipped fixtures hold the placements
        ok = ok and bool(np.array_equal(z["score"][:total].astype(np.int64), score[:total]))
    return ok, total, f"tests/golden/{name} ({meta['oracle']}, {meta['pods']} pods)", "score" in z.files


def workload_profile(wl):
    """(profile, LoadAwareSchedulingArgs) of a workload (None = the engine defaults)."""
    from koordinator_amd import framework as F
    profile = None
    if wl == "c4":
        profile = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.NODE_NUMA_RESOURCE),
                            score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.NODE_NUMA_RESOURCE: 1})
    elif wl == "c5ds":  # shipped weights: DeviceShare 1 (config/manager/scheduler-config.yaml:82-91)
        profile = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.DEVICE_SHARE),
                            score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.DEVICE_SHARE: 1})
    elif wl == "c5":  # one profile: Reservation 5000, DeviceShare 1, ElasticQuota admission (PreFilter only)
        profile = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.RESERVATION, F.DEVICE_SHARE),
                            score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.RESERVATION: 5000, F.DEVICE_SHARE: 1})
    elif wl == "c5r":  # shipped weights: Reservation 5000 (config/manager/scheduler-config.yaml:90-91)
        profile = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.RESERVATION),
                            score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.RESERVATION: 5000})
    elif wl in ("stock", "stockz"):  # k8s v1.24 v1beta2 default weights + LoadAware; hostname spread / inter-pod affinity
        profile = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.TAINT_TOLERATION, F.NODE_AFFINITY,
                                    F.POD_TOPOLOGY_SPREAD, F.INTER_POD_AFFINITY),
                            score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.TAINT_TOLERATION: 1, F.NODE_AFFINITY: 1,
                                   F.BALANCED_ALLOCATION: 1, F.POD_TOPOLOGY_SPREAD: 2, F.INTER_POD_AFFINITY: 1})
    la = None
    if wl == "shipped":  # config/manager/scheduler-config.yaml:29-117: plugins, weights and LoadAware args
        profile = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.NODE_NUMA_RESOURCE, F.DEVICE_SHARE,
                                    F.RESERVATION),
                            score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.NODE_NUMA_RESOURCE: 1, F.DEVICE_SHARE: 1,
                                   F.RESERVATION: 5000})
        la = F.LoadAwareSchedulingArgs(filter_expired_node_metrics=False, node_metric_expiration_seconds=300)
    return profile, la


def cpu_sample(work, pods, budget_s, threads):
    """Oracle on this host over a bounded prefix of the queue: (pods, seconds, description)."""
    probe = min(64, len(pods))
    t0 = time.perf_counter()
    work.oracle_run(pods[:probe], threads)
    per_pod = (time.perf_counter() - t0) / probe
    m = int(min(len(pods), max(probe, budget_s / max(per_pod, 1e-9))))
    t0 = time.perf_counter()
    _, desc = work.oracle_run(pods[:m], threads)
    return m, time.perf_counter() - t0, desc


def pmc_traffic(path, kernel, nodes, batch, ppw, depth):
    """Per-launch HBM bytes of `kernel` (FETCH_SIZE x2 + WRITE_SIZE, gfx950-corrected by scripts/pmc_summary.py)
    from a committed rocprofv3 --pmc summary, if it was collected on this exact workload geometry."""
    try:
        with open(path) as fh:
            d = json.load(fh)
    except (OSError, ValueError):
        return None, None, None
    m = d.get("_meta", {})
    if (m.get("nodes"), m.get("batch_pods"), m.get("pods_per_wave"), m.get("depth")) != (nodes, batch, ppw, depth) \
            or kernel not in d:
        return None, None, None
    return d[kernel]["traffic_bytes"], os.path.relpath(path, ROOT), d[kernel].get("rocprof_avg_ns")


def main():
    args = parse()
    d = Dist(args.gpus)
    from koordinator_amd import Engine, framework
    from koordinator_amd.engine import nccl_unique_id

    nccl_id = None
    if d.world > 1:
        nccl_id = d.bcast_bytes(nccl_unique_id() if d.rank == 0 else None)
    wl = args.workload
    nodes0, pps0, b0, ppw0, check0 = WORKLOADS[wl]
    args.nodes = args.nodes or nodes0
    args.pods_per_step = args.pods_per_step or pps0
    args.batch = args.batch or b0
    args.pods_per_wave = args.pods_per_wave or ppw0
    args.check = check0 if args.check is None else args.check
    if wl == "c1" and args.steps == 10:
        args.steps = 1  # the whole 5k-pod queue of config 1
    profile, la = workload_profile(wl)
    cfg = framework.build_config(batch_pods=args.batch, pods_per_wave=args.pods_per_wave, device_id=d.local_rank,
                                 profile=profile, pipeline_depth=args.depth, la=la, multi_rank=args.multi_rank)
    work = Work(wl, args.nodes, cfg)
    cluster = work.cluster
    total = args.steps * args.pods_per_step
    n_prof = args.profile_pods if args.profile_pods is not None else min(args.pods_per_step, 20_000)
    n_single = args.single_pod_calls if d.world == 1 else 0
    pods = work.make_pods(total + n_prof + n_single, seed=work.seed + 1)
    work.set_queue(pods)

    def engine():
        e = Engine(cfg, cluster.n, rank=d.rank, n_ranks=d.world, nccl_id=nccl_id)
        work.load(e)
        return e

    # warmup on a throw-away engine (same cluster, different pods): code objects, caches, RCCL channels
    if args.warmup > 0:
        wp = work.make_pods(args.warmup * min(args.pods_per_step, 20_000), seed=work.seed + 7)
        with engine() as ew:
            ew.stage(wp)
            ew.schedule_staged(0, len(wp))

    e = engine()
    shard_ranks, replica_ranks = e.ranks  # (r6) the engine's resolved multi-rank mode
    # (r6) replicas (the multi-rank mode chose no sharding: the path then does not shard): N independent
    # schedulers, each over its own queue of the same shape — rank 0 keeps the reference queue (the oracle checks it),
    # rank r > 0 draws seed + 1 + 1000·r; the value is the pods all ranks scheduled per second ("scaling": "weak")
    independent = d.world > 1 and replica_ranks > 1
    if independent and d.rank > 0:
        e.close()
        pods = work.make_pods(total + n_prof + n_single, seed=work.seed + 1 + 1000 * d.rank)
        work.set_queue(pods)
        e = engine()
    e.stage(pods)
    d.barrier()
    t0 = time.perf_counter()
    rounds = 0
    active_s = 0.0  # resolvers' in-kernel active time (after the chain wait; s_memrealtime), round profiles
    slow_pods = 0.0  # resolver diagnostics: pods that re-scored modified rows (the chain's slow path)
    for k in range(args.steps):
        st = e.schedule_staged(k * args.pods_per_step, args.pods_per_step)
        rounds += int(st["device_batches"])
        active_s += float(st["reserved"][2])
        slow_pods += float(st["reserved"][0])
        if d.rank == 0:
            print(f"[bench] step {k + 1}/{args.steps} done", file=sys.stderr, flush=True)
    t1 = time.perf_counter()
    d.barrier()
    elapsed = d.max(t1 - t0)
    node_idx, score_tot = e.fetch(0, total)
    placed = int((node_idx >= 0).sum())

    # live kernel timing on the real pipelined runner, continuing the same queue (outside the timed region)
    live = {}
    if n_prof > 0:
        e.profile(True)
        e.schedule_staged(total, n_prof)
        live = {k: {"avg_ms": ms / n, "launches": n} for k, (ms, n) in e.profile_read().items()}
        e.profile(False)
    # the drop-in's per-pod call (scheduleOne): single-pod kg_pods_schedule_staged calls continuing the queue, and the
    # same pods again through kg_pods_schedule (host record in, host decision out) on a fresh engine
    single = None
    if n_single > 0:
        lat = []
        base = total + n_prof
        for j in range(n_single):
            tt = time.perf_counter()
            e.schedule_staged(base + j, 1)
            lat.append(time.perf_counter() - tt)
        lat = np.array(lat) * 1e6
        single = {"staged_p50_us": float(np.percentile(lat, 50)), "staged_p99_us": float(np.percentile(lat, 99)),
                  "calls": n_single}
        with engine() as es:
            lat2 = []
            for j in range(n_single):
                tt = time.perf_counter()
                es.schedule(pods[base + j:base + j + 1])
                lat2.append(time.perf_counter() - tt)
        lat2 = np.array(lat2) * 1e6
        single.update({"host_p50_us": float(np.percentile(lat2, 50)), "host_p99_us": float(np.percentile(lat2, 99)),
                       "note": "kg_pods_schedule_staged(count=1) continuing the staged queue after the timed region; "
                               "kg_pods_schedule(1 host pod) on a fresh engine: decode + upload + schedule + result"})
    # isolated replays of one round's kernels (warm caches, no concurrency) for comparison
    rsv_path = wl in ("c5r", "c5", "shipped", "stock", "stockz")
    names = (("rsv_eval", "rsv_select") if rsv_path else
             ("eval_round", "merge_round", "resolve_round") + (("ds_max_round", "ds_norm_reduce") if wl == "c5ds" else ()))
    isolated = {name: e.bench_kernel(which, args.kernel_iters) for which, name in enumerate(names)}

    # roofline kernel: the wide pass — the only kernel whose work scales with node evaluations.  One launch
    # processes the round's B pods against every node row of this rank's shard, reading each row once:
    # algorithmic bytes = rows × b_node + the candidate lists written + the pods read.
    dom = {"c5ds": "ds_max_round", "c5r": "rsv_eval", "c5": "rsv_eval", "shipped": "rsv_eval",
           "stock": "rsv_eval", "stockz": "rsv_eval"}.get(wl, "eval_round")
    n_local = -(-cluster.n // d.world)
    nt = max(1, -(-n_local // 256))
    B = 1 if rsv_path else args.batch
    if wl == "c5ds":  # ds_max_round also reads the 272-B GPU row and writes a 4-B packed value per (pod, node)
        algo = n_local * (B_NODE + 272.0) + B * n_local * 4.0 + B * nt * 8.0
    elif wl in ("stock", "stockz"):  # one pod per exact pass (rsv_eval): per node the Fit / LoadAware columns, the 32-B NodePred,
        # ~4 group counters, and the 8 + 4 + 8 B of values it writes
        algo = n_local * (B_NODE + 32.0 + 16.0 + 20.0)
    elif rsv_path:  # the exact wide pass (xr_eval, live time folded under "rsv_eval"): one launch scores the round's
        # pods (kXrPods = 32, or fewer) against every node.  Per launch: the node columns + rsv_n once, the 192-B slot
        # rows of nodes holding reservations, the 272-B GPU row per node when the round has device pods, the NUMA rows
        # (NumaStatic 144 B + NodeAllocation 104 B), and per (pod, node) the 8-B packed value (+ 4-B NUMA affinity)
        ev = live.get("rsv_eval", {})
        pods_per_launch = (n_prof / ev["launches"]) if ev.get("launches") else 1.0
        prof_pods = pods[total:total + n_prof] if n_prof > 0 else pods[:1]
        has_dev = work.devices is not None and bool(prof_pods["device_requests"].any())
        algo = n_local * (B_NODE + 4) + int((work.rsv["n"] > 0).sum()) * 192.0 + (n_local * 272.0 if has_dev else 0.0)
        algo += pods_per_launch * n_local * 8.0
        if work.numa is not None:
            algo += n_local * (144.0 + 104.0) + pods_per_launch * n_local * 4.0
        B = pods_per_launch
    else:  # (r4) one top-8 list per (pod, tile group of 4 tiles) written from 64 tiles on, per tile below
        algo = n_local * B_NODE + B * (-(-nt // 4) if nt >= 64 else nt) * 8 * 8.0 + B * 96.0
    dom_ms = live.get(dom, {}).get("avg_ms") or isolated[dom][0]
    achieved = algo / (dom_ms * 1e-3) / 1e9
    per_eval = B * n_local * B_NODE / (dom_ms * 1e-3) / 1e9  # §8d per-evaluation accounting (one table read per pod)

    # PCIe-inclusive path (host pods in, host decisions out) on a fresh engine, one step
    pcie = None
    if d.world == 1 and not args.no_pcie:
        with engine() as ep:
            tt = time.perf_counter()
            ep.schedule(pods[: args.pods_per_step])
            pcie = args.pods_per_step / (time.perf_counter() - tt)

    check = None
    fx = fixture_check(wl, cluster.n, pods, node_idx, score_tot, total) if d.rank == 0 else None
    if args.check and d.rank == 0:
        nchk = min(args.check, total)
        print(f"[bench] oracle check of the first {nchk} placements", file=sys.stderr, flush=True)
        on, _ = work.oracle_run(pods[:nchk], args.cpu_threads)
        check = bool(np.array_equal(on, node_idx[:nchk]))

    cpu = None
    if d.rank == 0 and d.world == 1 and not args.no_cpu_baseline:
        print("[bench] cpu baseline samples", file=sys.stderr, flush=True)
        threads = args.cpu_threads
        m, dt, desc = cpu_sample(work, pods[:total], args.cpu_seconds, threads)
        m1, dt1, _ = cpu_sample(work, pods[:total], args.cpu_seconds / 3, 1)
        cpu = {"value": m / dt, "unit": "pods/s", "cores": threads, "kind": "port",
               "sample": f"first {m} pods of the same queue, {cluster.n} nodes, {desc}, {threads} thread(s); "
                         f"host nproc={os.cpu_count()} (the GPU box's CPU share is 16 threads per GPU)",
               "node_evals_per_sec": m * cluster.n / dt,
               "single_thread": {"value": m1 / dt1, "sample_pods": m1}}
        nproc = os.cpu_count() or threads
        if args.cpu_nproc and nproc > threads:  # §8d: the Parallelizer widened to every host thread as well
            mn, dtn, _ = cpu_sample(work, pods[:total], args.cpu_seconds / 2, nproc)
            cpu["nproc_threads"] = {"value": mn / dtn, "threads": nproc, "sample_pods": mn}
        elif nproc > threads:
            # (r6) the GPU box gives one GPU a 16-thread CPU share (nproc shows the whole machine), so the default run
            # does not start nproc threads; the nproc-wide Parallelizer is bounded above by linear scaling of the
            # 16-thread rate (measured 1 → 16 threads: the efficiency below)
            cpu["nproc_threads_linear_bound"] = {
                "value": m / dt * nproc / threads, "threads": nproc,
                "note": "upper bound: the %d-thread rate scaled linearly to nproc (the measured 1 -> %d-thread "
                        "efficiency is %.2f); --cpu-nproc measures it when the box's CPU share allows"
                        % (threads, threads, (m / dt) / (m1 / dt1) / threads)}

    tfile = args.traffic_file or next((f for f in (os.path.join(ROOT, "profiles", r, f"traffic_{wl}.json")
                                                   for r in ("r06", "r05", "r04", "r03", "r02")) if os.path.exists(f)),
                                      os.path.join(ROOT, "profiles", "r02", f"traffic_{wl}.json"))
    # live timing folds every wide pass under one name: the kernel rocprof sees
    pmc_name = {"c4": "eval_round_numa", "c5": "xr_eval", "c5r": "xr_eval", "shipped": "xr_eval",
                "stock": "rsv_eval", "stockz": "rsv_eval"}.get(wl, dom)
    traffic, traffic_src, rocprof_ns = (pmc_traffic(tfile, pmc_name, cluster.n, args.batch, args.pods_per_wave,
                                                    args.depth) if d.world == 1 else (None, None, None))
    # period decomposition of the round pipeline (Fit + LoadAware / DeviceShare round profiles): per round, the serial
    # resolver's active time (its own s_memrealtime stamps, after the chain wait) against the wall-clock period, and the
    # wide pass + merge stream (live HIP events) against the depth rounds it overlaps
    period = None
    if not rsv_path and rounds > 0:
        per = elapsed / rounds
        ev_ms = live.get("eval_round", {}).get("avg_ms") or live.get("ds_max_round", {}).get("avg_ms")
        mg_ms = live.get("merge_round", {}).get("avg_ms")
        depth = args.depth or (1 if wl == "c5ds" else 2)
        res_us = active_s / rounds * 1e6
        # the resolver's algorithmic bytes per launch: the round's records and pods (LDS-DMA) + the rows it writes back
        res_bytes = B * (1024.0 + 96.0) + B * 80.0
        period = {"us_per_round": per * 1e6, "pods_per_round": total / rounds,
                  "resolver_active_us": res_us if active_s > 0 else None,
                  "resolver_share": active_s / elapsed if active_s > 0 else None,
                  "eval_us": ev_ms * 1e3 if ev_ms else None, "merge_us": mg_ms * 1e3 if mg_ms else None,
                  "depth": depth,
                  "slow_pod_frac": slow_pods / total if total else None,
                  "eval_stream_share": ((ev_ms or 0) + (mg_ms or 0)) * 1e-3 / (depth * per) if ev_ms else None,
                  "dominant": ("resolver" if active_s > 0 and active_s / elapsed >= ((ev_ms or 0) + (mg_ms or 0)) * 1e-3
                               / (depth * per) else "eval_stream"),
                  "resolver_roofline": ({"algo_bytes_per_launch": res_bytes,
                                         "frac": res_bytes / (res_us * 1e-6) / 1e9 / HBM_PEAK_GBS}
                                        if active_s > 0 else None),
                  "note": "resolver_share = in-kernel active time / wall time of the timed steps (the serial chain "
                          "sets the period when it is near 1); eval_stream_share = (eval + merge) / (depth x period)"}
    if d.world == 1:
        parallelism = "1 GPU"
    elif replica_ranks > 1:
        parallelism = ("replicas x%d (multi_rank %s: the sharding model of DESIGN §6 predicts no gain at %d nodes, so "
                       "every rank is an independent scheduler over its own %d-pod queue on its own full table, no "
                       "exchange; value = the pods all ranks scheduled per second)"
                       % (d.world, args.multi_rank, cluster.n, total))
    elif wl in ("stock", "stockz"):
        parallelism = ("replicas x%d (per-pod exact pass: every rank evaluates its full replica, no exchange)" % d.world)
    elif rsv_path:
        parallelism = ("node-sharded exact rounds x%d (replicated table; per round an RCCL all-gather of the pod "
                       "statistics and of the merged records)" % shard_ranks)
    else:
        parallelism = "node-sharded x%d (replicated table, RCCL all-gather)" % shard_ranks
    if d.rank == 0:
        pods_s = total * (d.world if independent else 1) / elapsed
        desc = {
            "c1": "C1 cluster: %d nodes, %d-pod FIFO queue, NodeResourcesFit+LoadAwareScheduling, %d pods per step",
            "c2": "C2 cluster: %d nodes, %d-pod FIFO queue, NodeResourcesFit+LoadAwareScheduling, %d pods per step",
            "shipped": "shipped profile (config/manager/scheduler-config.yaml:66-117): %d 2-socket 256-cpu NUMA nodes x "
                       "8 GPUs (30%% with 1-4 cpu/memory reservations), %d-pod FIFO queue (70%% cpuset LSR/LSE, 30%% "
                       "GPU-share, 20%% reservation-owned, 80%% in 16 ElasticQuota groups), NodeResourcesFit+"
                       "LoadAwareScheduling+NodeNUMAResource+DeviceShare+Reservation (w 1/1/1/1/5000)+ElasticQuota, "
                       "batched exact rounds of 32 pods, %d pods per step",
            "c3": "C3 cluster: %d nodes, %d-pod FIFO queue, NodeResourcesFit+LoadAwareScheduling, %d pods per step",
            "c4": "C4 cluster: %d 2-socket 256-cpu nodes (node count: builder's choice, BASELINE names none), "
                  "%d-pod FIFO queue (70%% cpuset LSR/LSE), NodeResourcesFit+LoadAwareScheduling+NodeNUMAResource, "
                  "%d pods per step",
            "c5ds": "C5 (DeviceShare part): %d nodes x 8 GPUs, %d-pod FIFO queue (30%% GPU-share), "
                    "NodeResourcesFit+LoadAwareScheduling+DeviceShare, %d pods per step",
            "c5": "C5 (one profile): %d nodes x 8 GPUs (30%% with 1-4 cpu/memory reservations, 64 owner groups), "
                  "%d-pod FIFO queue (30%% GPU-share, 20%% reservation-owned, 80%% in 16 ElasticQuota groups), "
                  "NodeResourcesFit+LoadAwareScheduling+Reservation (w 5000)+DeviceShare+ElasticQuota admission, "
                  "batched exact rounds of 32 pods, %d pods per step",
            "c5r": "C5 (Reservation part): %d nodes (30%% with 1-4 reservations), %d-pod FIFO queue (20%% "
                   "reservation-owned), NodeResourcesFit+LoadAwareScheduling+Reservation (w 5000), batched exact "
                   "rounds of 32 pods, %d pods per step",
            "stock": "k8s v1.24 default profile + LoadAware: %d nodes (labels, NoSchedule / PreferNoSchedule taints), "
                     "%d-pod FIFO queue of 8 deployments in 4 teams (40%% DoNotSchedule / 50%% ScheduleAnyway hostname "
                     "spread, 15%% required anti-affinity, 10%% required affinity, 30%% preferred terms), NodeResourcesFit"
                     "+LoadAware+TaintToleration+NodeAffinity+BalancedAllocation+PodTopologySpread(w2)+InterPodAffinity, "
                     "one pod per exact pass, %d pods per step",
            "stockz": "k8s v1.24 default profile + LoadAware with zone keys: %d nodes in 4 zones (5%% without the zone "
                      "label), %d-pod FIFO queue of 8 deployments in 4 teams (hostname and zone spread constraints in "
                      "random order; a third of required anti-affinity, half of required affinity and half of "
                      "preferred terms zone-keyed), the stock profile's plugins and weights, one pod per exact pass, "
                      "%d pods per step",
        }[wl] % (cluster.n, total, args.pods_per_step)
        out = {
            "metric": {"c3": "pods scheduled/sec at 100k nodes (node-evals/sec alongside)",
                       "c1": "pods scheduled/sec, config 1 (500 nodes; node-evals/sec alongside)",
                       "c2": "pods scheduled/sec, config 2 (10k nodes; node-evals/sec alongside)",
                       "shipped": "pods scheduled/sec, the shipped koord-scheduler profile (node-evals/sec alongside)",
                       "c4": "pods scheduled/sec, NodeNUMAResource cpuset/NUMA profile (node-evals/sec alongside)",
                       "c5ds": "pods scheduled/sec, DeviceShare GPU-share profile (node-evals/sec alongside)",
                       "c5r": "pods scheduled/sec, Reservation profile (node-evals/sec alongside)",
                       "c5": "pods scheduled/sec, Reservation+DeviceShare+ElasticQuota profile (node-evals/sec "
                             "alongside)",
                       "stock": "pods scheduled/sec, default plugins + hostname PodTopologySpread / InterPodAffinity "
                                "(node-evals/sec alongside)",
                       "stockz": "pods scheduled/sec, default plugins + hostname / zone PodTopologySpread / "
                                 "InterPodAffinity (node-evals/sec alongside)"}[wl],
            "value": pods_s,
            "unit": "pods/s",
            "n_gpus": d.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak" if independent else "strong",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic (SURVEY §8d generator, seed %d)" % work.seed,
            "config": {"workload": desc, "nodes": cluster.n, "pods": total, "batch_pods": args.batch,
                       "pods_per_wave": args.pods_per_wave, "pipeline_depth": args.depth or "default",
                       "parallelism": parallelism},
            "node_evals_per_sec": pods_s * cluster.n,
            "placed": placed,
            "device_rounds": rounds,
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                         "kernel_ms": dom_ms, "algo_bytes_per_launch": algo,
                         "timing": "live HIP events around every launch of %d extra queued pods (kg_profile_enable)"
                                   % n_prof if dom in live else "isolated replay (kg_bench_kernel)",
                         "per_evaluation_rate_gbs": per_eval, "pods_per_launch": B,
                         "traffic_rate_gbs": traffic / (dom_ms * 1e-3) / 1e9 if traffic else None,
                         "traffic_frac": traffic / (dom_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if traffic else None,
                         # the same kernel's rocprof average (trace pass of the committed PMC command): live
                         # events also hold the command processor's dispatch of each launch
                         "rocprof_kernel_ms": rocprof_ns / 1e6 if rocprof_ns else None,
                         "frac_rocprof": algo / (rocprof_ns * 1e-9) / 1e9 / HBM_PEAK_GBS if rocprof_ns else None,
                         "live_ms": {k: v["avg_ms"] for k, v in live.items()},
                         "live_launches": {k: v["launches"] for k, v in live.items()},
                         "isolated_ms": {k: v[0] for k, v in isolated.items()},
                         "period": period},
            "cpu_baseline": cpu,
            "pcie_inclusive_pods_per_sec": pcie,
            "single_pod_call": single,
            # (r6) the whole timed queue against the committed oracle fixture when one covers it, and the live oracle
            # on the first --check pods (the fixture's own check on this box)
            "oracle_check": (None if check is None and fx is None else
                             (check is not False) and (fx is None or fx[0])),
            "oracle_check_pods": max(min(args.check, total) if args.check else 0, fx[1] if fx else 0),
            "oracle_check_live_pods": min(args.check, total) if args.check else 0,
            "oracle_check_fixture": ({"ok": fx[0], "pods": fx[1], "placements_and_totals": fx[3], "source": fx[2]}
                                     if fx else None),
        }
        print(json.dumps(out), flush=True)
    e.close()
    d.close()


if __name__ == "__main__":
    main()
