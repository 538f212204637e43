#!/usr/bin/env python3
"""Benchmark: FIFO pod scheduling throughput of the MI355X engine on BASELINE config 3's cluster.

Workload (BASELINE.json metric "at 100k nodes"): a 100k-node synthetic cluster (SURVEY §8d generator,
seed 20250117) and a queue of pods; profile NodeResourcesFit + LoadAwareScheduling (weights 1/1),
percentageOfNodesToScore=100, ties → lowest index.  One step = scheduling `--pods-per-step` queued pods
(each one filtered + scored on every node and assumed before the next).  The default K=10 steps × 100k pods
schedules the whole 1M-pod queue of config 3.  Inputs are resident in HBM before the timed region (nodes
ingested, pod queue staged); PCIe-inclusive timing of kg_pods_schedule is reported separately.

N>1 (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N): the node table is replicated
and its evaluation sharded over ranks; candidate lists are exchanged with RCCL all-gather over xGMI.  Total
work is fixed as N grows → "scaling": "strong".

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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=("c3", "c4", "c5", "c5r"), default="c3",
                    help="c3: Fit+LoadAware at 100k nodes (the BASELINE metric); c4: + NodeNUMAResource cpuset/NUMA "
                         "on 2-socket 256-cpu nodes")
    ap.add_argument("--nodes", type=int, default=None, help="default 100k (c3) / 10k (c4)")
    ap.add_argument("--pods-per-step", type=int, default=None, help="default 100k (c3) / 10k (c4)")
    ap.add_argument("--batch", type=int, default=None, help="default 32 (c3, c5) / 16 (c4)")
    ap.add_argument("--pods-per-wave", type=int, default=None, help="default 8 (c3) / 1 (c4) / 4 (c5)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="budget of the CPU baseline sample")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--kernel-iters", type=int, default=50)
    ap.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "r01", "traffic_c3.json"),
                    help="PMC summary (scripts/pmc_summary.py) of the same workload: per-launch HBM bytes")
    ap.add_argument("--check", type=int, default=0, help="verify the first N placements against the oracle")
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


def cpu_baseline(cfg, cluster, pods, budget_s, threads, numa=None, devices=None, rsv=None):
    """Oracle (C restatement of the same Go algorithm, oracle/oracle.c [+ numa.c / deviceshare.c]) on this host,
    bounded sample."""
    from oracle import oracle
    st = oracle.states(cluster.n)
    oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
    buf = oracle.numa_states(numa) if numa is not None else None
    dev = devices.copy() if devices is not None else None
    rs = rsv.copy() if rsv is not None else None

    def run(p):
        if rs is not None:  # or_schedule_resv is single-threaded
            oracle.schedule_resv(cfg, cluster.nodes, cluster.metrics, st, rs, p, cluster.now_ns)
        elif dev is not None:
            oracle.schedule_full(cfg, cluster.nodes, cluster.metrics, st, p, cluster.now_ns, threads, devices=dev)
        elif buf is None:
            oracle.schedule(cfg, cluster.nodes, cluster.metrics, st, p, cluster.now_ns, threads)
        else:
            oracle.schedule_numa(cfg, cluster.nodes, cluster.metrics, st, buf, p, cluster.now_ns, threads)

    probe = 64
    t0 = time.perf_counter()
    run(pods[:probe])
    per_pod = (time.perf_counter() - t0) / probe
    m = int(min(len(pods) - probe, max(probe, budget_s / max(per_pod, 1e-9))))
    t0 = time.perf_counter()
    run(pods[probe:probe + m])
    dt = time.perf_counter() - t0
    return m, dt


def pmc_traffic(path, kernel, nodes, batch, ppw):
    """Per-launch HBM bytes of `kernel` (FETCH_SIZE x2 + WRITE_SIZE, gfx950-corrected by scripts/pmc_summary.py)
    from a committed rocprofv3 --pmc summary, if it was collected on this exact workload geometry."""
    try:
        with open(path) as fh:
            d = json.load(fh)
    except (OSError, ValueError):
        return None, None
    m = d.get("_meta", {})
    if (m.get("nodes"), m.get("batch_pods"), m.get("pods_per_wave")) != (nodes, batch, ppw) or kernel not in d:
        return None, None
    return d[kernel]["traffic_bytes"], os.path.relpath(path, ROOT)


def main():
    args = parse()
    d = Dist(args.gpus)
    from koordinator_amd import Engine, framework, synth
    from koordinator_amd.engine import nccl_unique_id

    nccl_id = None
    if d.world > 1:
        nccl_id = d.bcast_bytes(nccl_unique_id() if d.rank == 0 else None)
    c4 = args.workload == "c4"
    c5 = args.workload == "c5"
    c5r = args.workload == "c5r"
    args.nodes = args.nodes or (10_000 if c4 else (50_000 if (c5 or c5r) else 100_000))
    args.pods_per_step = args.pods_per_step or (10_000 if (c4 or c5 or c5r) else 100_000)
    # geometry sweeps: profiles/r01/c4_sweep.txt, c5_sweep.txt
    args.pods_per_wave = args.pods_per_wave or (1 if c4 else (4 if c5 else 8))
    args.batch = args.batch or (16 if c4 else 32)
    F = framework
    profile = None
    if c4:
        profile = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.NODE_NUMA_RESOURCE),
                            score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.NODE_NUMA_RESOURCE: 1})
    elif c5:  # shipped weights: DeviceShare 1 (config/manager/scheduler-config.yaml:82-91)
        profile = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.DEVICE_SHARE),
                            score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.DEVICE_SHARE: 1})
    elif c5r:  # shipped weights: Reservation 5000 (config/manager/scheduler-config.yaml:90-91)
        profile = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.RESERVATION),
                            score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.RESERVATION: 5000})
    cfg = framework.build_config(batch_pods=args.batch, pods_per_wave=args.pods_per_wave, device_id=d.local_rank,
                                 profile=profile)
    numa = devices = rsv = None
    if c4:
        seed = synth.BASE_SEED + 4
        cluster, numa = synth.make_numa_cluster(args.nodes, seed=seed)
        make_pods = synth.make_numa_pods
    elif c5:
        seed = synth.BASE_SEED + 6
        cluster, devices = synth.make_gpu_cluster(args.nodes, seed=seed)
        make_pods = synth.make_gpu_pods
    elif c5r:
        seed = synth.BASE_SEED + 8
        cluster, rsv = synth.make_rsv_cluster(args.nodes, seed=seed)
        make_pods = synth.make_rsv_pods
    else:
        seed = synth.BASE_SEED + 3
        cluster = synth.make_cluster(args.nodes, seed=seed)
        make_pods = synth.make_pods
    total = args.steps * args.pods_per_step
    pods = make_pods(total, seed=seed + 1)

    def engine():
        e = Engine(cfg, cluster.n, rank=d.rank, n_ranks=d.world, nccl_id=nccl_id)
        if c4:
            synth.load_numa_into(e, cluster, numa)
        elif c5:
            synth.load_gpu_into(e, cluster, devices)
        elif c5r:
            synth.load_rsv_into(e, cluster, rsv)
        else:
            synth.load_into(e, cluster)
        return e

    # warmup on a throw-away engine (same cluster, different pods): code objects, caches, RCCL channels
    if args.warmup > 0:
        wp = make_pods(args.warmup * min(args.pods_per_step, 20_000), seed=seed + 7)
        with engine() as ew:
            ew.stage(wp)
            ew.schedule_staged(0, len(wp))

    e = engine()
    e.stage(pods)
    d.barrier()
    t0 = time.perf_counter()
    rounds = 0
    for k in range(args.steps):
        st = e.schedule_staged(k * args.pods_per_step, args.pods_per_step)
        rounds += int(st["device_batches"])
        if d.rank == 0:
            print(f"[bench] step {k + 1}/{args.steps} done", file=sys.stderr, flush=True)
    t1 = time.perf_counter()
    d.barrier()
    elapsed = d.max(t1 - t0)
    node_idx, score = e.fetch(0, total)
    placed = int((node_idx >= 0).sum())

    # per-kernel live timing (HIP events on the engine stream) for the roofline
    names = (("rsv_eval", "rsv_select") if c5r else
             ("eval_round", "merge_round", "resolve_round") + (("ds_max_round", "ds_norm_reduce") if c5 else ()))
    kernels = {name: e.bench_kernel(which, args.kernel_iters) for which, name in enumerate(names)}
    # roofline kernel: the wide pass, the only kernel whose work scales with node evaluations (SURVEY §8d's
    # 76 B per evaluation); merge and the single-wave FIFO resolver are latency-bound per round
    # (C5: ds_max_round is the DeviceShare profile's full evaluation; eval_round_ds only normalizes its output)
    # (C5 Reservation: rsv_eval is the per-pod wide pass; rsv_select re-reads 8 B per node, rsv_apply is one lane)
    dom = "ds_max_round" if c5 else ("rsv_eval" if c5r else "eval_round")
    dom_ms, dom_bytes = kernels[dom]
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9

    # PCIe-inclusive path (host pods in, host decisions out) on a fresh engine, one step
    pcie = None
    if d.world == 1:
        with engine() as ep:
            tt = time.perf_counter()
            ep.schedule(pods[: args.pods_per_step])
            pcie = args.pods_per_step / (time.perf_counter() - tt)

    check = None
    if args.check and d.rank == 0:
        from oracle import oracle
        if c5r:
            st = oracle.states(cluster.n)
            oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
            on, _, _ = oracle.schedule_resv(cfg, cluster.nodes, cluster.metrics, st, rsv.copy(), pods[: args.check],
                                            cluster.now_ns)
        elif c5:
            st = oracle.states(cluster.n)
            oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
            on, _, _, _ = oracle.schedule_full(cfg, cluster.nodes, cluster.metrics, st, pods[: args.check],
                                               cluster.now_ns, args.cpu_threads, devices=devices.copy())
        elif c4:
            st = oracle.states(cluster.n)
            oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
            on, _ = oracle.schedule_numa(cfg, cluster.nodes, cluster.metrics, st, oracle.numa_states(numa),
                                         pods[: args.check], cluster.now_ns, args.cpu_threads)
        else:
            on, _, _ = oracle.schedule_cluster(cfg, cluster, pods[: args.check], n_threads=args.cpu_threads)
        check = bool(np.array_equal(on, node_idx[: args.check]))

    cpu = None
    if d.rank == 0 and d.world == 1 and not args.no_cpu_baseline:
        print("[bench] cpu baseline sample", file=sys.stderr, flush=True)
        m, dt = cpu_baseline(cfg, cluster, pods, args.cpu_seconds, args.cpu_threads, numa, devices, rsv)
        threads = 1 if c5r else args.cpu_threads
        cpu = {"value": m / dt, "unit": "pods/s", "cores": threads, "kind": "port",
               "sample": f"first {m} pods of the same queue after a 64-pod probe, {cluster.n} nodes, "
                         f"oracle/{'reservation.c or_schedule_resv' if c5r else 'oracle.c ' + ('or_schedule_numa' if c4 else ('or_schedule_full' if c5 else 'or_schedule'))}, "
                         f"{threads} thread(s) "
                         f"{'(single-threaded loop)' if c5r else '(Parallelizer chunking)'}, "
                         f"host nproc={os.cpu_count()}",
               "node_evals_per_sec": m * cluster.n / dt}

    traffic, traffic_src = (pmc_traffic(args.traffic_file, dom, cluster.n, args.batch, args.pods_per_wave)
                            if d.world == 1 and not (c4 or c5) else (None, None))
    if d.rank == 0:
        pods_s = total / elapsed
        out = {
            "metric": ("pods scheduled/sec, NodeNUMAResource cpuset/NUMA profile (node-evals/sec alongside)" if c4
                       else ("pods scheduled/sec, Reservation profile (node-evals/sec alongside)" if c5r else
                             "pods scheduled/sec, DeviceShare GPU-share profile (node-evals/sec alongside)" if c5
                             else "pods scheduled/sec at 100k nodes (node-evals/sec alongside)")),
            "value": pods_s,
            "unit": "pods/s",
            "n_gpus": d.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic (SURVEY §8d generator, seed %d)" % seed,
            "config": {"workload": ("C4 cluster: %d 2-socket 256-cpu nodes, %d-pod FIFO queue (70%% cpuset LSR/LSE), "
                                    "NodeResourcesFit+LoadAwareScheduling+NodeNUMAResource, %d pods per step" if c4 else
                                    ("C5 (Reservation part): %d nodes (30%% with 1-4 reservations), %d-pod FIFO queue "
                                     "(20%% reservation-owned), NodeResourcesFit+LoadAwareScheduling+Reservation (w 5000), "
                                     "one pod per device pass, %d pods per step" if c5r else
                                     "C5 (DeviceShare part): %d nodes x 8 GPUs, %d-pod FIFO queue (30%% GPU-share), "
                                     "NodeResourcesFit+LoadAwareScheduling+DeviceShare, %d pods per step" if c5 else
                                     "C3 cluster: %d nodes, %d-pod FIFO queue, NodeResourcesFit+LoadAwareScheduling, "
                                     "%d pods per step")) % (cluster.n, total, args.pods_per_step),
                       "nodes": cluster.n, "pods": total, "batch_pods": 1 if c5r else args.batch,
                       "parallelism": "node-sharded x%d (replicated table, RCCL all-gather)" % d.world},
            "node_evals_per_sec": pods_s * cluster.n,
            "placed": placed,
            "device_rounds": rounds,
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_source": traffic_src,
                         "kernels_ms": {k: v[0] for k, v in kernels.items()},
                         "algo_bytes": {k: v[1] for k, v in kernels.items()}},
            "cpu_baseline": cpu,
            "pcie_inclusive_pods_per_sec": pcie,
            "oracle_check": check,
        }
        print(json.dumps(out), flush=True)
    e.close()
    d.close()


if __name__ == "__main__":
    main()
