"""The multi-rank ENGINE across processes: a world_size-2 torch.distributed gloo group, one process per
rank, each with its own engine on cuda:0 (the one-GPU box has one device; RCCL refuses two ranks on one device).
The engines are created with kg_engine_create_hosted, so every per-round exchange of the rank records — and
DeviceShare's per-pod (max, holders) — goes through gloo's all_gather on the host instead of RCCL; every other step
is the engine's own multi-rank path: the sharded wide pass, merge_round<true> over the gathered records, the
replicated FIFO resolver.

Bar: both ranks' placements, totals and node state bit-exact with the single-process oracle."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from koordinator_amd import framework as F, synth
from oracle import oracle

pytestmark = pytest.mark.gpu

DS_PROFILE = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.DEVICE_SHARE),
                       score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.DEVICE_SHARE: 1})


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


RSV_PROFILE = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.RESERVATION),
                        score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.RESERVATION: 5000})
SHIPPED_PROFILE = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.NODE_NUMA_RESOURCE, F.DEVICE_SHARE,
                                    F.RESERVATION),
                            score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.NODE_NUMA_RESOURCE: 1,
                                   F.DEVICE_SHARE: 1, F.RESERVATION: 5000})


STOCK_PROFILE = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.TAINT_TOLERATION, F.NODE_AFFINITY,
                                  F.POD_TOPOLOGY_SPREAD, F.INTER_POD_AFFINITY),
                          score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.TAINT_TOLERATION: 1, F.NODE_AFFINITY: 1,
                                 F.BALANCED_ALLOCATION: 1, F.POD_TOPOLOGY_SPREAD: 2, F.INTER_POD_AFFINITY: 1})


def _exact_case(kind):
    """(r4) the exact profiles, which run as replicas on every rank: Reservation, the shipped profile
    (NUMA + DeviceShare + Reservation + ElasticQuota), and the upstream defaults with hostname / zone
    PodTopologySpread and InterPodAffinity (the per-pod pass)."""
    if kind == "stock":
        cfg = F.build_config(multi_rank="shard", profile=STOCK_PROFILE)
        cluster = synth.make_cluster(800, seed=981)
        synth.make_pod_groups(cluster.existing_pods, seed=984, zones=True)
        pods = synth.make_pod_groups(synth.make_pods(300, seed=982), seed=985, zones=True)
        preds = synth.make_predicates(800, pods, seed=983, no_zone=0.05)[1]
        return cfg, dict(cluster=cluster, pods=pods, preds=preds)
    if kind == "rsv":
        cfg = F.build_config(multi_rank="shard", profile=RSV_PROFILE)
        cluster, rsv = synth.make_rsv_cluster(1500, seed=961)
        return cfg, dict(cluster=cluster, rsv=rsv, pods=synth.make_rsv_pods(800, seed=962))
    cfg = F.build_config(multi_rank="shard", profile=SHIPPED_PROFILE,
                         la=F.LoadAwareSchedulingArgs(filter_expired_node_metrics=False,
                                                      node_metric_expiration_seconds=300))
    cluster, numa, dev, rsv = synth.make_shipped_cluster(600, seed=971)
    pods = synth.make_shipped_pods(500, seed=972)
    return cfg, dict(cluster=cluster, numa=numa, dev=dev, rsv=rsv, pods=pods,
                     quotas=synth.make_c5_quotas(pods, seed=973))


def _case(kind):
    if kind == "ds":
        cfg = F.build_config(multi_rank="shard", profile=DS_PROFILE, batch_pods=32, pods_per_wave=4)
        cluster, dev = synth.make_gpu_cluster(1200, seed=951)
        pods = synth.make_gpu_pods(1500, seed=952)
        return cfg, cluster, pods, dev
    cfg = F.build_config(multi_rank="shard", batch_pods=32, pods_per_wave=8, pipeline_depth=2)
    cluster = synth.make_cluster(2000, seed=941)
    pods = synth.make_pods(3000, seed=942)
    return cfg, cluster, pods, None


def _rank_main(rank, world, port, kind, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from koordinator_amd.engine import Engine, HostExchange

        calls = [0]

        def allgather(buf):
            t = torch.from_numpy(buf)
            parts = [torch.empty_like(t) for _ in range(world)]
            dist.all_gather(parts, t)
            calls[0] += 1
            return torch.cat(parts).numpy()

        ex = HostExchange(allgather)
        if kind in ("rsv", "shipped", "stock"):
            cfg, w = _exact_case(kind)
            cluster, pods = w["cluster"], w["pods"]
            with Engine(cfg, cluster.n, rank=rank, n_ranks=world, exchange=ex) as e:
                if kind == "rsv":
                    synth.load_rsv_into(e, cluster, w["rsv"])
                elif kind == "stock":
                    synth.load_into(e, cluster)
                    e.upsert_predicates(w["preds"])
                else:
                    synth.load_shipped_into(e, cluster, w["numa"], w["dev"], w["rsv"], w["quotas"])
                e.stage(pods)
                half = len(pods) // 2
                e.schedule_staged(0, half)
                e.schedule_staged(half, len(pods) - half)
                node, score = e.fetch(0, len(pods))
                np.save(os.path.join(out_dir, f"node{rank}.npy"), node)
                np.save(os.path.join(out_dir, f"score{rank}.npy"), score)
                np.save(os.path.join(out_dir, f"slot{rank}.npy"), e.fetch_reservations(0, len(pods)))
                np.save(os.path.join(out_dir, f"cpu{rank}.npy"), e.read_state()["requested_cpu"])
                np.save(os.path.join(out_dir, f"calls{rank}.npy"), np.array([calls[0]]))
            assert ex.error is None, ex.error
            return
        cfg, cluster, pods, dev = _case(kind)
        with Engine(cfg, cluster.n, rank=rank, n_ranks=world, exchange=ex) as e:
            if dev is not None:
                synth.load_gpu_into(e, cluster, dev)
            else:
                synth.load_into(e, cluster)
            e.stage(pods)
            half = len(pods) // 2
            e.schedule_staged(0, half)
            e.schedule_staged(half, len(pods) - half)
            node, score = e.fetch(0, len(pods))
            state = e.read_state()
            np.save(os.path.join(out_dir, f"node{rank}.npy"), node)
            np.save(os.path.join(out_dir, f"score{rank}.npy"), score)
            np.save(os.path.join(out_dir, f"cpu{rank}.npy"), state["requested_cpu"])
            np.save(os.path.join(out_dir, f"calls{rank}.npy"), np.array([calls[0]]))
            if dev is not None:
                np.save(os.path.join(out_dir, f"minors{rank}.npy"), e.fetch_devices(0, len(pods)))
        assert ex.error is None, ex.error
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["fit_loadaware", "ds"])
def test_two_process_gloo_engine(tmp_path, kind):
    world = 2
    mp.spawn(_rank_main, args=(world, _free_port(), kind, str(tmp_path)), nprocs=world, join=True)
    cfg, cluster, pods, dev = _case(kind)
    st = oracle.states(cluster.n)
    oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
    if dev is None:
        want, want_score = oracle.schedule(cfg, cluster.nodes, cluster.metrics, st, pods, cluster.now_ns, 8)
        want_minors = None
    else:
        want, want_score, _, want_minors = oracle.schedule_full(cfg, cluster.nodes, cluster.metrics, st, pods,
                                                                cluster.now_ns, 8, devices=dev.copy())
    for r in range(world):
        node = np.load(tmp_path / f"node{r}.npy")
        bad = np.nonzero(node != want)[0]
        assert bad.size == 0, f"rank {r}: first mismatch at pod {bad[0]}: {node[bad[0]]} vs oracle {want[bad[0]]}"
        np.testing.assert_array_equal(np.load(tmp_path / f"score{r}.npy"), want_score)
        np.testing.assert_array_equal(np.load(tmp_path / f"cpu{r}.npy"), st["requested"][:, 0])
        assert int(np.load(tmp_path / f"calls{r}.npy")[0]) > 0  # the rounds really exchanged through gloo
        if want_minors is not None:
            np.testing.assert_array_equal(np.load(tmp_path / f"minors{r}.npy"), want_minors)
    assert (want >= 0).mean() > 0.3


@pytest.mark.parametrize("kind", ["rsv", "shipped", "stock"])
def test_two_process_gloo_exact_profiles(tmp_path, kind):
    """The exact profiles on two ranks.  Reservation and the shipped profile run the batched exact rounds
    sharded by node range: each rank evaluates its half of the tiles, the per-pod statistics and merged records go
    through the exchange every round, and the other half's candidates are evaluated on the rank's replica (xr_fill).
    The stock profile (PodTopologySpread / InterPodAffinity: the per-pod pass) stays a replica on every rank.  Both
    ranks' placements, totals, reservation slots and node state equal the oracle's."""
    world = 2
    mp.spawn(_rank_main, args=(world, _free_port(), kind, str(tmp_path)), nprocs=world, join=True)
    cfg, w = _exact_case(kind)
    cluster, pods = w["cluster"], w["pods"]
    st = oracle.states(cluster.n)
    oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
    if kind == "stock":
        g = oracle.groups_init(cluster.n, cluster.existing_pods, cluster.existing_node)
        want, want_score, want_slot = oracle.schedule_resv(cfg, cluster.nodes, cluster.metrics, st, None, pods,
                                                           cluster.now_ns, n_threads=8, preds=w["preds"], groups=g)
    elif kind == "rsv":
        want, want_score, want_slot = oracle.schedule_resv(cfg, cluster.nodes, cluster.metrics, st, w["rsv"].copy(),
                                                           pods, cluster.now_ns, n_threads=8)
    else:
        want, want_score, want_slot = oracle.schedule_resv(cfg, cluster.nodes, cluster.metrics, st, w["rsv"].copy(),
                                                           pods, cluster.now_ns, devices=w["dev"].copy(),
                                                           quotas=w["quotas"].copy(), n_threads=8,
                                                           numa_buf=oracle.numa_states(w["numa"]))
    for r in range(world):
        node = np.load(tmp_path / f"node{r}.npy")
        bad = np.nonzero(node != want)[0]
        assert bad.size == 0, f"rank {r}: first mismatch at pod {bad[0]}: {node[bad[0]]} vs oracle {want[bad[0]]}"
        np.testing.assert_array_equal(np.load(tmp_path / f"score{r}.npy"), want_score)
        np.testing.assert_array_equal(np.load(tmp_path / f"slot{r}.npy"), want_slot)
        np.testing.assert_array_equal(np.load(tmp_path / f"cpu{r}.npy"), st["requested"][:, 0])
        calls = int(np.load(tmp_path / f"calls{r}.npy")[0])
        if kind == "stock":
            assert calls == 0  # replicas: nothing to exchange
        else:
            assert calls >= 2 * 10, calls  # two exchanges per exact round, ≥ 10 rounds for these queues
    assert (want >= 0).mean() > 0.3
