"""Multi-rank engine on one GPU: G engines in one process, each rank evaluating its node shard,
exchanging per-round candidate records through the kg_loopback test hook (device copies ordered by HIP events —
RCCL runs one rank per device, so this is how the multi-rank code runs on a one-GPU box), merging the G rank
records with merge_round<true> and replaying the same FIFO resolver on its replicated table.

Bar: every rank's placements, totals and node state bit-exact with the single-process oracle — the exact
multi-rank path the driver's 2/4/8-GPU run takes, minus the transport."""
import threading

import numpy as np
import pytest

from koordinator_amd import abi, framework as F, synth
from koordinator_amd.engine import Engine, Loopback
from oracle import oracle

pytestmark = pytest.mark.gpu

NUMA_PROFILE = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.NODE_NUMA_RESOURCE),
                         score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.NODE_NUMA_RESOURCE: 1})
DS_PROFILE = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.DEVICE_SHARE),
                       score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.DEVICE_SHARE: 1})


def run_ranks(cfg, n_ranks, capacity, load, pods, chunks=1, fetch=None):
    """Schedules `pods` on n_ranks loopback engines, one host thread per rank; returns each rank's
    (node, score, state[, extra])."""
    out, errors = [None] * n_ranks, []
    with Loopback(n_ranks) as lb:
        engines = [Engine(cfg, capacity, rank=r, n_ranks=n_ranks, loopback=lb) for r in range(n_ranks)]
        try:
            for e in engines:
                load(e)
                e.stage(pods)
            bounds = np.linspace(0, len(pods), chunks + 1).astype(int)

            def work(r):
                try:
                    for a, b in zip(bounds[:-1], bounds[1:]):
                        engines[r].schedule_staged(int(a), int(b - a))
                    node, score = engines[r].fetch(0, len(pods))
                    out[r] = (node, score, engines[r].read_state(), fetch(engines[r]) if fetch else None)
                except Exception as ex:  # surfaced below
                    errors.append((r, ex))

            threads = [threading.Thread(target=work, args=(r,)) for r in range(n_ranks)]
            for t in threads:
                t.start()
            for t in threads:
                t.join(timeout=150)
            assert not any(t.is_alive() for t in threads), "a rank did not finish"
            assert not errors, errors
        finally:
            for e in engines:
                e.close()
    return out


def same_on_every_rank(out, want_node, want_score, st):
    for r, (node, score, state, _) in enumerate(out):
        bad = np.nonzero(node != want_node)[0]
        assert bad.size == 0, f"rank {r}: first mismatch at pod {bad[0]}: {node[bad[0]]} vs oracle {want_node[bad[0]]}"
        assert np.array_equal(score, want_score), r
        assert np.array_equal(state["requested_cpu"], st["requested"][:, abi.RES_CPU]), r
        assert np.array_equal(state["num_pods"], st["num_pods"]), r


@pytest.mark.parametrize("n_ranks,depth,batch", [(2, 1, 32), (2, 2, 32), (3, 2, 16), (4, 0, 32), (2, 2, 38)])
def test_fit_loadaware_ranks(n_ranks, depth, batch):
    cluster = synth.make_cluster(3000, seed=901 + n_ranks)
    pods = synth.make_pods(6000, seed=902 + depth)
    cfg = F.build_config(multi_rank="shard", batch_pods=batch, pods_per_wave=8, pipeline_depth=depth)
    st = oracle.states(cluster.n)
    oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
    want, want_score = oracle.schedule(cfg, cluster.nodes, cluster.metrics, st, pods, cluster.now_ns, 8)
    out = run_ranks(cfg, n_ranks, cluster.n, lambda e: synth.load_into(e, cluster), pods, chunks=2)
    same_on_every_rank(out, want, want_score, st)
    assert (want >= 0).mean() > 0.5


def test_fit_loadaware_ranks_with_quotas_and_ragged_shards():
    """1000 nodes over 3 ranks (shards 334/334/332, a partial last tile) and ElasticQuota admission replicated."""
    cluster = synth.make_cluster(1000, seed=911)
    pods = synth.make_pods(3000, seed=912)
    rng = np.random.default_rng(913)
    pods["quota_id"] = np.where(rng.random(len(pods)) < 0.8, rng.integers(1, 5, len(pods)), 0)
    quotas = np.zeros(4, dtype=abi.QUOTA_DTYPE)
    quotas["used_limit"] = -1
    quotas["min"] = -1
    quotas["used_limit"][:, 0] = pods["requests"][:, 0].sum() // 8
    cfg = F.build_config(multi_rank="shard")
    st = oracle.states(cluster.n)
    oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
    q = quotas.copy()
    want, want_score, _, _ = oracle.schedule_full(cfg, cluster.nodes, cluster.metrics, st, pods, cluster.now_ns, 8,
                                                  quotas=q)

    def load(e):
        synth.load_into(e, cluster)
        e.set_quotas(quotas)

    out = run_ranks(cfg, 3, cluster.n, load, pods, fetch=lambda e: e.read_quotas(len(quotas)))
    same_on_every_rank(out, want, want_score, st)
    for r in range(3):
        assert np.array_equal(out[r][3], q), r
    assert (want < 0).any()


def test_numa_ranks():
    cfg = F.build_config(multi_rank="shard", profile=NUMA_PROFILE, batch_pods=16, pods_per_wave=1)
    cluster, numa = synth.make_numa_cluster(600, seed=921)
    pods = synth.make_numa_pods(1500, seed=922)
    st = oracle.states(cluster.n)
    oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
    buf = oracle.numa_states(numa)
    want, want_score, want_cpus = oracle.schedule_numa(cfg, cluster.nodes, cluster.metrics, st, buf, pods,
                                                       cluster.now_ns, n_threads=8, with_cpusets=True)
    out = run_ranks(cfg, 2, cluster.n, lambda e: synth.load_numa_into(e, cluster, numa), pods,
                    fetch=lambda e: e.fetch_cpusets(0, len(pods)))
    same_on_every_rank(out, want, want_score, st)
    for r in range(2):
        assert np.array_equal(out[r][3], want_cpus), r


def test_deviceshare_ranks():
    cfg = F.build_config(multi_rank="shard", profile=DS_PROFILE, batch_pods=32, pods_per_wave=4)
    cluster, dev = synth.make_gpu_cluster(1500, seed=931)
    pods = synth.make_gpu_pods(3000, seed=932)
    st = oracle.states(cluster.n)
    oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
    d = dev.copy()
    want, want_score, _, want_minors = oracle.schedule_full(cfg, cluster.nodes, cluster.metrics, st, pods,
                                                            cluster.now_ns, 8, devices=d)
    out = run_ranks(cfg, 2, cluster.n, lambda e: synth.load_gpu_into(e, cluster, dev), pods, chunks=2,
                    fetch=lambda e: (e.fetch_devices(0, len(pods)), e.read_devices()))
    same_on_every_rank(out, want, want_score, st)
    for r in range(2):
        minors, (uc, um, ur) = out[r][3]
        assert np.array_equal(minors, want_minors), r
        assert np.array_equal(uc, d["used_core"]) and np.array_equal(ur, d["used_ratio"]), r


C5_PROFILE = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.RESERVATION, F.DEVICE_SHARE),
                       score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.RESERVATION: 5000, F.DEVICE_SHARE: 1})


@pytest.mark.parametrize("n_ranks,n_nodes", [(2, 2000), (3, 2000), (3, 500)])
def test_reservation_profile_ranks_sharded(n_ranks, n_nodes):
    """C5 as one profile (Reservation + DeviceShare + ElasticQuota) on several ranks: (r5) the batched exact rounds
    sharded by tile range — each rank evaluates its tiles, the per-pod statistics and merged records are exchanged
    every round, and the other shards' listed candidates are evaluated on the rank's replica — so
    every rank's placements, reservation slots, GPU minors and quota charges equal the oracle's.  500 nodes = 2 tiles
    over 3 ranks: the last rank's shard is empty."""
    cfg = F.build_config(multi_rank="shard", profile=C5_PROFILE)
    cluster, dev, rsv = synth.make_c5_cluster(n_nodes, seed=961)
    pods = synth.make_c5_pods(1500, seed=962)
    quotas = synth.make_c5_quotas(pods, seed=963)
    st = oracle.states(cluster.n)
    oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
    r, d, q = rsv.copy(), dev.copy(), quotas.copy()
    want, want_score, want_slot, want_minors = oracle.schedule_resv(cfg, cluster.nodes, cluster.metrics, st, r, pods,
                                                                    cluster.now_ns, devices=d, quotas=q, n_threads=8,
                                                                    with_minors=True)
    out = run_ranks(cfg, n_ranks, cluster.n, lambda e: synth.load_c5_into(e, cluster, dev, rsv, quotas), pods,
                    chunks=2, fetch=lambda e: (e.fetch_reservations(0, len(pods)), e.fetch_devices(0, len(pods)),
                                               e.read_quotas(len(quotas))))
    same_on_every_rank(out, want, want_score, st)
    for rk in range(n_ranks):
        slot, minors, qq = out[rk][3]
        assert np.array_equal(slot, want_slot), rk
        assert np.array_equal(minors, want_minors), rk
        assert np.array_equal(qq, q), rk


SHIPPED_PROFILE = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.NODE_NUMA_RESOURCE, F.DEVICE_SHARE,
                                    F.RESERVATION),
                            score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.NODE_NUMA_RESOURCE: 1,
                                   F.DEVICE_SHARE: 1, F.RESERVATION: 5000})


def test_shipped_profile_ranks_sharded():
    """The shipped profile (NUMA + DeviceShare + Reservation + ElasticQuota) on 4 ranks of sharded exact rounds: the
    NUMA affinity of another shard's candidate comes from xr_fill on the rank's replica."""
    cfg = F.build_config(multi_rank="shard", profile=SHIPPED_PROFILE,
                         la=F.LoadAwareSchedulingArgs(filter_expired_node_metrics=False,
                                                      node_metric_expiration_seconds=300))
    cluster, numa, dev, rsv = synth.make_shipped_cluster(1100, seed=1971)
    pods = synth.make_shipped_pods(700, seed=1972)
    quotas = synth.make_c5_quotas(pods, seed=1973)
    st = oracle.states(cluster.n)
    oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
    want, want_score, want_slot = oracle.schedule_resv(cfg, cluster.nodes, cluster.metrics, st, rsv.copy(), pods,
                                                       cluster.now_ns, devices=dev.copy(), quotas=quotas.copy(),
                                                       n_threads=8, numa_buf=oracle.numa_states(numa))
    out = run_ranks(cfg, 4, cluster.n, lambda e: synth.load_shipped_into(e, cluster, numa, dev, rsv, quotas), pods,
                    chunks=2, fetch=lambda e: e.fetch_reservations(0, len(pods)))
    same_on_every_rank(out, want, want_score, st)
    for rk in range(4):
        assert np.array_equal(out[rk][3], want_slot), rk
    assert (want >= 0).mean() > 0.3


def test_auto_multi_rank_runs_small_tables_as_replicas():
    """(r6) kg_config.multi_rank_mode AUTO: below the sharding threshold an engine of a 2-rank group is a
    replica of one GPU — it shards nothing, never calls the exchange, and places exactly as one GPU does; SHARD forces
    the exchange at the same size."""
    from koordinator_amd.engine import HostExchange
    cluster = synth.make_cluster(3000, seed=991)
    pods = synth.make_pods(1500, seed=992)
    calls = [0]

    def allgather(buf):
        calls[0] += 1
        return np.concatenate([buf, buf])

    one = F.build_config(batch_pods=32)
    with Engine(one, cluster.n) as e:
        synth.load_into(e, cluster)
        want = e.schedule(pods)[:2]
    ex = HostExchange(allgather)
    with Engine(F.build_config(batch_pods=32, multi_rank="auto"), cluster.n, rank=1, n_ranks=2, exchange=ex) as e:
        assert e.ranks == (1, 2)
        synth.load_into(e, cluster)
        got = e.schedule(pods)[:2]
    assert calls[0] == 0 and ex.error is None
    np.testing.assert_array_equal(got[0], want[0])
    np.testing.assert_array_equal(got[1], want[1])
    with Engine(F.build_config(batch_pods=32, multi_rank="shard"), cluster.n, rank=0, n_ranks=2,
                exchange=HostExchange(allgather)) as e:
        assert e.ranks == (2, 1)
