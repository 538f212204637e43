"""ElasticQuota admission: the oracle against the reference's PreFilter test tables
(tests/golden/elasticquota.json, tests/golden/make_golden_quota.py), and — on the GPU — the engine's in-resolver
admission against the oracle: each pod's PreFilter sees the quota charged by every earlier placement of the batch."""
import json
import os

import numpy as np
import pytest

from koordinator_amd import Engine, abi, framework, synth
from oracle import oracle

F = framework
HERE = os.path.dirname(os.path.abspath(__file__))


def _cases():
    with open(os.path.join(HERE, "golden", "elasticquota.json")) as f:
        return json.load(f)["cases"]


def _quota(c):
    q = c["quota"]
    return F.make_quota(used_limit=q.get("used_limit"), used=q.get("used"), min=q.get("min"),
                        non_preemptible_used=q.get("non_preemptible_used"))


def _pod(c):
    return F.make_pod({"cpu": f"{c['pod']['cpu']}m", "memory": str(c["pod"]["memory"])}, quota_id=1,
                      non_preemptible=c["non_preemptible"])


def _one_node_schedule_oracle(cfg, quotas, pods):
    node = F.make_node({"cpu": "1000", "memory": str(1 << 50)}, allowed_pods=100000)
    metrics = np.zeros(1, dtype=abi.METRIC_DTYPE)
    st = oracle.states(1)
    q = quotas.copy()
    out, _, _, _ = oracle.schedule_full(cfg, node, metrics, st, pods, 0, quotas=q)
    return out, q


@pytest.mark.parametrize("c", _cases(), ids=lambda c: c["name"])
def test_golden_prefilter_oracle(c):
    out, _ = _one_node_schedule_oracle(F.build_config(), _quota(c), _pod(c))
    assert ("Success" if out[0] == 0 else "Unschedulable") == c["want"], c["source"]


def _quota_cluster(n_nodes, n_pods, n_quotas, seed):
    cluster = synth.make_cluster(n_nodes, seed=seed)
    pods = synth.make_pods(n_pods, seed=seed + 1)
    rng = np.random.default_rng(seed + 2)
    pods["quota_id"] = np.where(rng.random(n_pods) < 0.8, rng.integers(1, n_quotas + 1, n_pods), 0)
    pods["flags"] |= np.where(rng.random(n_pods) < 0.2, abi.POD_NON_PREEMPTIBLE, 0)
    quotas = np.zeros(n_quotas, dtype=abi.QUOTA_DTYPE)
    # limits that run out during the queue: ~ a share of the queue's demand per quota
    share = pods["requests"][:, :2].sum(axis=0) // n_quotas
    quotas["used_limit"][:, 0] = (share[0] * rng.uniform(0.2, 1.2, n_quotas)).astype(np.int64)
    quotas["used_limit"][:, 1] = (share[1] * rng.uniform(0.2, 1.2, n_quotas)).astype(np.int64)
    quotas["used_limit"][rng.random(n_quotas) < 0.2, 1] = -1  # no memory key in the runtime
    quotas["min"][:, 0] = quotas["used_limit"][:, 0] // 4
    quotas["min"][:, 1] = np.where(quotas["used_limit"][:, 1] >= 0, quotas["used_limit"][:, 1] // 4, -1)
    return cluster, pods, quotas


def test_oracle_quota_bookkeeping():
    cluster, pods, quotas = _quota_cluster(200, 1500, 16, 7)
    cfg = F.build_config()
    st = oracle.states(cluster.n)
    oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
    q = quotas.copy()
    node, _, _, _ = oracle.schedule_full(cfg, cluster.nodes, cluster.metrics, st, pods, cluster.now_ns, quotas=q)
    placed = node >= 0
    for k in range(len(quotas)):
        mine = placed & (pods["quota_id"] == k + 1)
        assert q["used"][k, 0] == pods["requests"][mine, abi.RES_CPU].sum()
        npm = mine & ((pods["flags"] & abi.POD_NON_PREEMPTIBLE) != 0)
        assert q["non_preemptible_used"][k, 1] == pods["requests"][npm, abi.RES_MEMORY].sum()
    assert (~placed & (pods["quota_id"] > 0)).any()  # some quotas ran out


@pytest.mark.gpu
@pytest.mark.parametrize("c", _cases(), ids=lambda c: c["name"])
def test_golden_prefilter_device(c):
    with Engine(F.build_config(), 1) as e:
        e.upsert_nodes(F.make_node({"cpu": "1000", "memory": str(1 << 50)}, allowed_pods=100000))
        e.set_quotas(_quota(c))
        node, _, _ = e.schedule(_pod(c))
    assert ("Success" if node[0] == 0 else "Unschedulable") == c["want"], c["source"]


@pytest.mark.gpu
@pytest.mark.parametrize("batch,ppw", [(32, 8), (1, 1), (13, 4), (64, 8)])
def test_schedule_parity_with_quotas(batch, ppw):
    cluster, pods, quotas = _quota_cluster(1500, 4000, 16, 100 + batch)
    cfg = F.build_config(batch_pods=batch, pods_per_wave=ppw)
    st = oracle.states(cluster.n)
    oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
    q = quotas.copy()
    want, want_score, _, _ = oracle.schedule_full(cfg, cluster.nodes, cluster.metrics, st, pods, cluster.now_ns, 8,
                                                  quotas=q)
    with Engine(cfg, cluster.n) as e:
        synth.load_into(e, cluster)
        e.set_quotas(quotas)
        e.stage(pods)
        for s in range(0, len(pods), 1000):
            e.schedule_staged(s, 1000)
        node, score = e.fetch(0, len(pods))
        got_q = e.read_quotas(len(quotas))
    assert np.array_equal(node, want) and np.array_equal(score, want_score)
    assert np.array_equal(got_q, q)


@pytest.mark.gpu
def test_quotas_with_deviceshare_profile():
    cluster, dev = synth.make_gpu_cluster(400, seed=5)
    pods = synth.make_gpu_pods(1500, seed=6)
    rng = np.random.default_rng(9)
    pods["quota_id"] = np.where(rng.random(len(pods)) < 0.7, rng.integers(1, 5, len(pods)), 0)
    quotas = np.zeros(4, dtype=abi.QUOTA_DTYPE)
    quotas["used_limit"] = -1
    quotas["min"] = -1
    quotas["used_limit"][:, :2] = [[200_000, 400 << 30], [100_000, -1], [300_000, 200 << 30], [50_000, 100 << 30]]
    core, ratio = 2 + abi.DEV_GPU_CORE, 2 + abi.DEV_GPU_MEMORY_RATIO  # device pods are admitted on their GPU keys too
    quotas["used_limit"][:, core] = [4000, 1500, -1, 800]
    quotas["used_limit"][:, ratio] = [4000, -1, 2500, 800]
    prof = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.DEVICE_SHARE),
                     score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.DEVICE_SHARE: 1})
    cfg = F.build_config(profile=prof)
    st = oracle.states(cluster.n)
    oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
    q, d = quotas.copy(), dev.copy()
    want, _, _, want_minors = oracle.schedule_full(cfg, cluster.nodes, cluster.metrics, st, pods, cluster.now_ns, 8,
                                                   devices=d, quotas=q)
    with Engine(cfg, cluster.n) as e:
        synth.load_gpu_into(e, cluster, dev)
        e.set_quotas(quotas)
        node, _, _ = e.schedule(pods)
        minors = e.fetch_devices(0, len(pods))
        got_q = e.read_quotas(len(quotas))
    assert np.array_equal(node, want) and np.array_equal(minors, want_minors)
    assert np.array_equal(got_q, q)
    assert (want < 0).any() and (minors != 0).any()
