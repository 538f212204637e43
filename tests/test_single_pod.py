"""The drop-in's per-pod call: koord-scheduler's scheduleOne schedules ONE pod per SchedulePod call
(frameworkext/framework_extender_factory.go:156-185).  The engine serves calls of at most two pods with its exact
per-pod pass (one coalesced pass over the nodes + a normalize / argmax pass + Reserve, one hipGraph launch) instead of
the round machinery, for every profile.  These tests schedule whole queues one call per pod and compare with the
oracle's sequential loop: placements, totals and node state bit-exact — Fit + LoadAware (with ephemeral-storage /
scalar requests and ElasticQuota), NodeNUMAResource and DeviceShare profiles; plus the exact pass with
ephemeral-storage / scalar requests in a Reservation profile."""
import numpy as np
import pytest

import test_fit_aux as TA
from koordinator_amd import Engine, abi, framework as F, synth
from oracle import oracle

pytestmark = pytest.mark.gpu


def _one_by_one(e, pods, step=1):
    e.stage(pods)
    for j in range(0, len(pods), step):
        e.schedule_staged(j, min(step, len(pods) - j))
    return e.fetch(0, len(pods))


@pytest.mark.parametrize("step", [1, 2])
def test_fit_loadaware_single_pod_calls(step):
    cluster = TA._aux_cluster(1500, seed=901)
    pods = TA._aux_pods(400, seed=902)
    q = np.zeros(4, dtype=abi.QUOTA_DTYPE)
    q["used_limit"] = -1
    q["min"] = -1
    q["used_limit"][:, 0] = [20_000, 60_000, 10**9, 5_000]
    pods["quota_id"] = np.arange(len(pods)) % 5
    cfg = F.build_config()
    st = oracle.states(cluster.n)
    oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
    qo = q.copy()
    want, want_score, _, _ = oracle.schedule_full(cfg, cluster.nodes, cluster.metrics, st, pods, cluster.now_ns, 8,
                                                  quotas=qo)
    with Engine(cfg, cluster.n) as e:
        synth.load_into(e, cluster)
        e.set_quotas(q)
        node, score = _one_by_one(e, pods, step)
        state = e.read_state()
        used = e.read_quotas(len(q))["used"]
    assert np.array_equal(node, want) and np.array_equal(score, want_score)
    assert np.array_equal(state["requested_cpu"], st["requested"][:, abi.RES_CPU])
    assert np.array_equal(state["la_est_cpu"], st["la_est_all"][:, 0])
    assert np.array_equal(used, qo["used"])


def test_numa_single_pod_calls():
    cfg = F.build_config(profile=F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.NODE_NUMA_RESOURCE),
                                           score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.NODE_NUMA_RESOURCE: 1}))
    cluster, numa = synth.make_numa_cluster(600, seed=911)
    pods = synth.make_numa_pods(300, seed=912)
    st = oracle.states(cluster.n)
    oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
    buf = oracle.numa_states(numa)
    want, want_score, want_cpus, _ = oracle.schedule_full(cfg, cluster.nodes, cluster.metrics, st, pods, cluster.now_ns,
                                                          8, numa_buf=buf)
    with Engine(cfg, cluster.n) as e:
        synth.load_numa_into(e, cluster, numa)
        node, score = _one_by_one(e, pods)
        cpus = e.fetch_cpusets(0, len(pods))
        ga, gc, gm = e.read_numa()
    assert np.array_equal(node, want) and np.array_equal(score, want_score)
    assert np.array_equal(cpus, want_cpus)
    wa, wc, wm = oracle.numa_state_read(buf, cluster.n)
    assert np.array_equal(ga, wa) and np.array_equal(gc, wc) and np.array_equal(gm, wm)


def test_deviceshare_single_pod_calls():
    cfg = F.build_config(profile=F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.DEVICE_SHARE),
                                           score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.DEVICE_SHARE: 1}))
    cluster, dev = synth.make_gpu_cluster(800, seed=921)
    pods = synth.make_gpu_pods(400, seed=922)
    st = oracle.states(cluster.n)
    oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
    d = dev.copy()
    want, want_score, _, want_minors = oracle.schedule_full(cfg, cluster.nodes, cluster.metrics, st, pods,
                                                            cluster.now_ns, 8, devices=d)
    with Engine(cfg, cluster.n) as e:
        synth.load_gpu_into(e, cluster, dev)
        node, score = _one_by_one(e, pods)
        minors = e.fetch_devices(0, len(pods))
        used = e.read_devices()
    assert np.array_equal(node, want) and np.array_equal(score, want_score)
    assert np.array_equal(minors, want_minors) and np.array_equal(used[2], d["used_ratio"])


def test_reservation_profile_with_scalar_requests():
    """Ephemeral-storage / batch / mid requests in a Reservation profile: NodeResourcesFit's Allocatable - Requested
    compare on the exact pass, Requested moved by Reserve and Unreserve."""
    prof = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.RESERVATION),
                     score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.RESERVATION: 5000})
    cfg = F.build_config(profile=prof)
    cluster = TA._aux_cluster(700, seed=931)
    cluster, rsv = synth.make_rsv_cluster(700, seed=932, cluster=cluster)
    pods = synth.make_rsv_pods(900, seed=933, base=TA._aux_pods(900, seed=934))
    st = oracle.states(cluster.n)
    oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
    r = rsv.copy()
    want, want_score, want_slot = oracle.schedule_resv(cfg, cluster.nodes, cluster.metrics, st, r, pods,
                                                       cluster.now_ns, n_threads=8)
    with Engine(cfg, cluster.n) as e:
        synth.load_rsv_into(e, cluster, rsv)
        e.stage(pods)
        e.schedule_staged(0, len(pods))
        node, score = e.fetch(0, len(pods))
        slot = e.fetch_reservations(0, len(pods))
    assert np.array_equal(node, want) and np.array_equal(score, want_score) and np.array_equal(slot, want_slot)
    aux = pods["requests"][:, abi.RES_EPHEMERAL:abi.RES_MID_MEMORY + 1].any(axis=1)
    assert (aux & (node >= 0)).sum() > 20 and (aux & (node < 0)).any()
