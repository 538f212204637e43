"""GPU parity of NodeNUMAResource (config C4): the HIP engine (through the C ABI) against the oracle restatement
(oracle/numa.c) and the reference's own test tables (tests/golden/numa_*.json).

Bar: bit-exact — Filter verdicts, plugin scores, stored NUMA affinities, placements and total scores, the
cpuset Reserve allocates to every pod (the cpu accumulator's exact choice), and the final NodeAllocation
(allocated cpus, per-NUMA allocated cpu/memory) plus NodeInfo/LoadAware node state."""
import numpy as np
import pytest

import golden_cases as G
import test_golden_numa as TG
from koordinator_amd import Engine, abi, framework, synth
from oracle import oracle

pytestmark = pytest.mark.gpu
F = framework

FULL_PROFILE = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.NODE_NUMA_RESOURCE),
                         score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.NODE_NUMA_RESOURCE: 1})


def _node(cpu_m, mem):
    return F.make_node({"cpu": f"{cpu_m}m", "memory": str(mem)})


def _one_node(cfg, nn, cpu_m, mem, requested=(0, 0)):
    e = Engine(cfg, 1)
    e.upsert_nodes(_node(cpu_m, mem))
    e.upsert_numa(nn)
    if requested[0] or requested[1]:
        e.add_pods(F.make_pod({"cpu": f"{requested[0]}m", "memory": str(requested[1])}), np.zeros(1, np.int32))
    return e


# ---------------------------------------------------------------------------------------------------------
# the reference's test tables through the device path
# ---------------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("dc", TG._cases("numa_filter.json"), ids=TG._id)
def test_golden_filter_device(dc):
    _, c = dc
    cfg, nn, pod = TG.filter_case(c)
    with _one_node(cfg, nn, 96000, 512 << 30) as e:
        ok, _, _ = e.evaluate_numa(pod)
    assert ("Success" if ok[0] else "UnschedulableAndUnresolvable") == c["want"], c["source_line"]


@pytest.mark.parametrize("dc", TG._cases("numa_score.json"), ids=TG._id)
def test_golden_score_device(dc):
    _, c = dc
    cfg, pod = TG.score_case(c)
    got = []
    for nn, req, alloc in TG.score_nodes(c):
        with _one_node(cfg, nn, alloc[0], alloc[1], req) as e:
            ok, sc, _ = e.evaluate_numa(pod)
        assert ok[0], c["source_line"]
        got.append(int(sc[0]))
    assert got == c["want"], c["source_line"]


@pytest.mark.parametrize("dc", TG._cases("numa_affinity.json"), ids=TG._id)
def test_golden_affinity_device(dc):
    doc, c = dc
    cfg, nn, pod = TG.affinity_case(doc, c)
    with _one_node(cfg, nn, 104000, 256 << 30) as e:
        ok, _, mask = e.evaluate_numa(pod)
    assert ok[0], c["source_line"]
    assert [b for b in range(4) if (int(mask[0]) >> b) & 1] == c["want"], c["source_line"]


def _schedule_one(cfg, nn, pod, cpu_m=1 << 20, mem=1 << 40):
    with _one_node(cfg, nn, cpu_m, mem) as e:
        e.stage(pod)
        e.schedule_staged(0, 1)
        node, _ = e.fetch(0, 1)
        cpus = e.fetch_cpusets(0, 1)[0]
    return int(node[0]), F.cpuset_of(cpus)


@pytest.mark.parametrize("dc", TG._cases("numa_take_cpus.json"), ids=TG._id)
def test_golden_take_cpus_device(dc):
    """takeCPUs through Reserve: one node of the case's topology (NUMA policy none, the case's allocate
    strategy as the node label), one LSR pod preferring the case's bind policy."""
    _, c = dc
    cfg = F.build_config(profile=TG.NUMA_PROFILE)
    nn = F.make_node_numa(*c["topo"], numa_allocate_strategy=c["strategy"], allocated_cpus=c["alloc"])
    pod = F.make_pod({"cpu": str(c["need"])}, priority_class="koord-prod", qos="LSR",
                     preferred_cpu_bind_policy=c["policy"])
    node, cpus = _schedule_one(cfg, nn, pod)
    assert node == 0 and cpus == sorted(c["want"]), c["source_line"]


@pytest.mark.parametrize("dc", TG._cases("numa_take_cpus_exclusive.json"), ids=TG._id)
def test_golden_take_cpus_exclusive_device(dc):
    """TestTakeCPUsWithExclusivePolicy through Reserve: the allocated cpus hold alloc_policy on the node
    (kg_node_numa.exclusive_*_cpus), the pod prefers the case's exclusive and bind policies."""
    _, c = dc
    cfg = F.build_config(profile=TG.NUMA_PROFILE)
    ex = {"exclusive_pcpu_cpus": c["alloc"]} if c["alloc_policy"] == "PCPULevel" else {"exclusive_numa_cpus": c["alloc"]}
    nn = F.make_node_numa(*c["topo"], numa_allocate_strategy=c["strategy"], allocated_cpus=c["alloc"], **ex)
    pod = F.make_pod({"cpu": str(c["need"])}, priority_class="koord-prod", qos="LSR",
                     preferred_cpu_bind_policy=c["policy"], preferred_cpu_exclusive_policy=c["excl"])
    node, cpus = _schedule_one(cfg, nn, pod)
    assert node == 0 and cpus == sorted(c["want"]), c["source_line"]


@pytest.mark.parametrize("dc", TG._cases("numa_reserve.json"), ids=TG._id)
def test_golden_reserve_device(dc):
    _, c = dc
    cfg, nn, pod = TG.reserve_case(c)
    node, cpus = _schedule_one(cfg, nn, pod)
    if c["want"] is None:
        assert node == -1, c["source_line"]
    else:
        assert node == 0 and cpus == sorted(c["want"]), c["source_line"]


# ---------------------------------------------------------------------------------------------------------
# synthetic C4 clusters against the oracle
# ---------------------------------------------------------------------------------------------------------
def _c4_engine(cfg, cluster, numa):
    e = Engine(cfg, cluster.n)
    synth.load_numa_into(e, cluster, numa)
    return e


def test_evaluate_numa_matches_oracle():
    cfg = F.build_config(profile=FULL_PROFILE)
    cluster, numa = synth.make_numa_cluster(256, seed=synth.BASE_SEED + 40)
    pods = synth.make_numa_pods(24, seed=synth.BASE_SEED + 41)
    st = oracle.states(cluster.n)
    oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
    alloc = cluster.nodes["allocatable"]
    with _c4_engine(cfg, cluster, numa) as e:
        for k in range(len(pods)):
            ok, sc, af = e.evaluate_numa(pods[k:k + 1])
            for i in range(cluster.n):
                want = oracle.numa_eval(cfg, numa[i:i + 1], pods[k:k + 1],
                                        (st["requested"][i, abi.RES_CPU], st["requested"][i, abi.RES_MEMORY]),
                                        (alloc[i, abi.RES_CPU], alloc[i, abi.RES_MEMORY]))
                assert (bool(ok[i]), int(sc[i]), int(af[i])) == want, (k, i)


def _numa_parity(cfg, cluster, numa, pods):
    st = oracle.states(cluster.n)
    oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
    buf = oracle.numa_states(numa)
    on, os_, oc = oracle.schedule_numa(cfg, cluster.nodes, cluster.metrics, st, buf, pods, cluster.now_ns,
                                       n_threads=8, with_cpusets=True)
    with _c4_engine(cfg, cluster, numa) as e:
        gn, gs, _ = e.schedule(pods)
        mism = np.nonzero(gn != on)[0]
        assert mism.size == 0, f"first mismatch at pod {mism[:5]}: gpu {gn[mism[:5]]} oracle {on[mism[:5]]}"
        np.testing.assert_array_equal(gs, os_)
        np.testing.assert_array_equal(e.fetch_cpusets(0, len(pods)), oc)
        ga, gc, gm = e.read_numa()
        wa, wc, wm = oracle.numa_state_read(buf, cluster.n)
        np.testing.assert_array_equal(ga, wa)
        np.testing.assert_array_equal(gc, wc)
        np.testing.assert_array_equal(gm, wm)
        s = e.read_state()
        np.testing.assert_array_equal(s["requested_cpu"], st["requested"][:, abi.RES_CPU])
        np.testing.assert_array_equal(s["num_pods"], st["num_pods"])
    return on, oc


@pytest.mark.parametrize("batch", [32, 64, 7, 1])
def test_c4_schedule_parity(batch):
    cfg = F.build_config(profile=FULL_PROFILE, batch_pods=batch, pods_per_wave=min(8, batch))
    cluster, numa = synth.make_numa_cluster(600, seed=synth.BASE_SEED + 42)
    pods = synth.make_numa_pods(2500 if batch > 1 else 300, seed=synth.BASE_SEED + 43)
    node, cpus = _numa_parity(cfg, cluster, numa, pods)
    assert (node >= 0).mean() > 0.5
    assert (cpus != 0).any()


@pytest.mark.parametrize("batch,depth", [(16, 2), (16, 3), (8, 4), (15, 3)])
def test_c4_pipelined_parity(batch, depth):
    """(r5) Pipelined NUMA rounds: the resolver re-scores every row the earlier rounds in flight modified (their
    winner lists), so depth 2..4 stays bit-exact although NodeNUMAResource is not monotone."""
    cfg = F.build_config(profile=FULL_PROFILE, batch_pods=batch, pods_per_wave=min(8, batch), pipeline_depth=depth)
    cluster, numa = synth.make_numa_cluster(700, seed=synth.BASE_SEED + 142)
    pods = synth.make_numa_pods(2000, seed=synth.BASE_SEED + 143)
    node, cpus = _numa_parity(cfg, cluster, numa, pods)
    assert (node >= 0).mean() > 0.5
    assert (cpus != 0).any()


def test_c4_full_size_parity():
    """(r5) C4 at its bench size on the device: 10k two-socket 256-cpu nodes, the bench geometry
    (16 pods per round, depth 2), 3,000 queued pods — placements, totals, cpusets, the NodeAllocation state and the
    node table all equal the oracle's (the bench line checks the first 2k placements only)."""
    cfg = F.build_config(profile=FULL_PROFILE, batch_pods=16, pods_per_wave=1, pipeline_depth=2)
    cluster, numa = synth.make_numa_cluster(10_000, seed=synth.BASE_SEED + 242)
    pods = synth.make_numa_pods(3000, seed=synth.BASE_SEED + 243)
    node, cpus = _numa_parity(cfg, cluster, numa, pods)
    assert (node >= 0).mean() > 0.9 and (cpus != 0).any(axis=1).sum() > 1000


@pytest.mark.parametrize("variant", ["score_only", "most_allocated", "numa_only_spread_default"])
def test_c4_profile_variants(variant):
    if variant == "score_only":
        prof = F.Profile(filter=(F.NODE_RESOURCES_FIT,), score={F.NODE_RESOURCES_FIT: 1, F.NODE_NUMA_RESOURCE: 2})
        cfg = F.build_config(profile=prof)
    elif variant == "most_allocated":
        numa_args = F.NodeNUMAResourceArgs(scoring_strategy="MostAllocated", numa_scoring_strategy="MostAllocated")
        cfg = F.build_config(profile=FULL_PROFILE, numa=numa_args)
    else:
        numa_args = F.NodeNUMAResourceArgs(default_cpu_bind_policy="SpreadByPCPUs")
        cfg = F.build_config(profile=TG.NUMA_PROFILE, numa=numa_args)
    cluster, numa = synth.make_numa_cluster(300, seed=synth.BASE_SEED + 44)
    pods = synth.make_numa_pods(1500, seed=synth.BASE_SEED + 45)
    _numa_parity(cfg, cluster, numa, pods)


def test_numa_upsert_requires_profile():
    cfg = F.build_config()
    with Engine(cfg, 4) as e:
        with pytest.raises(abi.KoordGPUError):
            e.upsert_numa(F.make_node_numa(2, 1, 4, 2))


def _with_exclusive(numa, pods, seed):
    """Marks half of every node's allocated cpus as held by PCPULevel / NUMANodeLevel pods and gives 30 % / 20 % of the
    queue those preferred exclusive policies (the rest None)."""
    rng = np.random.default_rng(seed)
    numa = numa.copy()
    for i in range(len(numa)):
        alloc = F.cpuset_of(numa[i]["allocated_cpus"])
        pick = rng.random(len(alloc))
        for name, lo, hi in (("exclusive_pcpu_cpus", 0.0, 0.3), ("exclusive_numa_cpus", 0.3, 0.5)):
            w = np.zeros(abi.MAX_CPUS // 64, dtype=np.uint64)
            for c, u in zip(alloc, pick):
                if lo <= u < hi:
                    w[c // 64] |= np.uint64(1) << np.uint64(c % 64)
            numa[i][name] = w
    pods = pods.copy()
    u = rng.random(len(pods))
    pods["preferred_cpu_exclusive_policy"] = np.where(u < 0.3, 1, np.where(u < 0.5, 2, 0))
    return numa, pods


@pytest.mark.parametrize("batch", [16, 1])
def test_c4_exclusive_policies_parity(batch):
    """C4 with CPU exclusive policies (cpu_accumulator.go:247-330): bit-exact placements, cpusets and NodeAllocation
    against the oracle, the masks carried across Reserve."""
    cfg = F.build_config(profile=FULL_PROFILE, batch_pods=batch, pods_per_wave=min(8, batch))
    cluster, numa = synth.make_numa_cluster(500, seed=synth.BASE_SEED + 46)
    pods = synth.make_numa_pods(2000 if batch > 1 else 300, seed=synth.BASE_SEED + 47)
    numa, pods = _with_exclusive(numa, pods, 48)
    node, cpus = _numa_parity(cfg, cluster, numa, pods)
    assert (node >= 0).mean() > 0.5
    assert (cpus != 0).any()
