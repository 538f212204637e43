"""The C4 synthetic workload on the oracle (CPU): cpuset accounting invariants of NodeNUMAResource Reserve."""
import numpy as np

from koordinator_amd import abi, framework, synth
from oracle import oracle

F = framework


def test_c4_oracle_cpuset_invariants():
    prof = F.Profile(filter=(F.NODE_RESOURCES_FIT, F.LOAD_AWARE, F.NODE_NUMA_RESOURCE),
                     score={F.NODE_RESOURCES_FIT: 1, F.LOAD_AWARE: 1, F.NODE_NUMA_RESOURCE: 1})
    cfg = F.build_config(profile=prof)
    cluster, numa = synth.make_numa_cluster(200, seed=synth.BASE_SEED + 50)
    pods = synth.make_numa_pods(800, seed=synth.BASE_SEED + 51)
    st = oracle.states(cluster.n)
    oracle.add_pods(cfg, st, cluster.existing_pods, cluster.existing_node)
    buf = oracle.numa_states(numa)
    node, score, cpus = oracle.schedule_numa(cfg, cluster.nodes, cluster.metrics, st, buf, pods, cluster.now_ns,
                                             n_threads=4, with_cpusets=True)
    assert (node >= 0).mean() > 0.5
    counts = np.array([len(F.cpuset_of(c)) for c in cpus])
    cpuset_pod = (pods["qos"] <= abi.QOS["LSR"]) & (pods["qos"] > 0) & (pods["priority_class"] == abi.PRIO_PROD) \
        & (pods["requests"][:, abi.RES_CPU] > 0)
    placed = node >= 0
    # every placed LSE/LSR prod pod got exactly its whole-cpu request as a cpuset; nobody else got cpus
    np.testing.assert_array_equal(counts[placed & cpuset_pod], pods["requests"][placed & cpuset_pod, abi.RES_CPU] // 1000)
    assert (counts[~(placed & cpuset_pod)] == 0).all()
    # the final NodeAllocation = the initial one ∪ the cpusets placed on each node, all disjoint
    alloc, _, _ = oracle.numa_state_read(buf, cluster.n)
    want = numa["allocated_cpus"].copy()
    for k in np.nonzero(placed)[0]:
        assert not (want[node[k]] & cpus[k]).any()
        want[node[k]] |= cpus[k]
    np.testing.assert_array_equal(alloc, want)
