"""Writes the NodeNUMAResource golden fixtures under tests/golden/ — hand transcriptions of the reference's own
table-driven tests (paths under /root/reference/pkg/scheduler/plugins/nodenumaresource/), with source lines.

* numa_take_cpus.json  cpu_accumulator_test.go TestTakeFullPCPUs (:59-173, NUMAMostAllocated),
                       TestTakeFullPCPUsWithNUMALeastAllocated (:175-289), TestTakeSpreadByPCPUs (:301-362).
* numa_take_cpus_exclusive.json  TestTakeCPUsWithExclusivePolicy (:435-558): PCPULevel / NUMANodeLevel / None.
                       topology = buildCPUTopologyForTest(sockets, nodesPerSocket, coresPerNode, cpusPerCore).
* numa_filter.json     plugin_test.go TestPlugin_Filter (:548-816): the cases expressible as a pod (state written
                       by PreFilter; 96 cpu / 512Gi node; zones = CPUsPerNode cores + 32Gi each, :779-786).
                       Kubelet FullPCPUsOnly is the same NodeCPUBindPolicy as the node label (numa_aware.go:314).
* numa_reserve.json    plugin_test.go TestPlugin_Reserve (:931-1150): the chosen cpusets (no zones → no hint).
* numa_score.json      scoring_test.go TestNUMANodeScore (:47-330): zones = capacity / numaNodeCounts, topology
                       buildCPUTopologyForTest(count, 1, cpu/2/count, 2); every existing pod allocates its requests
                       on NUMA node 0 and LSR pods also cpus 0..n-1 (:290-311).  ScoringStrategy MostAllocated.
* numa_affinity.json   plugin_test.go TestFilterWithNUMANodeScoring (:1529-1750): the affinity the topology
                       manager stores, under each NUMAScoringStrategy.
Quantities stay in k8s string form (tests convert them like resource.MustParse + MilliValue/Value).

Run: python tests/golden/make_golden_numa.py   (rewrites the JSON files next to this script)
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
ACC = "pkg/scheduler/plugins/nodenumaresource/cpu_accumulator_test.go"
PLG = "pkg/scheduler/plugins/nodenumaresource/plugin_test.go"
SCO = "pkg/scheduler/plugins/nodenumaresource/scoring_test.go"


def rng(a, b):
    return list(range(a, b + 1))


TAKE = [
    # TestTakeFullPCPUs — NUMAMostAllocated (:159-162)
    dict(line=70, topo=[1, 1, 4, 2], alloc=[], need=2, policy="FullPCPUs", strategy="MostAllocated", want=[0, 1]),
    dict(line=77, topo=[1, 1, 4, 2], alloc=[0, 1], need=2, policy="FullPCPUs", strategy="MostAllocated", want=[2, 3]),
    dict(line=85, topo=[2, 1, 4, 2], alloc=[], need=8, policy="FullPCPUs", strategy="MostAllocated", want=rng(0, 7)),
    dict(line=92, topo=[2, 1, 4, 2], alloc=[], need=12, policy="FullPCPUs", strategy="MostAllocated", want=rng(0, 11)),
    dict(line=99, topo=[2, 1, 4, 2], alloc=[0, 1], need=8, policy="FullPCPUs", strategy="MostAllocated",
         want=rng(8, 15)),
    dict(line=107, topo=[2, 2, 4, 2], alloc=rng(0, 5) + rng(16, 23), need=6, policy="FullPCPUs",
         strategy="MostAllocated", want=rng(24, 29)),
    dict(line=115, topo=[2, 2, 4, 2], alloc=rng(0, 5) + rng(16, 23), need=12, policy="FullPCPUs",
         strategy="MostAllocated", want=rng(6, 15) + [24, 25]),
    dict(line=123, topo=[2, 2, 4, 2], alloc=rng(0, 3) + rng(8, 11), need=4, policy="FullPCPUs",
         strategy="MostAllocated", want=rng(4, 7)),
    dict(line=131, topo=[2, 2, 2, 2], alloc=[0, 2, 4, 8, 12], need=4, policy="FullPCPUs", strategy="MostAllocated",
         want=[10, 11, 14, 15]),
    dict(line=139, topo=[2, 2, 2, 2], alloc=[0, 2, 4, 8, 10, 12], need=6, policy="FullPCPUs",
         strategy="MostAllocated", want=[5, 6, 7, 13, 14, 15]),
    dict(line=147, topo=[2, 2, 2, 2], alloc=[0, 2, 4, 8, 9, 10, 12], need=6, policy="FullPCPUs",
         strategy="MostAllocated", want=[6, 7, 11, 13, 14, 15]),
    # TestTakeFullPCPUsWithNUMALeastAllocated (:276-278)
    dict(line=186, topo=[1, 1, 4, 2], alloc=[], need=2, policy="FullPCPUs", strategy="LeastAllocated", want=[0, 1]),
    dict(line=193, topo=[1, 1, 4, 2], alloc=[0, 1], need=2, policy="FullPCPUs", strategy="LeastAllocated", want=[2, 3]),
    dict(line=201, topo=[2, 1, 4, 2], alloc=[], need=8, policy="FullPCPUs", strategy="LeastAllocated", want=rng(0, 7)),
    dict(line=208, topo=[2, 1, 4, 2], alloc=[], need=12, policy="FullPCPUs", strategy="LeastAllocated",
         want=rng(0, 11)),
    dict(line=215, topo=[2, 1, 4, 2], alloc=[0, 1], need=8, policy="FullPCPUs", strategy="LeastAllocated",
         want=rng(8, 15)),
    dict(line=223, topo=[2, 2, 4, 2], alloc=rng(0, 5) + rng(16, 23), need=6, policy="FullPCPUs",
         strategy="LeastAllocated", want=rng(8, 13)),
    dict(line=231, topo=[2, 2, 4, 2], alloc=rng(0, 5) + rng(16, 23), need=12, policy="FullPCPUs",
         strategy="LeastAllocated", want=rng(6, 15) + [24, 25]),
    dict(line=239, topo=[2, 2, 4, 2], alloc=rng(0, 3) + rng(8, 11), need=4, policy="FullPCPUs",
         strategy="LeastAllocated", want=rng(16, 19)),
    dict(line=247, topo=[2, 2, 2, 2], alloc=[0, 2, 4, 8, 12], need=4, policy="FullPCPUs", strategy="LeastAllocated",
         want=[10, 11, 14, 15]),
    dict(line=255, topo=[2, 2, 2, 2], alloc=[0, 2, 4, 8, 10, 12], need=6, policy="FullPCPUs",
         strategy="LeastAllocated", want=[1, 3, 6, 7, 14, 15]),
    dict(line=263, topo=[2, 2, 4, 2], alloc=[0, 2, 4, 8, 9, 10, 12], need=6, policy="FullPCPUs",
         strategy="LeastAllocated", want=rng(16, 21)),
    # TestTakeSpreadByPCPUs — NUMAMostAllocated (:348-350)
    dict(line=312, topo=[1, 1, 4, 2], alloc=[], need=4, policy="SpreadByPCPUs", strategy="MostAllocated",
         want=[0, 2, 4, 6]),
    dict(line=319, topo=[2, 1, 4, 2], alloc=[0, 2], need=4, policy="SpreadByPCPUs", strategy="MostAllocated",
         want=[1, 3, 4, 6]),
    dict(line=327, topo=[2, 1, 4, 2], alloc=[0, 1, 2, 3], need=4, policy="SpreadByPCPUs", strategy="MostAllocated",
         want=[8, 10, 12, 14]),
    dict(line=335, topo=[2, 1, 4, 2], alloc=[0, 2], need=6, policy="SpreadByPCPUs", strategy="MostAllocated",
         want=[1] + rng(3, 7)),
]

# TestPlugin_Filter: node 96 cpu / 512Gi, topology buildCPUTopologyForTest(2, 1, 4, 2), zones 8 cpus + 32Gi
# each; the pod requests only cpu (state.requests = {cpu: numCPUsNeeded}, :799-801) and is LSR/prod so that
# PreFilter writes requestCPUBind with the listed policies.
FILTER = [
    dict(line=596, name="verify FullPCPUsOnly with SMTAlignmentError", node_bind="FullPCPUsOnly", numa_policy="",
         required="", preferred="FullPCPUs", cpus=5, want="UnschedulableAndUnresolvable"),
    dict(line=610, name="verify required FullPCPUs SMTAlignmentError", node_bind="", numa_policy="",
         required="FullPCPUs", preferred="FullPCPUs", cpus=5, want="UnschedulableAndUnresolvable"),
    dict(line=622, name="verify FullPCPUsOnly with preferred SpreadByPCPUs", node_bind="FullPCPUsOnly", numa_policy="",
         required="", preferred="SpreadByPCPUs", cpus=4, want="UnschedulableAndUnresolvable"),
    dict(line=636, name="verify FullPCPUsOnly with required SpreadByPCPUs", node_bind="FullPCPUsOnly", numa_policy="",
         required="SpreadByPCPUs", preferred="SpreadByPCPUs", cpus=4, want="UnschedulableAndUnresolvable"),
    dict(line=651, name="verify Kubelet FullPCPUsOnly with SMTAlignmentError", node_bind="FullPCPUsOnly",
         numa_policy="", required="", preferred="FullPCPUs", cpus=5, want="UnschedulableAndUnresolvable"),
    dict(line=668, name="verify Kubelet FullPCPUsOnly with RequiredFullPCPUsPolicy", node_bind="FullPCPUsOnly",
         numa_policy="", required="", preferred="SpreadByPCPUs", cpus=4, want="UnschedulableAndUnresolvable"),
    dict(line=685, name="verify required FullPCPUs with none NUMA topology policy", node_bind="", numa_policy="",
         required="FullPCPUs", preferred="FullPCPUs", cpus=4, want="Success"),
    dict(line=696, name="verify FullPCPUs with NUMA Topology Policy", node_bind="", numa_policy="SingleNUMANode",
         required="FullPCPUs", preferred="FullPCPUs", cpus=4, want="Success"),
]

# TestPlugin_Reserve: node 96 cpu / 512Gi, no zones (no hint), the listed topology/allocations/labels.
RESERVE = [
    dict(line=975, name="succeed with valid cpu topology", topo=[2, 1, 4, 2], alloc=[], node_bind="",
         strategy=None, preferred="FullPCPUs", cpus=4, want=[0, 1, 2, 3]),
    dict(line=987, name="allocated by node cpu bind policy", topo=[2, 1, 4, 2], alloc=[], node_bind="SpreadByPCPUs",
         strategy=None, preferred="FullPCPUs", cpus=4, want=[0, 2, 4, 6]),
    dict(line=1007, name="error with big request cpu", topo=[2, 1, 4, 2], alloc=[], node_bind="", strategy=None,
         preferred="FullPCPUs", cpus=24, want=None),
    dict(line=1017, name="succeed with valid cpu topology and node numa least allocate strategy", topo=[2, 1, 8, 2],
         alloc=[0, 1, 2, 3], node_bind="", strategy="LeastAllocated", preferred="FullPCPUs", cpus=4,
         want=[16, 17, 18, 19]),
    dict(line=1033, name="succeed with valid cpu topology and node numa most allocate strategy", topo=[2, 1, 8, 2],
         alloc=[0, 1, 2, 3], node_bind="", strategy="MostAllocated", preferred="FullPCPUs", cpus=4,
         want=[4, 5, 6, 7]),
]


def node(name, cpu, mem, policy):
    return dict(name=name, cpu=cpu, memory=mem, numa_policy=policy)


# TestNUMANodeScore (MostAllocated ScoringStrategy, default LeastAllocated NUMAScoringStrategy)
SCORE = [
    dict(line=58, name="single numa nodes score", strategy="MostAllocated",
         nodes=[node("test-node-1", "104", "256Gi", "SingleNUMANode"), node("test-node-2", "64", "128Gi",
                                                                           "SingleNUMANode")],
         numa_counts=[2, 1], pod=dict(cpu="21", memory="40Gi", qos=""), existing=[], want=[35, 31]),
    dict(line=99, name="restricted numa nodes score", strategy="MostAllocated",
         nodes=[node("test-node-1", "104", "256Gi", "Restricted"), node("test-node-2", "64", "128Gi", "Restricted")],
         numa_counts=[2, 1], pod=dict(cpu="50", memory="40Gi", qos=""), existing=[], want=[63, 54]),
    dict(line=140, name="single numa nodes score with same capacity but different requested", strategy="MostAllocated",
         nodes=[node("test-node-%d" % i, "104", "256Gi", "SingleNUMANode") for i in (1, 2, 3)],
         numa_counts=[2, 2, 2], pod=dict(cpu="4", memory="40Gi", qos=""),
         existing=[dict(node=0, cpu="4", memory="8Gi", qos=""), dict(node=1, cpu="8", memory="32Gi", qos=""),
                   dict(node=2, cpu="32", memory="40Gi", qos="")],
         want=[19, 19, 19]),
    dict(line=195, name="single numa nodes score with same capacity but different requested and LSR",
         strategy="MostAllocated",
         nodes=[node("test-node-%d" % i, "104", "256Gi", "SingleNUMANode") for i in (1, 2, 3)],
         numa_counts=[2, 2, 2], pod=dict(cpu="4", memory="40Gi", qos="LSR"),
         existing=[dict(node=0, cpu="4", memory="8Gi", qos=""), dict(node=0, cpu="4", memory="8Gi", qos="LSR"),
                   dict(node=1, cpu="8", memory="32Gi", qos=""), dict(node=1, cpu="8", memory="32Gi", qos="LSR"),
                   dict(node=2, cpu="16", memory="40Gi", qos=""), dict(node=2, cpu="16", memory="40Gi", qos="LSR")],
         want=[23, 27, 34]),
]

# TestFilterWithNUMANodeScoring: node 104 cpu / 256Gi, zones capacity/count; existing pods allocate on the
# given NUMA node; want = the stored affinity's bits.
AFFINITY = [
    dict(line=1566, name="single numa nodes and select most allocated", policy="SingleNUMANode", count=2,
         numa_strategy="MostAllocated", existing={0: [("4", "8Gi")], 1: [("40", "8Gi")]}, want=[1]),
    dict(line=1588, name="single numa nodes and select least allocated", policy="SingleNUMANode", count=2,
         numa_strategy="LeastAllocated", existing={0: [("4", "8Gi")], 1: [("40", "8Gi")]}, want=[0]),
    dict(line=1610, name="single numa nodes and only one node can be used", policy="SingleNUMANode", count=2,
         numa_strategy="LeastAllocated", existing={0: [("4", "8Gi")], 1: [("52", "8Gi")]}, want=[0]),
    dict(line=1632, name="restricted numa nodes and select most allocated and preferred", policy="Restricted",
         count=4, numa_strategy="MostAllocated",
         existing={0: [("24", "8Gi")], 1: [("23", "8Gi")], 2: [("4", "8Gi")], 3: [("8", "8Gi")]}, want=[3]),
    dict(line=1660, name="restricted numa nodes and select least allocated and preferred", policy="Restricted",
         count=4, numa_strategy="LeastAllocated",
         existing={0: [("24", "8Gi")], 1: [("23", "8Gi")], 2: [("4", "8Gi")], 3: [("8", "8Gi")]}, want=[2]),
]


# TestTakeCPUsWithExclusivePolicy (:435-558): allocatedExclusiveCPUs are allocated (not available) and hold
# allocatedExclusivePolicy (default PCPULevel, :530-534); the pod's exclusivePolicy defaults to PCPULevel (:538-540),
# bindPolicy to SpreadByPCPUs (:541-543); maxRefCount 1; NUMAMostAllocated (:547).
EXCL = [
    dict(line=448, name="allocate cpus on full-free socket with PCPULevel", topo=[2, 1, 4, 2], alloc=[0, 2],
         alloc_policy="PCPULevel", excl="PCPULevel", policy="SpreadByPCPUs", need=4, want=[8, 10, 12, 14]),
    dict(line=456, name="allocate overlapped cpus with PCPULevel", topo=[2, 1, 4, 2], alloc=[],
         alloc_policy="PCPULevel", excl="PCPULevel", policy="SpreadByPCPUs", need=10,
         want=[0, 1, 2, 3, 4, 6, 8, 10, 12, 14]),
    dict(line=463, name="allocate cpus on large-size partially-allocated socket with PCPULevel", topo=[2, 1, 8, 2],
         alloc=[0, 2], alloc_policy="PCPULevel", excl="PCPULevel", policy="SpreadByPCPUs", need=4,
         want=[4, 6, 8, 10]),
    dict(line=471, name="allocate cpus with none exclusive policy", topo=[2, 1, 8, 2], alloc=[0, 2],
         alloc_policy="PCPULevel", excl="None", policy="SpreadByPCPUs", need=4, want=[1, 3, 4, 6]),
    dict(line=480, name="allocate cpus on full-free socket with NUMANodeLevel", topo=[2, 1, 4, 2], alloc=[0, 2],
         alloc_policy="NUMANodeLevel", excl="NUMANodeLevel", policy="SpreadByPCPUs", need=4, want=[8, 10, 12, 14]),
    dict(line=490, name="allocate cpus on partially-allocated socket without NUMANodeLevel", topo=[2, 1, 4, 2],
         alloc=[0, 2], alloc_policy="NUMANodeLevel", excl="None", policy="SpreadByPCPUs", need=4,
         want=[1, 3, 4, 6]),
    dict(line=500, name="allocate cpus on full-free socket with NUMANodeLevel with PCPUs", topo=[2, 1, 4, 2],
         alloc=[0, 2], alloc_policy="NUMANodeLevel", excl="NUMANodeLevel", policy="FullPCPUs", need=4,
         want=[8, 9, 10, 11]),
    dict(line=511, name="allocate cpus on partially-allocated socket without NUMANodeLevel with PCPUs",
         topo=[2, 1, 4, 2], alloc=[0, 2], alloc_policy="NUMANodeLevel", excl="None", policy="FullPCPUs", need=4,
         want=[4, 5, 6, 7]),
]
for c in EXCL:
    c["strategy"] = "MostAllocated"


def main():
    docs = {
        "numa_take_cpus_exclusive.json": dict(source=ACC, harness="takeCPUs(topology, 1, available, allocated with "
                                                                  "alloc_policy, need, policy, excl, NUMAMostAllocated)",
                                              cases=EXCL),
        "numa_take_cpus.json": dict(source=ACC, harness="takeCPUs(topology, 1, available, allocated, need, policy, "
                                                        "CPUExclusivePolicyNone, strategy)", cases=TAKE),
        "numa_filter.json": dict(source=PLG, harness="TestPlugin_Filter :744-815", cases=FILTER),
        "numa_reserve.json": dict(source=PLG, harness="TestPlugin_Reserve :1064-1149", cases=RESERVE),
        "numa_score.json": dict(source=SCO, harness="TestNUMANodeScore :261-329", pod_request="st.MakePod().Req",
                                cases=SCORE),
        "numa_affinity.json": dict(source=PLG, harness="TestFilterWithNUMANodeScoring :1689-1749",
                                   pod=dict(cpu="4", memory="40Gi"), cases=AFFINITY),
    }
    for name, doc in docs.items():
        for c in doc["cases"]:
            c["source_line"] = f"{doc['source']}:{c['line']}"
        with open(os.path.join(HERE, name), "w") as fh:
            json.dump(doc, fh, indent=1)
        print("wrote", name, len(doc["cases"]), "cases")


if __name__ == "__main__":
    main()
