"""Writes two more NodeNUMAResource Score fixtures, hand-transcribed from the reference's scoring_test.go
(paths under /root/reference/pkg/scheduler/plugins/nodenumaresource/), with source lines.

* numa_plugin_score.json   TestPlugin_Score (scoring_test.go:332-554): Score called straight after a preFilterState
  is written (no Filter, so no stored affinity).  Node: Allocatable cpu = the topology's cpus x 1000 (96 without a
  topology), memory 512Gi, node labels per case; no NUMA zones, no NUMA policy.  ScoringStrategy MostAllocated over
  cpu weight 1 (:486-494).  The preFilterState is expressed as the pod PreFilter turns into it: requestCPUBind with
  numCPUsNeeded n = an LSR koord-prod pod requesting n cpus (requests = cpu only, :521-526) whose preferred bind
  policy is the state's.  The cases that write a state PreFilter cannot produce (a missing state, requestCPUBind
  with zero cpus, an empty CPUTopology) are listed under "skipped" with the reason.
* numa_score_amplified.json  TestScoreWithAmplifiedCPUs (scoring_test.go:556-814): node1 cpu 32 / 40Gi ratio 1,
  node2 cpu 64 / 60Gi ratio 2 (makeNode sets the amplification-ratio annotation, plugin_test.go:114-118); with NRT the
  topology is buildCPUTopologyForTest(2, 1, 8, 2) and each of the 2 NUMA zones has Amplify(16, ratio) cpus and 20Gi
  (:765-788); the existing pod (20 cpu, 4Gi) holds cpus 0-19 when it is a cpuset pod (makePodOnNode
  plugin_test.go:120-133: the resource-status annotation carries only the CPUSet, so the NodeAllocation has no NUMA
  resources).  Score runs after PreFilter only (:796-808).

Run: python tests/golden/make_golden_numa_score2.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
SCO = "pkg/scheduler/plugins/nodenumaresource/scoring_test.go"

PLUGIN_SCORE = [
    # line, name, topology, needed, preferred policy, node labels {numa_allocate_strategy, node_cpu_bind_policy}, want
    dict(line=367, name="succeed with skip", topo=None, needed=0, preferred="", labels={}, want=0),
    dict(line=376, name="score with full empty node FullPCPUs", topo=[2, 1, 4, 2], needed=4, preferred="FullPCPUs",
         labels={}, want=25),
    dict(line=388, name="score with satisfied node FullPCPUs", topo=[2, 1, 4, 2], needed=8, preferred="FullPCPUs",
         labels={}, want=50),
    dict(line=401, name="score with full empty node SpreadByPCPUs", topo=[2, 1, 4, 2], needed=4,
         preferred="SpreadByPCPUs", labels={}, want=25),
    dict(line=413, name="score with exceed socket FullPCPUs", topo=[2, 1, 4, 2], needed=16, preferred="FullPCPUs",
         labels={}, want=100),
    dict(line=425, name="score with satisfied socket FullPCPUs", topo=[2, 2, 4, 2], needed=16, preferred="FullPCPUs",
         labels={}, want=50),
    dict(line=437, name="score with full empty socket SpreadByPCPUs", topo=[2, 1, 4, 2], needed=4,
         preferred="SpreadByPCPUs", labels={}, want=25),
    dict(line=449, name="score with Node NUMA Allocate Strategy", topo=[2, 1, 4, 2], needed=2,
         preferred="SpreadByPCPUs", labels={"numa_allocate_strategy": "LeastAllocated"}, want=12),
    dict(line=464, name="score with Node CPU Bind Policy", topo=[2, 1, 4, 2], needed=8, preferred="SpreadByPCPUs",
         labels={"node_cpu_bind_policy": "FullPCPUsOnly"}, want=50),
]
PLUGIN_SKIPPED = [
    dict(line=343, name="error with missing preFilterState", reason="no preFilterState: PreFilter always writes one"),
    dict(line=348, name="error with missing allocationState",
         reason="requestCPUBind with numCPUsNeeded 0: PreFilter sets requestCPUBind only for a non-zero cpu request"),
    dict(line=357, name="error with invalid cpu topology",
         reason="same state as :348 (requestCPUBind, no cpus) on an empty CPUTopology"),
]

AMP = [
    # line, name, strategy, pod cpuset, existing cpuset (None = no existing pod), nrt, want
    dict(line=569, name="ScoringStrategy MostAllocated, no cpuset pod", strategy="MostAllocated", pod_cpuset=False,
         existing=None, nrt=False, want=[0, 0]),
    dict(line=585, name="ScoringStrategy MostAllocated, cpuset pods on node", strategy="MostAllocated",
         pod_cpuset=False, existing=True, nrt=True, want=[68, 54]),
    dict(line=610, name="ScoringStrategy MostAllocated, scheduling cpuset pod", strategy="MostAllocated",
         pod_cpuset=True, existing=False, nrt=True, want=[37, 29]),
    dict(line=635, name="ScoringStrategy MostAllocated, cpuset pods on node, scheduling cpuset pod",
         strategy="MostAllocated", pod_cpuset=True, existing=True, nrt=True, want=[68, 60]),
    dict(line=660, name="ScoringStrategy LeastAllocated, no cpuset pod", strategy="LeastAllocated", pod_cpuset=False,
         existing=False, nrt=False, want=[0, 0]),
    dict(line=680, name="ScoringStrategy LeastAllocated, cpuset pods on node", strategy="LeastAllocated",
         pod_cpuset=False, existing=True, nrt=True, want=[31, 45]),
    dict(line=705, name="ScoringStrategy LeastAllocated, scheduling cpuset pod", strategy="LeastAllocated",
         pod_cpuset=True, existing=False, nrt=True, want=[62, 70]),
    dict(line=730, name="ScoringStrategy LeastAllocated, cpuset pods on node,scheduling cpuset pod",
         strategy="LeastAllocated", pod_cpuset=True, existing=True, nrt=True, want=[31, 39]),
]


def main():
    for c in PLUGIN_SCORE + PLUGIN_SKIPPED + AMP:
        c["source_line"] = f"{SCO}:{c.pop('line')}"
    docs = {
        "numa_plugin_score.json": {"strategy": "MostAllocated", "resources": {"cpu": 1}, "node_memory": "512Gi",
                                   "cases": PLUGIN_SCORE, "skipped": PLUGIN_SKIPPED},
        "numa_score_amplified.json": {
            "nodes": [{"cpu": "32", "memory": "40Gi", "ratio": 1.0}, {"cpu": "64", "memory": "60Gi", "ratio": 2.0}],
            "topology": [2, 1, 8, 2], "zone_memory": "20Gi", "pod": {"cpu": "8", "memory": "16Gi"},
            "existing_pod": {"cpu": "20", "memory": "4Gi"}, "resources": {"cpu": 1, "memory": 1}, "cases": AMP},
    }
    for name, doc in docs.items():
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(doc, f, indent=1)
        print(name, len(doc["cases"]))


if __name__ == "__main__":
    main()
