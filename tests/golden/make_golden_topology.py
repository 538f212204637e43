"""Writes tests/golden/topology_policy.json: the reference's topology-manager policy tables, hand-transcribed.

Source (read as text, never executed): /root/reference/pkg/scheduler/frameworkext/topologymanager/
  policy_test.go:60-341      commonPolicyMergeTestCases (run by every policy's Merge test)
  policy_test.go:344-609     bestEffortPolicy.mergeTestCases (also the restricted policy's: restrictedPolicy embeds
                             bestEffortPolicy, policy_restricted_test.go:71-78)
  policy_test.go:612-883     singleNumaNodePolicy.mergeTestCases
  policy_best_effort_test.go:53-60, policy_restricted_test.go:71-78, policy_single_numa_node_test.go:159-166
                             the Merge tests (numaNodes = {0, 1}; Merge's hint is compared, testPolicyMerge :885-899)
  policy_*_test.go canAdmitPodResult tables (best effort :24-51, restricted :42-69, single :25-47)
  policy_single_numa_node_test.go:49-157  TestPolicySingleNumaNodeFilterHints (filterSingleNumaHints)

Encoding: a provider is null (GetPodTopologyHints returns a nil map), {} (an empty map) or {resource: hints} where hints
is null (a nil slice), [] (an empty slice) or a list of [mask, preferred] with mask = the NUMA node ids of
NewTestBitMask(...) or null for a nil NUMANodeAffinity.  Scores are all 0 in these tables.  An expected hint is
[mask or null, preferred]."""
import json
import os

T, F = True, False
FILE = "pkg/scheduler/frameworkext/topologymanager/policy_test.go"


def prov(**res):
    return {k: v for k, v in res.items()}


COMMON = [
    (63, "Two providers, 1 hint each, same mask, both preferred 1/2",
     [prov(resource1=[[[0], T]]), prov(resource2=[[[0], T]])], [[0], T]),
    (92, "Two providers, 1 hint each, same mask, both preferred 2/2",
     [prov(resource1=[[[1], T]]), prov(resource2=[[[1], T]])], [[1], T]),
    (121, "Two providers, 1 no hints, 1 single hint preferred 1/2",
     [None, prov(resource=[[[0], T]])], [[0], T]),
    (141, "Two providers, 1 no hints, 1 single hint preferred 2/2",
     [None, prov(resource=[[[1], T]])], [[1], T]),
    (161, "Two providers, 1 with 2 hints, 1 with single hint matching 1/2",
     [prov(resource1=[[[0], T], [[1], T]]), prov(resource2=[[[0], T]])], [[0], T]),
    (194, "Two providers, 1 with 2 hints, 1 with single hint matching 2/2",
     [prov(resource1=[[[0], T], [[1], T]]), prov(resource2=[[[1], T]])], [[1], T]),
    (227, "Two providers, both with 2 hints, matching narrower preferred hint from both",
     [prov(resource1=[[[0], T], [[1], T]]), prov(resource2=[[[0], T], [[0, 1], F]])], [[0], T]),
    (264, "Ensure less narrow preferred hints are chosen over narrower non-preferred hints",
     [prov(resource1=[[[1], T], [[0, 1], F]]), prov(resource2=[[[0], T], [[1], T], [[0, 1], F]])], [[1], T]),
    (305, "Multiple resources, same provider",
     [prov(resource1=[[[1], T], [[0, 1], F]], resource2=[[[0], T], [[1], T], [[0, 1], F]])], [[1], T]),
]

BEST_EFFORT = [
    (347, "NUMATopologyHint not set", [], [[0, 1], T]),
    (355, "NUMATopologyHintProvider returns empty non-nil map[string][]NUMATopologyHint", [{}], [[0, 1], T]),
    (367, "NUMATopologyHintProvider returns -nil map[string][]NUMATopologyHint from provider",
     [prov(resource=None)], [[0, 1], T]),
    (381, "NUMATopologyHintProvider returns empty non-nil map[string][]NUMATopologyHint from provider",
     [prov(resource=[])], [[0, 1], F]),
    (394, "Single NUMATopologyHint with Preferred as true and NUMANodeAffinity as nil",
     [prov(resource=[[None, T]])], [[0, 1], T]),
    (413, "Single NUMATopologyHint with Preferred as false and NUMANodeAffinity as nil",
     [prov(resource=[[None, F]])], [[0, 1], F]),
    (432, "Two providers, 1 hint each, no common mask",
     [prov(resource1=[[[0], T]]), prov(resource2=[[[1], T]])], [[0, 1], F]),
    (461, "Two providers, 1 hint each, same mask, 1 preferred, 1 not 1/2",
     [prov(resource1=[[[0], T]]), prov(resource2=[[[0], F]])], [[0], F]),
    (490, "Two providers, 1 hint each, same mask, 1 preferred, 1 not 2/2",
     [prov(resource1=[[[1], T]]), prov(resource2=[[[1], F]])], [[1], F]),
    (519, "Two providers, 1 hint each, 1 wider mask, both preferred 1/2",
     [prov(resource1=[[[0], T]]), prov(resource2=[[[0, 1], T]])], [[0], T]),
    (548, "Two providers, 1 with 2 hints, 1 with single non-preferred hint matching",
     [prov(resource1=[[[0], T], [[1], T]]), prov(resource2=[[[0, 1], F]])], [[0], F]),
    (581, "Two providers, 1 hint each, 1 wider mask, both preferred 1/2",
     [prov(resource1=[[[1], T]]), prov(resource2=[[[0, 1], T]])], [[1], T]),
]

SINGLE = [
    (615, "NUMATopologyHint not set", [], [None, T]),
    (623, "NUMATopologyHintProvider returns empty non-nil map[string][]NUMATopologyHint", [{}], [None, T]),
    (635, "NUMATopologyHintProvider returns -nil map[string][]NUMATopologyHint from provider",
     [prov(resource=None)], [None, T]),
    (649, "NUMATopologyHintProvider returns empty non-nil map[string][]NUMATopologyHint from provider",
     [prov(resource=[])], [None, F]),
    (662, "Single NUMATopologyHint with Preferred as true and NUMANodeAffinity as nil",
     [prov(resource=[[None, T]])], [None, T]),
    (681, "Single NUMATopologyHint with Preferred as false and NUMANodeAffinity as nil",
     [prov(resource=[[None, F]])], [None, F]),
    (700, "Two providers, 1 hint each, no common mask",
     [prov(resource1=[[[0], T]]), prov(resource2=[[[1], T]])], [None, F]),
    (729, "Two providers, 1 hint each, same mask, 1 preferred, 1 not 1/2",
     [prov(resource1=[[[0], T]]), prov(resource2=[[[0], F]])], [None, F]),
    (758, "Two providers, 1 hint each, same mask, 1 preferred, 1 not 2/2",
     [prov(resource1=[[[1], T]]), prov(resource2=[[[1], F]])], [None, F]),
    (787, "Two providers, 1 with 2 hints, 1 with single non-preferred hint matching",
     [prov(resource1=[[[0], T], [[1], T]]), prov(resource2=[[[0, 1], F]])], [None, F]),
    (820, "Single NUMA hint generation",
     [prov(resource1=[[[0, 1], T]], resource2=[[[0], T], [[1], T], [[0, 1], F]])], [None, F]),
    (853, "One no-preference provider",
     [prov(resource1=[[[0], T], [[1], T], [[0, 1], F]]), None], [[0], T]),
]

# TestPolicySingleNumaNodeFilterHints (policy_single_numa_node_test.go:49-157): input lists -> filtered lists
FILTER = [
    (56, "filter empty resources", [], []),
    (61, "filter hints with nil socket mask 1/2",
     [[[None, F]], [[None, T]]], [[], [[None, T]]]),
    (78, "filter hints with nil socket mask 2/2",
     [[[[0], T], [None, F]], [[[1], T], [None, T]]], [[[[0], T]], [[[1], T], [None, T]]]),
    (100, "filter hints with empty resource socket mask",
     [[[[1], T], [[0], T], [None, F]], []], [[[[1], T], [[0], T]], []]),
    (118, "filter hints with wide sockemask",
     [[[[0], T], [[1], T], [[1, 2], F], [[0, 1, 2], F], [None, F]],
      [[[1, 2], F], [[0, 1, 2], F], [[0, 2], F], [[3], F]],
      [[[1, 2], F], [[0, 1, 2], F], [[0, 2], F]]],
     [[[[0], T], [[1], T]], [], []]),
]

# canAdmitPodResult: hint {nil, preferred} -> admit
ADMIT = {
    "best-effort": [("policy_best_effort_test.go:31", F, T), ("policy_best_effort_test.go:36", T, T)],
    "restricted": [("policy_restricted_test.go:49", F, F), ("policy_restricted_test.go:54", T, T)],
    "single-numa-node": [("policy_single_numa_node_test.go:32", F, F)],
}


def cases(policy, rows):
    return [{"policy": policy, "name": n, "providers": hp, "want": w, "source_line": f"{FILE}:{ln}"}
            for ln, n, hp, w in rows]


def main():
    out = {
        "numa_nodes": [0, 1],
        "merge": cases("best-effort", COMMON + BEST_EFFORT) + cases("restricted", COMMON + BEST_EFFORT) +
        cases("single-numa-node", COMMON + SINGLE),
        "single_numa_filter": [{"name": n, "lists": a, "want": w,
                                "source_line": f"pkg/scheduler/frameworkext/topologymanager/policy_single_numa_node_test.go:{ln}"}
                               for ln, n, a, w in FILTER],
        "admit": {k: [{"source_line": f"pkg/scheduler/frameworkext/topologymanager/{s}", "preferred": p, "want": w}
                      for s, p, w in v] for k, v in ADMIT.items()},
    }
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "topology_policy.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(path, len(out["merge"]), "merge cases")


if __name__ == "__main__":
    main()
