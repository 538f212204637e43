"""Writes tests/golden/numa_amplify.json — a hand transcription of the reference's TestFilterWithAmplifiedCPUs
(pkg/scheduler/plugins/nodenumaresource/plugin_test.go:818-913), with source lines.

Each case: node cpu = Amplify(32 cpus, ratio) cores, memory 40Gi, annotated with the cpu amplification ratio
(makeNode :115-119); topology buildCPUTopologyForTest(2, 1, 8, 2) = 32 cpus; with an NRT the two NUMA zones
hold Amplify(16, ratio) cores + 20Gi each (:896-909).  The one existing pod is bound to the node (makePodOnNode
:121-135: a cpuset pod is LSR with ResourceStatus cpuset 0-(n-1)); the pod to filter is LSR/prod when it is a
cpuset pod.  want = the Filter status.

Run: python tests/golden/make_golden_numa_amp.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = "pkg/scheduler/plugins/nodenumaresource/plugin_test.go"

CASES = [
    dict(line=829, name="no resources requested always fits", pod=None, pod_cpuset=False, existing=4,
         existing_cpuset=False, nrt=False, ratio=2.0, want="Success"),
    dict(line=836, name="no filtering without node cpu amplification", pod=32, pod_cpuset=False, existing=32,
         existing_cpuset=False, nrt=False, ratio=1.0, want="Success"),
    dict(line=843, name="cpu fits on no NRT node", pod=32, pod_cpuset=False, existing=32, existing_cpuset=False,
         nrt=False, ratio=2.0, want="Success"),
    dict(line=850, name="insufficient cpu", pod=32, pod_cpuset=False, existing=64, existing_cpuset=False, nrt=False,
         ratio=2.0, want="Unschedulable"),
    dict(line=858, name="insufficient cpu with cpuset pod on node", pod=32, pod_cpuset=False, existing=32,
         existing_cpuset=True, nrt=True, ratio=2.0, want="Unschedulable"),
    dict(line=867, name="insufficient cpu when scheduling cpuset pod", pod=32, pod_cpuset=True, existing=32,
         existing_cpuset=False, nrt=True, ratio=2.0, want="Unschedulable"),
    dict(line=876, name="insufficient cpu when scheduling cpuset pod with cpuset pod on node", pod=32,
         pod_cpuset=True, existing=32, existing_cpuset=True, nrt=True, ratio=2.0, want="Unschedulable"),
]

if __name__ == "__main__":
    out = {"source": SRC, "topology": [2, 1, 8, 2], "node_memory": "40Gi", "zone_memory": "20Gi",
           "cases": [dict(c, source_line=f"{SRC}:{c.pop('line')}") for c in CASES]}
    with open(os.path.join(HERE, "numa_amplify.json"), "w") as f:
        json.dump(out, f, indent=1)
