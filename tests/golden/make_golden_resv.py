"""Writes tests/golden/reservation.json: Reservation plugin cases transcribed from the reference's own tests.

Every value below is read off the cited test table (no reference code is run: there is no Go toolchain here).
Each case is one node with an explicit nodeReservationState whose `matched` holds every listed reservation, as the
tests build it; expected values are the tests' assertions:
  * reservation/scoring_test.go TestScore (:40-253) — Score after PreScore on one node (node Status empty:
    allocatable 0, AllowedPodNumber 0), podRequested / rAllocated nil;
  * reservation/scoring_test.go TestPreScore (:392-729) — the nominated reservation on that node;
  * reservation/plugin_test.go Test_filterWithReservations (:670-1280) — filterWithReservations status, node
    32 cpu / 32Gi / 100 pods (the test passes an empty pod, so no reservation's ResourceNames intersect it).
"""
import json
import os

GI = 1 << 30


def slot(cpu_cores, mem_gi, allocated=(0, 0), policy=0):
    return {"allocatable_cpu": cpu_cores * 1000, "allocatable_mem": int(mem_gi * GI),
            "allocated_cpu": allocated[0], "allocated_mem": allocated[1], "policy": policy}


R4C8G, R2C4G = slot(4, 8), slot(2, 4)
EMPTY_NODE = {"alloc": [0, 0], "allowed_pods": 0, "num_pods": 0, "pod_requested": [0, 0], "r_allocated": [0, 0]}
NODE32 = {"alloc": [32000, 32 * GI], "allowed_pods": 100, "num_pods": 0, "r_allocated": [0, 0]}

CASES = [
    # TestScore
    dict(ref="scoring_test.go:121 no reservation matched on the node", pod=[0, 0], slots=[], has_state=0,
         **EMPTY_NODE, want_score=0),
    dict(ref="scoring_test.go:127 reservation matched but zero-request pod", pod=[0, 0], slots=[R2C4G], has_state=1,
         **EMPTY_NODE, want_score=0),
    dict(ref="scoring_test.go:135 reservation matched and pod has part empty resource requests", pod=[2000, 4 * GI],
         slots=[R4C8G], has_state=1, **EMPTY_NODE, want_score=50),
    dict(ref="scoring_test.go:156 allocated reservation matched", pod=[2000, 4 * GI],
         slots=[slot(2, 4, allocated=(2000, 3 * GI))], has_state=1, **EMPTY_NODE, want_score=0),
    dict(ref="scoring_test.go:183 multi reservations matched", pod=[2000, 4 * GI], slots=[R4C8G, R2C4G], has_state=1,
         **EMPTY_NODE, want_score=100),
    # TestPreScore nomination
    dict(ref="scoring_test.go:590 allocated reservation", pod=[2000, 4 * GI],
         slots=[R4C8G, slot(2, 4, allocated=(2000, 4 * GI))], has_state=1, **EMPTY_NODE, want_nominated=0),
    dict(ref="scoring_test.go:621 matched reservations", pod=[2000, 4 * GI], slots=[R4C8G, R2C4G], has_state=1,
         **EMPTY_NODE, want_nominated=1),
    # Test_filterWithReservations (empty pod)
    dict(ref="plugin_test.go:688 filter aligned reservation with nodeInfo", pod=[0, 0], affinity=0,
         slots=[dict(slot(6, 0), policy=1)], has_state=1, pod_requested=[30000, 24 * GI], **NODE32, want_pass=1),
    dict(ref="plugin_test.go:703 failed to filter aligned reservation with nodeInfo", pod=[0, 0], affinity=1,
         slots=[dict(slot(6, 0), policy=1)], has_state=1, pod_requested=[32000, 24 * GI], **NODE32, want_pass=0),
    dict(ref="plugin_test.go:748 filter restricted reservation with nodeInfo", pod=[0, 0], affinity=0,
         slots=[dict(slot(6, 0), policy=2)], has_state=1, pod_requested=[30000, 24 * GI], **NODE32, want_pass=1),
    dict(ref="plugin_test.go:792 failed to filter restricted reservation with nodeInfo", pod=[0, 0], affinity=1,
         slots=[dict(slot(6, 0), policy=2)], has_state=1, pod_requested=[30000, 24 * GI], **NODE32, want_pass=0),
]

if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reservation.json")
    with open(out, "w") as f:
        json.dump({"source": "hhyasdf/koordinator pkg/scheduler/plugins/reservation tests", "cases": CASES}, f,
                  indent=1)
    print(f"wrote {len(CASES)} cases to {out}")
