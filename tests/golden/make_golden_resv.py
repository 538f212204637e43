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

# nominator_test.go TestNominateReservation (:40-283): the nominated reservation of one node whose state matches every
# listed reservation; node Status empty, pod 2C4G (`reservations` order = slot order).  "reserve pod" (:169) is out of
# scope: reserve pods themselves are scheduled on the Go path.
CASES += [
    dict(ref="nominator_test.go:110 reserve pod", pod=[0, 0], slots=[], has_state=0, **EMPTY_NODE, want_nominated=-1,
         reserve=1),
    # derived from nominator.go:77 (a reserve pod nominates nothing) with the :253 reservations on the node: not a
    # reference table row
    dict(ref="nominator.go:77 reserve pod beside matching reservations (derived)", pod=[2000, 4 * GI],
         slots=[R4C8G, R2C4G], has_state=1, **EMPTY_NODE, want_nominated=-1, reserve=1),
    dict(ref="nominator_test.go:121 node without reservations", pod=[2000, 4 * GI], slots=[], has_state=0, **EMPTY_NODE,
         want_nominated=-1),
    dict(ref="nominator_test.go:126 preferred reservation", pod=[2000, 4 * GI],
         slots=[dict(slot(2, 4), order=100), slot(2, 4)], has_state=1, **EMPTY_NODE, want_nominated=0),
    dict(ref="nominator_test.go:224 allocated reservation", pod=[2000, 4 * GI],
         slots=[R4C8G, slot(2, 4, allocated=(2000, 4 * GI))], has_state=1, **EMPTY_NODE, want_nominated=0),
    dict(ref="nominator_test.go:253 matched reservations", pod=[2000, 4 * GI], slots=[R4C8G, R2C4G], has_state=1,
         **EMPTY_NODE, want_nominated=1),
]

# BeforePreFilter's restore (transformer.go:49-346): one node, its bound pods (cpu cores, memory GiB; "reserve" = a
# reservation's reserve pod) and reservation slots, the pod's owner-group mask / required-affinity flag, and the
# restored node (transformer_test.go assertions).  Owner groups: the caller decodes ReservationInfo.Match into the pod's
# mask.  (ABI 12) A required reservation affinity travels as predicates: "rsv_affinity" = the pod's
# reservationSelector / ReservationSelectorTerms, "node_labels" / "slot_labels" = matchReservation's fakeNode
# (transformer.go:348-372), compiled through PredicateTable by the test.
AFF_A_TRUE = {"terms": [{"matchExpressions": [{"key": "reservation-a", "operator": "In", "values": ["true"]}]}]}
AFF_A_FALSE = {"terms": [{"matchExpressions": [{"key": "reservation-a", "operator": "In", "values": ["false"]}]}]}
AFF_TYPE = {"terms": [{"matchExpressions": [{"key": "reservation-type", "operator": "In",
                                             "values": ["reservation-test"]}]}]}
RESTORE = [
    dict(ref="transformer_test.go:41 TestRestoreReservation", node=[32, 64],
         pods=[[4, 8, 0], [8, 16, 0], [12, 24, 1], [8, 16, 1], [4, 8, 0]],
         slots=[dict(slot(12, 24, allocated=(4000, 8 * GI)), owner=1, assigned=1, allocate_once=0),
                dict(slot(8, 16), owner=0, allocate_once=1)],
         mask=1, affinity=0,
         want=dict(has_state=1, matched=0b10, requested_cpu=24000, requested_mem=48 * GI, nonzero_cpu=24000,
                   nonzero_mem=48 * GI, num_pods=4, pod_requested_cpu=32000, pod_requested_mem=64 * GI)),
    dict(ref="transformer_test.go:510 pod has no reservation affinity", node=[32, 64], pods=[[8, 16, 1]],
         slots=[dict(slot(8, 16), owner=0, allocate_once=1)], mask=1, affinity=0,
         node_labels={"test": "true"}, slot_labels=[{"reservation-a": "true"}], want=dict(has_state=1, matched=1)),
    dict(ref="transformer_test.go:514 pod has reservation affinity and matched", node=[32, 64], pods=[[8, 16, 1]],
         slots=[dict(slot(8, 16), owner=0, allocate_once=1)], mask=1, affinity=1, rsv_affinity=AFF_A_TRUE,
         node_labels={"test": "true"}, slot_labels=[{"reservation-a": "true"}], want=dict(has_state=1, matched=1)),
    dict(ref="transformer_test.go:533 pod has reservation affinity but failed to match", node=[32, 64],
         pods=[[8, 16, 1]], slots=[dict(slot(8, 16), owner=0, allocate_once=1)], mask=1, affinity=1,
         rsv_affinity=AFF_A_FALSE, node_labels={"test": "true"}, slot_labels=[{"reservation-a": "true"}],
         want=dict(has_state=0, matched=0)),
    # Test_matchReservation (transformer_test.go:348-442) through the restore: the pod matches the owners; with the
    # affinity term on the reservation's own label it still matches (both "want: true")
    dict(ref="transformer_test.go:356 only match reservation owners", node=[32, 64], pods=[[8, 16, 1]],
         slots=[dict(slot(8, 16), owner=0, allocate_once=0)], mask=1, affinity=0,
         slot_labels=[{}], want=dict(has_state=1, matched=1)),
    dict(ref="transformer_test.go:379 match reservation owners and match reservation affinity", node=[32, 64],
         pods=[[8, 16, 1]], slots=[dict(slot(8, 16), owner=0, allocate_once=0)], mask=1, affinity=1,
         rsv_affinity=AFF_TYPE, slot_labels=[{"reservation-type": "reservation-test"}],
         want=dict(has_state=1, matched=1)),
]

if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reservation.json")
    with open(out, "w") as f:
        json.dump({"source": "hhyasdf/koordinator pkg/scheduler/plugins/reservation tests", "cases": CASES,
                   "restore": RESTORE,
                   "skipped": []},
                  f, indent=1)
    print(f"wrote {len(CASES)} cases to {out}")
