"""Writes tests/golden/numa_reservation.json: NodeNUMAResource with reservations that hold cpusets (round 6, SURVEY §8
A15) — hand transcriptions of the reference's own tests (paths under /root/reference/pkg/scheduler/plugins/
nodenumaresource/), with source lines.

* restore        plugin_test.go TestRestoreReservation (:1327-1431): the reservation holds cpus 6-9 on
                 buildCPUTopologyForTest(1, 2, 8, 2); its AssignedPods hold {6,7} (then also {8,9}); the restored
                 reservedCPUs are {8,9} (then the state is nil: nothing reserved).
* available      node_allocation_test.go Test_cpuAllocation_getAvailableCPUs_with_preferred_cpus (:151-169): cpus 0-4
                 allocated (RefCount 1) on buildCPUTopologyForTest(2, 1, 4, 2), maxRefCount 1; with preferred {1,2}
                 their RefCount drops to 0 and they are available.
* take_preferred cpu_accumulator_test.go TestTakePreferredCPUs (:759-776) on buildCPUTopologyForTest(2, 1, 16, 2),
                 SpreadByPCPUs, NUMAMostAllocated.
* reserve        plugin_test.go TestPlugin_Reserve "succeed allocate from reservation reserved cpus" (:1049-1062,
                 harness :1064-1149): the reservation holds cpus 4-10 (addCPUs, RefCount 1), the pod is nominated into
                 it and its restore state reserves those cpus; 4 FullPCPUs → {4,5,6,7}.
Run: python tests/golden/make_golden_numa_rsv.py   (rewrites the JSON next to this script)
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = "pkg/scheduler/plugins/nodenumaresource/"


def rng(a, b):
    return list(range(a, b + 1))


DOC = {
    "source": SRC,
    "restore": [
        {"name": "assigned pod A", "source_line": SRC + "plugin_test.go:1424-1426", "topo": [1, 2, 8, 2],
         "reservation_cpus": [6, 7, 8, 9], "assigned_cpus": [[6, 7]], "want": [8, 9]},
        {"name": "assigned pods A and B", "source_line": SRC + "plugin_test.go:1428-1431", "topo": [1, 2, 8, 2],
         "reservation_cpus": [6, 7, 8, 9], "assigned_cpus": [[6, 7], [8, 9]], "want": []},
    ],
    "available": [
        {"name": "no preferred", "source_line": SRC + "node_allocation_test.go:161-164", "topo": [2, 1, 4, 2],
         "allocated": rng(0, 4), "preferred": [], "want": rng(5, 15)},
        {"name": "preferred 1,2", "source_line": SRC + "node_allocation_test.go:166-168", "topo": [2, 1, 4, 2],
         "allocated": rng(0, 4), "preferred": [1, 2], "want": [1, 2] + rng(5, 15)},
    ],
    "take_preferred": [
        {"name": "no preferred", "source_line": SRC + "cpu_accumulator_test.go:762-764", "topo": [2, 1, 16, 2],
         "available": rng(0, 63), "preferred": [], "need": 2, "want": [0, 2]},
        {"name": "preferred 0,2", "source_line": SRC + "cpu_accumulator_test.go:766-768", "topo": [2, 1, 16, 2],
         "available": rng(0, 63), "preferred": [0, 2], "need": 2, "want": [0, 2]},
        {"name": "rest without preferred", "source_line": SRC + "cpu_accumulator_test.go:770-772",
         "topo": [2, 1, 16, 2], "available": [c for c in rng(0, 63) if c not in (0, 2)], "preferred": [], "need": 2,
         "want": [1, 3]},
        {"name": "preferred 11,13,15,17", "source_line": SRC + "cpu_accumulator_test.go:773-776",
         "topo": [2, 1, 16, 2], "available": rng(0, 63), "preferred": [11, 13, 15, 17], "need": 2, "want": [11, 13]},
    ],
    "take_preferred_policy": {"bind": "SpreadByPCPUs", "strategy": "MostAllocated"},
    "reserve": [
        {"name": "succeed allocate from reservation reserved cpus", "source_line": SRC + "plugin_test.go:1049-1062",
         "topo": [2, 1, 4, 2], "reservation_cpus": rng(4, 10), "assigned_cpus": [], "cpus": 4,
         "preferred": "FullPCPUs", "want": [4, 5, 6, 7]},
    ],
}

if __name__ == "__main__":
    with open(os.path.join(HERE, "numa_reservation.json"), "w") as f:
        json.dump(DOC, f, indent=1)
        f.write("\n")
