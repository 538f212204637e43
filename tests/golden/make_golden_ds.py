#!/usr/bin/env python3
"""Writes tests/golden/deviceshare.json: DeviceShare (GPU) golden vectors hand-transcribed from the reference's own
table-driven tests (paths under /root/reference/pkg/scheduler/plugins/deviceshare).  Every case carries its
source file:line.  Device maps the tests set directly (deviceFree / deviceUsed) are restated as total + used
(resetDeviceFree: free = total - used, device_cache.go:157-174).  Quantities: gpu-core / gpu-memory-ratio in
percent, gpu-memory in bytes.  Run: python tests/golden/make_golden_ds.py
"""
import json
import os

GI = 1 << 30
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "deviceshare.json")


def gpu(minor, core=100, ratio=100, mem=16 * GI, used=(0, 0, 0), healthy=True):
    return {"minor": minor, "healthy": healthy, "total": {"core": core, "ratio": ratio, "memory": mem},
            "used": {"core": used[0], "ratio": used[1], "memory": used[2]}}


CASES = [
    # ---- scoring_test.go TestScore (:40) — GPU cases; Score runs after Filter in a real cycle ----
    {"kind": "score", "name": "skip_true", "source": "scoring_test.go:77-81",
     "node": {"has_device": True, "gpus": [gpu(0)]}, "pod": {}, "strategy": "LeastAllocated",
     "want_filter": True, "want_score": 0},
    {"kind": "score", "name": "no_device_resources", "source": "scoring_test.go:96-114",
     "node": {"has_device": True, "gpus": []},
     "pod": {"koordinator.sh/gpu-core": 100, "koordinator.sh/gpu-memory-ratio": 100}, "strategy": "LeastAllocated",
     "want_filter": False, "want_score": 0},  # Score: UnschedulableAndUnresolvable "Insufficient gpu devices"
    {"kind": "score", "name": "completely_idle_node", "source": "scoring_test.go:115-144",
     "node": {"has_device": True, "gpus": [gpu(0)]},
     "pod": {"koordinator.sh/gpu-core": 100, "koordinator.sh/gpu-memory-ratio": 100}, "strategy": "LeastAllocated",
     "want_filter": True, "want_score": 0},
    {"kind": "score", "name": "multiple_gpu_devices_completely_idle", "source": "scoring_test.go:145-183",
     "node": {"has_device": True, "gpus": [gpu(0), gpu(1)]},
     "pod": {"koordinator.sh/gpu-core": 50, "koordinator.sh/gpu-memory-ratio": 50}, "strategy": "LeastAllocated",
     "want_filter": True, "want_score": 75},
    {"kind": "score", "name": "remaining_device_resources", "source": "scoring_test.go:184-228",
     "node": {"has_device": True, "gpus": [gpu(0, used=(25, 25, 4 * GI))]},
     "pod": {"koordinator.sh/gpu-core": 50, "koordinator.sh/gpu-memory-ratio": 50}, "strategy": "LeastAllocated",
     "want_filter": True, "want_score": 25},
    {"kind": "score", "name": "remaining_device_resources_most_allocated", "source": "scoring_test.go:229-274",
     "node": {"has_device": True, "gpus": [gpu(0, used=(25, 25, 4 * GI))]},
     "pod": {"koordinator.sh/gpu-core": 50, "koordinator.sh/gpu-memory-ratio": 50}, "strategy": "MostAllocated",
     "want_filter": True, "want_score": 75},
    # ---- plugin_test.go Test_Plugin_Filter (:869) — the GPU cases (a node = deviceTotal + deviceUsed; free =
    # total - used as resetDeviceFree keeps it) ----
    {"kind": "filter", "name": "filter_skip", "source": "plugin_test.go:890-893",
     "node": {"has_device": True, "gpus": [gpu(0)]}, "pod": {}, "want_filter": True},
    {"kind": "filter", "name": "filter_missing_nodecache", "source": "plugin_test.go:895-900",
     "node": {"has_device": False, "gpus": []}, "pod": {}, "want_filter": True},
    {"kind": "filter", "name": "filter_insufficient_1", "source": "plugin_test.go:902-919",
     "node": {"has_device": True, "gpus": []},
     "pod": {"koordinator.sh/gpu-core": 100, "koordinator.sh/gpu-memory-ratio": 100}, "want_filter": False},
    {"kind": "filter", "name": "filter_insufficient_2", "source": "plugin_test.go:921-983",
     "node": {"has_device": True, "gpus": [gpu(0, used=(25, 25, 4 * GI))]},
     "pod": {"koordinator.sh/gpu-core": 100, "koordinator.sh/gpu-memory-ratio": 100}, "want_filter": False},
    {"kind": "filter", "name": "filter_sufficient_4", "source": "plugin_test.go:1362-1445",
     "node": {"has_device": True, "gpus": [gpu(0, used=(75, 75, 12 * GI)), gpu(1)]},
     "pod": {"koordinator.sh/gpu-core": 100, "koordinator.sh/gpu-memory-ratio": 100}, "want_filter": True},
    {"kind": "filter", "name": "filter_sufficient_5", "source": "plugin_test.go:1447-1529",
     "node": {"has_device": True, "gpus": [gpu(0, used=(75, 75, 12 * GI)), gpu(1)]},
     "pod": {"koordinator.sh/gpu-memory-ratio": 100}, "want_filter": True},
    {"kind": "filter", "name": "filter_sufficient_6", "source": "plugin_test.go:1531-1593",
     "node": {"has_device": True, "gpus": [gpu(0, used=(75, 75, 12 * GI)), gpu(1)]},
     "pod": {"koordinator.sh/gpu-memory": 16 * GI}, "want_filter": True},
    # ---- scoring_test.go Test_resourceAllocationScorer_scoreDevice (:1092): scoreDevice over gpu-memory-ratio, as the
    # score of a one-GPU node (scoreNode over one minor = scoreDevice) for a pod asking only gpu-memory-ratio ----
    {"kind": "score", "name": "score_device_completely_idle", "source": "scoring_test.go:1102-1114",
     "node": {"has_device": True, "gpus": [gpu(0)]}, "pod": {"koordinator.sh/gpu-memory-ratio": 50},
     "strategy": "LeastAllocated", "want_filter": True, "want_score": 50},
    {"kind": "score", "name": "score_device_remaining", "source": "scoring_test.go:1128-1140",
     "node": {"has_device": True, "gpus": [gpu(0, used=(50, 50, 8 * GI))]},
     "pod": {"koordinator.sh/gpu-memory-ratio": 30}, "strategy": "LeastAllocated", "want_filter": True,
     "want_score": 20},
    {"kind": "score", "name": "score_device_remaining_most_allocated", "source": "scoring_test.go:1141-1153",
     "node": {"has_device": True, "gpus": [gpu(0, used=(50, 50, 8 * GI))]},
     "pod": {"koordinator.sh/gpu-memory-ratio": 30}, "strategy": "MostAllocated", "want_filter": True,
     "want_score": 80},
    # ---- device_allocator_test.go: minor selection of Allocate ----
    {"kind": "reserve", "name": "allocate_gpu_least_allocated_scorer", "source": "device_allocator_test.go:1924-2020",
     "node": {"has_device": True, "gpus": [gpu(1, mem=8 * GI, used=(50, 50, 4 * GI)),
                                           gpu(2, mem=8 * GI, used=(50, 50, 4 * GI)),
                                           gpu(3, mem=8 * GI), gpu(4, mem=8 * GI)]},
     "pod": {"koordinator.sh/gpu-core": 50, "koordinator.sh/gpu-memory-ratio": 50}, "strategy": "LeastAllocated",
     "want_minors": [3], "want_instance": {"core": 50, "ratio": 50, "memory": 4 * GI}},
    {"kind": "reserve", "name": "allocate_gpu_most_allocated_scorer", "source": "device_allocator_test.go:2022-2118",
     "node": {"has_device": True, "gpus": [gpu(1, mem=8 * GI), gpu(2, mem=8 * GI),
                                           gpu(3, mem=8 * GI, used=(50, 50, 4 * GI)),
                                           gpu(4, mem=8 * GI, used=(50, 50, 4 * GI))]},
     "pod": {"koordinator.sh/gpu-core": 50, "koordinator.sh/gpu-memory-ratio": 50}, "strategy": "MostAllocated",
     "want_minors": [3], "want_instance": {"core": 50, "ratio": 50, "memory": 4 * GI}},
    {"kind": "reserve", "name": "allocate_gpu_with_unhealthy_instance", "source": "device_allocator_test.go:2208-2257",
     "node": {"has_device": True, "gpus": [gpu(1, mem=8 * GI, healthy=False), gpu(2, mem=8 * GI)]},
     # podRequests there = {core 50, memory 4Gi, ratio 50}: the GPUCore|GPUMemory request after fillGPUTotalMem
     "pod": {"koordinator.sh/gpu-core": 50, "koordinator.sh/gpu-memory": 4 * GI}, "strategy": "",
     "want_minors": [2], "want_instance": {"core": 50, "ratio": 50, "memory": 4 * GI}},
    # ---- devicehandler_gpu_test.go Test_fillGPUTotalMem (:29) ----
    {"kind": "instance", "name": "fill_ratio_to_mem", "source": "devicehandler_gpu_test.go:38-56",
     "node": {"has_device": True, "gpus": [gpu(0, mem=32 * GI)]},
     "pod": {"koordinator.sh/gpu-core": 50, "koordinator.sh/gpu-memory-ratio": 50},
     "want": {"count": 1, "core": 50, "ratio": 50, "memory": 16 * GI}},
    {"kind": "instance", "name": "fill_mem_to_ratio", "source": "devicehandler_gpu_test.go:57-76",
     "node": {"has_device": True, "gpus": [gpu(0, mem=32 * GI)]},
     "pod": {"koordinator.sh/gpu-core": 50, "koordinator.sh/gpu-memory": 16 * GI},
     "want": {"count": 1, "core": 50, "ratio": 50, "memory": 16 * GI}},
    {"kind": "instance", "name": "fill_missing_total", "source": "devicehandler_gpu_test.go:76-90",
     "node": {"has_device": True, "gpus": [gpu(0, core=0, ratio=0, mem=0)]},
     "pod": {"koordinator.sh/gpu-core": 50, "koordinator.sh/gpu-memory-ratio": 50}, "want": None},
    # ---- utils_test.go memory conversions (:309, :317) ----
    {"kind": "ratio_to_bytes", "name": "memory_ratio_to_bytes", "source": "utils_test.go:309-315",
     "ratio": 50, "total": 64 * GI, "want": 32 * GI},
    {"kind": "bytes_to_ratio", "name": "memory_bytes_to_ratio", "source": "utils_test.go:317-323",
     "bytes": 32 * GI, "total": 64 * GI, "want": 50},
    # ---- utils_test.go TestValidateDeviceRequest (:29): GPU combinations (error = PreFilter rejects) ----
    {"kind": "validate", "name": "invalid_gpu_request_1", "source": "utils_test.go:43-50",
     "pod": {"koordinator.sh/gpu-core": 101}, "want_error": True},
    {"kind": "validate", "name": "invalid_gpu_request_2", "source": "utils_test.go:51-62",
     "pod": {"nvidia.com/gpu": 2, "koordinator.sh/gpu": 200, "koordinator.sh/gpu-core": 200,
             "koordinator.sh/gpu-memory": 32 * GI, "koordinator.sh/gpu-memory-ratio": 200}, "want_error": True},
    {"kind": "validate", "name": "invalid_gpu_request_3", "source": "utils_test.go:63-70",
     "pod": {"koordinator.sh/gpu": 101}, "want_error": True},
    {"kind": "validate", "name": "invalid_gpu_request_4", "source": "utils_test.go:71-79",
     "pod": {"koordinator.sh/gpu-core": 100, "koordinator.sh/gpu-memory-ratio": 101}, "want_error": True},
    {"kind": "validate", "name": "valid_nvidia_gpu", "source": "utils_test.go:80-87",
     "pod": {"nvidia.com/gpu": 2}, "want_error": False, "want_request": {"core": 200, "ratio": 200}},
    {"kind": "validate", "name": "valid_hygon_dcu", "source": "utils_test.go:88-95",
     "pod": {"dcu.com/gpu": 2}, "want_error": False, "want_request": {"core": 200, "ratio": 200}},
    {"kind": "validate", "name": "valid_koord_gpu", "source": "utils_test.go:96-103",
     "pod": {"koordinator.sh/gpu": 200}, "want_error": False, "want_request": {"core": 200, "ratio": 200}},
    {"kind": "validate", "name": "valid_core_memory", "source": "utils_test.go:104-112",
     "pod": {"koordinator.sh/gpu-core": 200, "koordinator.sh/gpu-memory": 64 * GI}, "want_error": False,
     "want_request": {"core": 200, "memory": 64 * GI}},
    {"kind": "validate", "name": "valid_core_ratio", "source": "utils_test.go:113-121",
     "pod": {"koordinator.sh/gpu-core": 200, "koordinator.sh/gpu-memory-ratio": 200}, "want_error": False,
     "want_request": {"core": 200, "ratio": 200}},
    {"kind": "validate", "name": "valid_ratio", "source": "utils_test.go:122-129",
     "pod": {"koordinator.sh/gpu-memory-ratio": 200}, "want_error": False, "want_request": {"ratio": 200}},
    {"kind": "validate", "name": "valid_memory", "source": "utils_test.go:130-137",
     "pod": {"koordinator.sh/gpu-memory": 64 * GI}, "want_error": False, "want_request": {"memory": 64 * GI}},
]



# ---- (ABI 13) reservations holding GPUs (reservation.go) ----
# A reservation slot: policy, the minors the reserve pod holds with its allocation per minor (allocatable: core, ratio,
# memory bytes) and the allocations of its assigned pods on those minors (allocated; absent = none).  The node's `used`
# includes the reserve pod's and the assigned pods' allocations, as nodeDevice.deviceUsed does.
def slot(policy="Default", alloc=None, allocated=None):
    return {"policy": policy, "alloc": alloc or {}, "allocated": allocated or {}}


HALF, QUARTER = (50, 50, 4 * GI), (25, 25, 2 * GI)


def two_8g(used0=(0, 0, 0), used1=(0, 0, 0)):
    return {"has_device": True, "gpus": [gpu(0, mem=8 * GI, used=used0), gpu(1, mem=8 * GI, used=used1)]}


HALF_POD = {"koordinator.sh/gpu-core": 50, "koordinator.sh/gpu-memory": 4 * GI}  # podRequestsHalfGPU
FULL8, FULL16 = (100, 100, 8 * GI), (100, 100, 16 * GI)

CASES += [
    # ---- reservation_test.go Test_Plugin_ReservationRestore (:38): mergeReservationAllocations of one matched slot ----
    {"kind": "rsv_restore", "name": "restore_matched_with_assigned_pod", "source": "reservation_test.go:38-222",
     "slot": slot(alloc={1: FULL8}, allocated={1: HALF}),
     "want": {"mat_alloc": {1: FULL8}, "mat_allocd": {1: HALF}, "remained": {1: HALF}}},
    # ---- reservation_test.go Test_tryAllocateFromReservation (:224): one matched slot, no scorer; node = 2 GPUs of
    # 100 / 8Gi / 100 with the case's deviceUsed ----
    {"kind": "rsv_try", "name": "no_matched_reservations", "source": "reservation_test.go:308-319",
     "node": two_8g(), "slot": None, "pod": HALF_POD, "required": False, "want_minors": None,
     "want_unschedulable": False},
    {"kind": "rsv_try", "name": "default_policy", "source": "reservation_test.go:321-352",
     "node": two_8g(), "slot": slot(alloc={0: QUARTER}), "pod": HALF_POD, "required": False, "want_minors": [0],
     "want_unschedulable": False},
    # the test's hand-built restore state carries remained = 50 % with allocated = 25 %; RestoreReservation computes
    # remained = allocatable − allocated (25 %), which gives the same allocation (preemptible 50 % vs 75 % of a minor
    # used 50 %: free 100 % either way)
    {"kind": "rsv_try", "name": "default_policy_required", "source": "reservation_test.go:354-396",
     "node": two_8g(used0=HALF), "slot": slot(alloc={0: HALF}, allocated={0: QUARTER}), "pod": HALF_POD,
     "required": True, "want_minors": [0], "want_unschedulable": False},
    {"kind": "rsv_try", "name": "default_policy_required_reservation_empty", "source": "reservation_test.go:398-440",
     "node": two_8g(used0=(150, 150, 12 * GI)), "slot": slot(alloc={0: HALF}, allocated={0: HALF}), "pod": HALF_POD,
     "required": True, "want_minors": [1], "want_unschedulable": False},
    {"kind": "rsv_try", "name": "aligned_policy", "source": "reservation_test.go:442-486",
     "node": two_8g(used0=FULL8, used1=FULL8), "slot": slot("Aligned", alloc={0: HALF}), "pod": HALF_POD,
     "required": False, "want_minors": [0], "want_unschedulable": False},
    {"kind": "rsv_try", "name": "aligned_bigger_request_no_node_remaining", "source": "reservation_test.go:488-527",
     "node": two_8g(used0=FULL8, used1=FULL8), "slot": slot("Aligned", alloc={0: HALF}),
     "pod": {"koordinator.sh/gpu-core": 60, "koordinator.sh/gpu-memory": 5 * GI}, "required": True,
     "want_minors": None, "want_unschedulable": True},
    {"kind": "rsv_try", "name": "aligned_remaining_little", "source": "reservation_test.go:529-570",
     "node": two_8g(used0=(125, 125, 10 * GI), used1=FULL8), "slot": slot("Aligned", alloc={0: HALF},
                                                                          allocated={0: QUARTER}),
     "pod": {"koordinator.sh/gpu-core": 30, "koordinator.sh/gpu-memory": 1 * GI}, "required": True,
     "want_minors": None, "want_unschedulable": True},
    {"kind": "rsv_try", "name": "restricted_policy", "source": "reservation_test.go:572-616",
     "node": two_8g(used0=FULL8, used1=FULL8), "slot": slot("Restricted", alloc={0: HALF}), "pod": HALF_POD,
     "required": False, "want_minors": [0], "want_unschedulable": False},
    {"kind": "rsv_try", "name": "restricted_node_remains_reservation_not", "source": "reservation_test.go:618-654",
     "node": two_8g(used0=(75, 75, 6 * GI), used1=FULL8), "slot": slot("Restricted", alloc={0: HALF},
                                                                       allocated={0: QUARTER}),
     "pod": HALF_POD, "required": True, "want_minors": None, "want_unschedulable": True},
    # ---- plugin_test.go Test_Plugin_Filter (:869) with a matched reservation (no reservation affinity) ----
    {"kind": "rsv_filter", "name": "filter_allocate_from_reserved", "source": "plugin_test.go:1670-1737",
     "node": {"has_device": True, "gpus": [gpu(0, used=FULL16)]}, "slot": slot(alloc={0: FULL16}),
     "pod": {"koordinator.sh/gpu-core": 100, "koordinator.sh/gpu-memory-ratio": 100}, "want_filter": True},
    {"kind": "rsv_filter", "name": "filter_reserved_remaining_zero", "source": "plugin_test.go:1739-1835",
     "node": {"has_device": True, "gpus": [gpu(0, used=FULL16), gpu(1)]}, "slot": slot(alloc={0: (0, 0, 0)}),
     "pod": {"koordinator.sh/gpu-core": 100, "koordinator.sh/gpu-memory-ratio": 100}, "want_filter": True},
    # ---- plugin_test.go Test_Plugin_FilterReservation (:1905): GPUs minor 1, 2 of 100 / 8Gi / 100; the reservation
    # holds minor 1; then a pod assigned to it takes minors 1 and 2 (only minor 1 counts as its allocated) ----
    {"kind": "rsv_filter_reservation", "name": "filter_reservation_free", "source": "plugin_test.go:1935-2006",
     "node": {"has_device": True, "gpus": [gpu(1, mem=8 * GI, used=FULL8), gpu(2, mem=8 * GI)]},
     "slot": slot(alloc={1: FULL8}), "pod": {"koordinator.sh/gpu": 100}, "want_filter": True},
    {"kind": "rsv_filter_reservation", "name": "filter_reservation_exhausted", "source": "plugin_test.go:2008-2046",
     "node": {"has_device": True, "gpus": [gpu(1, mem=8 * GI, used=(200, 200, 16 * GI)),
                                           gpu(2, mem=8 * GI, used=FULL8)]},
     "slot": slot(alloc={1: FULL8}, allocated={1: FULL8}), "pod": {"koordinator.sh/gpu": 100}, "want_filter": False},
    # ---- plugin_test.go Test_Plugin_Reserve (:2049) "reserve from reservation": the nominated reservation ----
    {"kind": "rsv_reserve", "name": "reserve_from_reservation", "source": "plugin_test.go:2937-3009",
     "node": {"has_device": True, "gpus": [gpu(0, used=FULL16)]}, "slot": slot(alloc={0: FULL16}),
     "pod": {"koordinator.sh/gpu-core": 100, "koordinator.sh/gpu-memory-ratio": 100}, "strategy": "LeastAllocated",
     "want_minors": [0], "want_instance": {"core": 100, "ratio": 100, "memory": 16 * GI}},
    # ---- scoring_test.go TestScoreReservation (:579): one GPU of 100 / 16Gi / 100, used = deviceUsed + the reserve
    # pod's allocation (updatePod); pod gpu-core 50 + gpu-memory-ratio 50 ----
    {"kind": "rsv_score", "name": "score_default_least", "source": "scoring_test.go:647-679",
     "node": {"has_device": True, "gpus": [gpu(0, used=(75, 75, 16 * GI))]}, "slot": slot(alloc={0: (50, 50, 12 * GI)}),
     "pod": {"koordinator.sh/gpu-core": 50, "koordinator.sh/gpu-memory-ratio": 50}, "strategy": "LeastAllocated",
     "want_score": 25},
    {"kind": "rsv_score", "name": "score_default_most", "source": "scoring_test.go:681-714",
     "node": {"has_device": True, "gpus": [gpu(0, used=(75, 75, 12 * GI))]}, "slot": slot(alloc={0: (50, 50, 8 * GI)}),
     "pod": {"koordinator.sh/gpu-core": 50, "koordinator.sh/gpu-memory-ratio": 50}, "strategy": "MostAllocated",
     "want_score": 75},
    {"kind": "rsv_score", "name": "score_aligned_least", "source": "scoring_test.go:716-749",
     "node": {"has_device": True, "gpus": [gpu(0, used=(75, 75, 12 * GI))]},
     "slot": slot("Aligned", alloc={0: (50, 50, 8 * GI)}),
     "pod": {"koordinator.sh/gpu-core": 50, "koordinator.sh/gpu-memory-ratio": 50}, "strategy": "LeastAllocated",
     "want_score": 25},
    {"kind": "rsv_score", "name": "score_aligned_most", "source": "scoring_test.go:751-784",
     "node": {"has_device": True, "gpus": [gpu(0, used=(75, 75, 12 * GI))]},
     "slot": slot("Aligned", alloc={0: (50, 50, 8 * GI)}),
     "pod": {"koordinator.sh/gpu-core": 50, "koordinator.sh/gpu-memory-ratio": 50}, "strategy": "MostAllocated",
     "want_score": 75},
    {"kind": "rsv_score", "name": "score_restricted_least", "source": "scoring_test.go:786-819",
     "node": {"has_device": True, "gpus": [gpu(0, used=(50, 50, 8 * GI))]},
     "slot": slot("Restricted", alloc={0: (50, 50, 8 * GI)}),
     "pod": {"koordinator.sh/gpu-core": 50, "koordinator.sh/gpu-memory-ratio": 50}, "strategy": "LeastAllocated",
     "want_score": 0},
    {"kind": "rsv_score", "name": "score_restricted_most", "source": "scoring_test.go:821-854",
     "node": {"has_device": True, "gpus": [gpu(0, used=(50, 50, 8 * GI))]},
     "slot": slot("Restricted", alloc={0: (50, 50, 8 * GI)}),
     "pod": {"koordinator.sh/gpu-core": 50, "koordinator.sh/gpu-memory-ratio": 50}, "strategy": "MostAllocated",
     "want_score": 100},
]

# Cases of those tables outside the accelerated scope (the engine refuses such pods / states with KG_E_UNSUPPORTED, so
# the Go path keeps them), with the reason:
SKIPPED = [
    {"source": "plugin_test.go:886-888", "name": "error missing preFilterState", "reason": "no preFilterState"},
    {"source": "plugin_test.go:985-1164", "name": "insufficient device resource 3 / 4",
     "reason": "FPGA requests (not accelerated)"},
    {"source": "plugin_test.go:1166-1360", "name": "sufficient device resource 1 / 2 / 3",
     "reason": "FPGA requests (not accelerated)"},
    {"source": "plugin_test.go:1595-1668", "name": "allocate from preemptible",
     "reason": "preemptible devices of a nominated preemption (preemption is out of scope)"},
    {"source": "scoring_test.go:1115-1127", "name": "scoreDevice completely used",
     "reason": "free 0: the pod does not fit, so Score is never called for it in a scheduling cycle"},
    {"source": "scoring_test.go:856-952", "name": "TestScoreReservation: aligned / restricted policy and preemptible",
     "reason": "preemptible devices of a nominated preemption (preemption is out of scope)"},
    {"source": "scoring_test.go:954-1001", "name": "TestScoreReservation: multi resources and MostAllocated",
     "reason": "RDMA requests (not accelerated)"},
    {"source": "plugin_test.go:2856-2935", "name": "Test_Plugin_Reserve: reserve from preemptible",
     "reason": "preemptible devices of a nominated preemption (preemption is out of scope)"},
]


def main():
    with open(OUT, "w") as f:
        json.dump({"generator": "tests/golden/make_golden_ds.py", "cases": CASES, "skipped": SKIPPED}, f, indent=1)
    print(f"wrote {len(CASES)} cases to {OUT}")


if __name__ == "__main__":
    main()
