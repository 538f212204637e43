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
    {"source": "plugin_test.go:1670-1835", "name": "allocate from reserved / remaining of reserved are zero",
     "reason": "reservations holding GPU devices (device reservation restore is not accelerated)"},
    {"source": "scoring_test.go:1115-1127", "name": "scoreDevice completely used",
     "reason": "free 0: the pod does not fit, so Score is never called for it in a scheduling cycle"},
    {"source": "scoring_test.go:579-1090", "name": "TestScoreReservation",
     "reason": "reservations holding GPU devices (not accelerated)"},
]


def main():
    with open(OUT, "w") as f:
        json.dump({"generator": "tests/golden/make_golden_ds.py", "cases": CASES, "skipped": SKIPPED}, f, indent=1)
    print(f"wrote {len(CASES)} cases to {OUT}")


if __name__ == "__main__":
    main()
