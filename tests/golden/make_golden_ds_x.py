"""(r6, ABI 17) Golden vectors for DeviceShare's RDMA / FPGA device types (the default handler), hand-transcribed from the
reference's own tests (paths under /root/reference/pkg/scheduler/plugins/deviceshare); writes deviceshare_x.json.

Each case is the node the test builds (its deviceTotal / deviceUsed per type and minor; the GPU memory in bytes) and the
pod's converted device request, with the test's want:
  kind "filter":  Test_Plugin_Filter (plugin_test.go:869-1445) — want_filter (nil status = true)
  kind "reserve": Test_Plugin_Reserve (plugin_test.go:2049-2760) — want_minors per type, or null for an Unschedulable
                  status; every chosen minor receives the per-instance request
  kind "score":   TestScore "requested multiple resources on the remaining resources of the node"
                  (scoring_test.go:274-351) — want_score (the sum over the requested types, default weights)
  kind "preempt": Test_allocateRDMA (device_allocator_test.go:2259-2340) — the minors a pod holds become preemptible;
                  rebuilt as a victim holding them (want_filter without / with the victim, want_minors after it left)
Pod requests use the pod-level resource names (koordinator.sh/gpu-core, -memory-ratio, koordinator.sh/rdma, fpga).
TEST INFRASTRUCTURE (run: python tests/golden/make_golden_ds_x.py)."""
import json
import os

GI = 1 << 30
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "deviceshare_x.json")


def gpu(minor, total=(100, 100, 16 * GI), used=(0, 0, 0)):
    return {"minor": minor, "healthy": True, "total": {"core": total[0], "ratio": total[1], "memory": total[2]},
            "used": {"core": used[0], "ratio": used[1], "memory": used[2]}}


def dev(minor, total=100, used=0):
    return {"minor": minor, "healthy": True, "total": total, "used": used}


GPU_100 = {"koordinator.sh/gpu-core": 100, "koordinator.sh/gpu-memory-ratio": 100}

CASES = [
    # ---- Test_Plugin_Filter -------------------------------------------------------------------------------------
    {"name": "filter insufficient device resource 3", "source": "plugin_test.go:985-1071", "kind": "filter",
     "node": {"gpus": [gpu(0, used=(25, 25, 4 * GI))], "fpga": [dev(0)]},
     "pod": {**GPU_100, "koordinator.sh/fpga": 100}, "want_filter": False},
    {"name": "filter insufficient device resource 4", "source": "plugin_test.go:1072-1164", "kind": "filter",
     "node": {"gpus": [gpu(0, used=(25, 25, 4 * GI))], "fpga": [dev(0, used=50)]},
     "pod": {**GPU_100, "koordinator.sh/fpga": 100}, "want_filter": False},
    {"name": "filter sufficient device resource 1", "source": "plugin_test.go:1165-1213", "kind": "filter",
     "node": {"fpga": [dev(0)]}, "pod": {"koordinator.sh/fpga": 100}, "want_filter": True},
    {"name": "filter sufficient device resource 2", "source": "plugin_test.go:1214-1283", "kind": "filter",
     "node": {"fpga": [dev(0, used=25), dev(1)]}, "pod": {"koordinator.sh/fpga": 100}, "want_filter": True},
    {"name": "filter sufficient device resource 3", "source": "plugin_test.go:1284-1360", "kind": "filter",
     "node": {"gpus": [gpu(0)], "fpga": [dev(0)]}, "pod": dict(GPU_100), "want_filter": True},
    # ---- Test_Plugin_Reserve ------------------------------------------------------------------------------------
    {"name": "reserve insufficient device resource 4", "source": "plugin_test.go:2283-2338", "kind": "reserve",
     "node": {"rdma": [dev(0, used=50)]}, "pod": {"koordinator.sh/rdma": 100}, "want_minors": None},
    {"name": "reserve insufficient device resource 5", "source": "plugin_test.go:2339-2410", "kind": "reserve",
     "node": {"rdma": [dev(0)], "fpga": [dev(0)]}, "pod": {"koordinator.sh/rdma": 200, "koordinator.sh/fpga": 200},
     "want_minors": None},
    {"name": "reserve sufficient device resource 1", "source": "plugin_test.go:2411-2537", "kind": "reserve",
     "node": {"gpus": [gpu(0)], "rdma": [dev(0)], "fpga": [dev(0)]},
     "pod": {**GPU_100, "koordinator.sh/rdma": 100, "koordinator.sh/fpga": 100},
     "want_minors": {"gpu": [0], "rdma": [0], "fpga": [0]},
     "want_instance": {"gpu": {"core": 100, "ratio": 100, "memory": 16 * GI}, "rdma": 100, "fpga": 100}},
    {"name": "reserve sufficient device resource 2", "source": "plugin_test.go:2538-2723", "kind": "reserve",
     "node": {"gpus": [gpu(0), gpu(1)], "rdma": [dev(0), dev(1)], "fpga": [dev(0), dev(1)]},
     "pod": {"koordinator.sh/gpu-core": 200, "koordinator.sh/gpu-memory-ratio": 200, "koordinator.sh/rdma": 200,
             "koordinator.sh/fpga": 200},
     "want_minors": {"gpu": [0, 1], "rdma": [0, 1], "fpga": [0, 1]},
     "want_instance": {"gpu": {"core": 100, "ratio": 100, "memory": 16 * GI}, "rdma": 100, "fpga": 100}},
    # ---- TestScore ----------------------------------------------------------------------------------------------
    {"name": "score requested multiple resources on the remaining resources of the node",
     "source": "scoring_test.go:274-351", "kind": "score",
     "node": {"gpus": [gpu(0, total=(1000, 1000, 160 * GI), used=(25, 25, 4 * GI))], "rdma": [dev(0, 1000, 50)]},
     "pod": {"koordinator.sh/gpu-core": 50, "koordinator.sh/gpu-memory-ratio": 50, "koordinator.sh/rdma": 25},
     "want_score": 184},
    # ---- Test_allocateRDMA: minors 1 and 2 fully used by one pod, preemptible; a 50 % RDMA request -------------------
    {"name": "allocate RDMA from preemptible", "source": "device_allocator_test.go:2259-2340", "kind": "preempt",
     "node": {"rdma": [dev(1, used=100), dev(2, used=100)]},
     "victim": {"koordinator.sh/rdma": 200}, "victim_minors": {"rdma": [1, 2]},
     "pod": {"koordinator.sh/rdma": 50}, "want_filter_without": False, "want_filter_with": True,
     "want_minors": {"rdma": [1]}},
]


if __name__ == "__main__":
    with open(OUT, "w") as f:
        json.dump({"source": "pkg/scheduler/plugins/deviceshare (see make_golden_ds_x.py)", "cases": CASES}, f, indent=1)
    print(f"wrote {len(CASES)} cases to {OUT}")
