#!/usr/bin/env python3
"""Writes tests/golden/elasticquota.json: ElasticQuota PreFilter golden vectors hand-transcribed from the reference's
tests (/root/reference/pkg/scheduler/plugins/elasticquota/plugin_test.go), each with its source line.

Units: cpu in milli (CPU(n) = n cores), memory in bytes (Mem(n) = n bytes, MakeResourceList, controller_test.go:550-558).
The tests also carry nvidia.com/gpu; that dimension passes in every case (pod 1 ≤ runtime 10, or no gpu key in the
runtime, which quotav1.LessThanOrEqual then does not compare) and is dropped here.  Runtimes the reference computes
(TestPlugin_Prefilter_QuotaNonPreempt) are taken from the expected status messages, or — where a message does not
print it — restated as the single quota's request (Σ pod requests incl. the pending pod) capped by max and the
cluster total.  Run: python tests/golden/make_golden_quota.py
"""
import json
import os

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "elasticquota.json")


def rl(cpu=None, mem=None):
    d = {}
    if cpu is not None:
        d["cpu"] = cpu * 1000
    if mem is not None:
        d["memory"] = mem
    return d


CASES = [
    {"name": "default", "source": "plugin_test.go:613-627",
     "quota": {"used_limit": rl(0, 20)}, "pod": rl(1, 2), "non_preemptible": False, "want": "Unschedulable"},
    {"name": "used_dimension_larger_than_runtime_value_enough", "source": "plugin_test.go:628-639",
     "quota": {"used_limit": rl(10, 20)}, "pod": rl(1, 2), "non_preemptible": False, "want": "Success"},
    {"name": "value_not_enough", "source": "plugin_test.go:640-655",
     "quota": {"used_limit": rl(1, 2)}, "pod": rl(1, 3), "non_preemptible": False, "want": "Unschedulable"},
    {"name": "runtime_not_enough_but_disable_runtime", "source": "plugin_test.go:668-681",
     # EnableRuntimeQuota = false → usedLimit = max {cpu 1, mem 3}
     "quota": {"used_limit": rl(1, 3)}, "pod": rl(1, 3), "non_preemptible": False, "want": "Success"},
    {"name": "nonpreempt_default", "source": "plugin_test.go:779-800",
     # init pods (cpu, mem): (2,1) (1,1) (1,1) → used (4,3); request incl. the pod (6,5) ≤ max (10,10), total (10,10)
     "quota": {"used": rl(4, 3), "used_limit": rl(6, 5), "min": rl(5, 5), "non_preemptible_used": rl(0, 0)},
     "pod": rl(2, 2), "non_preemptible": True, "want": "Success"},
    {"name": "nonpreempt_used_larger_than_min", "source": "plugin_test.go:801-826",
     # used (6,3); non-preemptible used (4,2) (message); runtime: request (8,5) capped by total (8,5)
     "quota": {"used": rl(6, 3), "used_limit": rl(8, 5), "min": rl(5, 5), "non_preemptible_used": rl(4, 2)},
     "pod": rl(2, 2), "non_preemptible": True, "want": "Unschedulable"},
    {"name": "nonpreempt_will_not_be_evicted", "source": "plugin_test.go:827-852",
     # message: runtime (7,5), used (6,4), pod (2,1)
     "quota": {"used": rl(6, 4), "used_limit": rl(7, 5), "min": rl(5, 5), "non_preemptible_used": rl(2, 2)},
     "pod": rl(2, 1), "non_preemptible": True, "want": "Unschedulable"},
]


def main():
    with open(OUT, "w") as f:
        json.dump({"generator": "tests/golden/make_golden_quota.py", "cases": CASES}, f, indent=1)
    print(f"wrote {len(CASES)} cases to {OUT}")


if __name__ == "__main__":
    main()
