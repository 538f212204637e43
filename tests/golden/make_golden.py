"""Writes the golden fixtures under tests/golden/ — hand transcriptions of the reference's own table-driven tests.

The reference (Go) cannot be built or imported here, so each case below is the input and the
expected output of one reference test case, copied by hand, with the source file:line it comes from
(paths under /root/reference).  Quantities stay in k8s string form; tests convert them with
koordinator_amd.quantity exactly like resource.MustParse + MilliValue/Value.

Conventions for the LoadAware cases (load_aware_test.go harness :806-908 for Filter, :1754-1850 for Score):
* node allocatable cpu 96 / memory 512Gi (:844-847, :1783-1786);
* "update_age_s" = time.Now() - NodeMetric.Status.UpdateTime (0 for time.Now(), 180 for Add(-180s));
* Filter harness sets FilterExpiredNodeMetrics=false (:807); Score harness keeps the defaults (expiration 180s);
* a nil test pod is &corev1.Pod{} (:573-576), whose default priority class is koord-batch (BestEffort → BE,
  apis/extension/priority_utils.go:26-48 + qos_utils.go);
* scope "core" = restated and accelerated now (aggregated percentile usages and the PodsMetric-based estimation of
  assigned pods included); scope "next" = kept for completeness, skipped with a reason by the tests (none left);
* an assigned pod's "name" matches NodeMetric.Status.PodsMetric entries by namespace/name; its timestamp is taken
  before the metric's UpdateTime (the Go literal evaluates assignedPod first), so age 0 = 1 ns before the update;
* "report_interval_s" = NodeMetric.Spec.CollectPolicy.ReportIntervalSeconds.

Run: python tests/golden/make_golden.py   (rewrites the JSON files next to this script)
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = "pkg/scheduler/plugins/loadaware/load_aware_test.go"
NODE = {"cpu": "96", "memory": "512Gi"}
G = {"cpu": "16", "memory": "32Gi"}  # the 16 core / 32Gi guaranteed container used across TestScore

FILTER_CASES = [
    dict(name="filter normal usage", line=277, metric=dict(update_age_s=0, node_usage={"cpu": "60", "memory": "256Gi"}),
         want="Success"),
    dict(name="filter node missing NodeMetrics", line=305, metric=None, want="Success"),
    dict(name="filter exceed cpu usage", line=310, metric=dict(update_age_s=0, node_usage={"cpu": "70", "memory": "256Gi"}),
         want="Unschedulable"),
    dict(name="filter exceed p95 cpu usage", line=338,
         args=dict(aggregated=dict(usage_thresholds={"cpu": 60}, type="p95", duration="5m")),
         metric=dict(update_age_s=0, node_usage={"cpu": "30", "memory": "100Gi"},
                     aggregated=[dict(duration="5m", p95={"cpu": "70", "memory": "256Gi"})]),
         want="Unschedulable"),
    dict(name="filter exceed memory usage", line=386, metric=dict(update_age_s=0, node_usage={"cpu": "30", "memory": "500Gi"}),
         want="Unschedulable"),
    dict(name="filter exceed memory usage by custom usage thresholds", line=414,
         custom_usage_thresholds={"memory": 60},
         metric=dict(update_age_s=0, node_usage={"cpu": "30", "memory": "316Gi"}), want="Unschedulable"),
    dict(name="filter exceed p95 cpu usage by custom usage", line=445,
         custom_aggregated=dict(usage_thresholds={"cpu": 60}, type="p95", duration="5m"),
         metric=dict(update_age_s=0, node_usage={"cpu": "30", "memory": "100Gi"},
                     aggregated=[dict(duration="5m", p95={"cpu": "70", "memory": "256Gi"})]),
         want="Unschedulable"),
    dict(name="disable filter exceed memory usage", line=493, args=dict(usage_thresholds={"memory": 0}),
         metric=dict(update_age_s=0, node_usage={"cpu": "30", "memory": "500Gi"}), want="Success"),
    dict(name="prod usage filter is not enabled by default", line=524,
         args=dict(usage_thresholds={"cpu": 100, "memory": 100}),
         metric=dict(update_age_s=0, node_usage={"cpu": "63", "memory": "500Gi"}, pods_metric_count=2,
                     prod_pods_usage={"cpu": "63", "memory": "500Gi"}),
         want="Success"),
    dict(name="filter prod cpu usage", line=582,
         args=dict(usage_thresholds={"cpu": 100, "memory": 100}, prod_usage_thresholds={"cpu": 50, "memory": 100}),
         metric=dict(update_age_s=0, node_usage={"cpu": "63", "memory": "500Gi"}, pods_metric_count=2,
                     prod_pods_usage={"cpu": "63", "memory": "500Gi"}),
         pod=dict(priority="koord-prod"), want="Unschedulable"),
    dict(name="filter prod memory usage", line=645,
         args=dict(usage_thresholds={"cpu": 100, "memory": 100}, prod_usage_thresholds={"cpu": 100, "memory": 50}),
         metric=dict(update_age_s=0, node_usage={"cpu": "63", "memory": "500Gi"}, pods_metric_count=2,
                     prod_pods_usage={"cpu": "63", "memory": "500Gi"}),
         pod=dict(priority="koord-prod"), want="Unschedulable"),
    dict(name="filter prod memory usage with custom usage configuration", line=708,
         args=dict(usage_thresholds={"cpu": 100, "memory": 100}, prod_usage_thresholds={"cpu": 100, "memory": 100}),
         custom_prod_usage_thresholds={"cpu": 100, "memory": 50},
         metric=dict(update_age_s=0, node_usage={"cpu": "63", "memory": "500Gi"}, pods_metric_count=2,
                     prod_pods_usage={"cpu": "63", "memory": "500Gi"}),
         pod=dict(priority="koord-prod"), want="Unschedulable"),
    dict(name="filter daemonset pod exceed cpu usage", line=775,
         metric=dict(update_age_s=0, node_usage={"cpu": "70", "memory": "256Gi"}),
         pod=dict(priority="koord-prod", daemonset=True), want="Success"),
]
# TestFilterExpiredNodeMetric (:141-259): default args (FilterExpiredNodeMetrics=true, 180s); node has no
# allocatable; pod &corev1.Pod{}.
EXPIRED_CASES = [
    dict(name="filter healthy nodeMetrics", line=148, metric=dict(update_age_s=0), want="Success"),
    dict(name="filter unhealthy nodeMetric with nil updateTime", line=167, metric=dict(update_age_s=None), want="Success"),
    dict(name="filter unhealthy nodeMetric with expired updateTime", line=181, metric=dict(update_age_s=180), want="Success"),
]

SCORE_CASES = [
    dict(name="score node with expired nodeMetric", line=926, pod=None, metric=dict(update_age_s=180), want=0),
    dict(name="score empty node", line=947, pod=dict(requests=G, limits=G), metric=dict(update_age_s=0), want=90),
    dict(name="score node missing NodeMetrics", line=991, pod=dict(requests=G, limits=G), metric=None, want=0),
    dict(name="score load node", line=1020, pod=dict(requests=G, limits=G),
         metric=dict(update_age_s=0, node_usage={"cpu": "32", "memory": "10Gi"}), want=72),
    dict(name="score load node with p95", line=1072, pod=dict(requests=G, limits=G),
         args=dict(score_aggregated=dict(type="p95", duration="5m")),
         metric=dict(update_age_s=0, node_usage={"cpu": "0", "memory": "0Gi"},
                     aggregated=[dict(duration="5m", p95={"cpu": "32", "memory": "10Gi"},
                                      p99={"cpu": "50", "memory": "70Gi"})]),
         want=72),
    dict(name="score load node with p95 but have not reported usage", line=1147,
         pod=dict(requests=G, limits=G), args=dict(score_aggregated=dict(type="p95", duration="5m")),
         metric=dict(update_age_s=0, node_usage={"cpu": "0", "memory": "0Gi"}), want=90),
    dict(name="score load node with p95 but have not reported usage and have assigned pods", line=1203,
         pod=dict(requests=G, limits=G), args=dict(score_aggregated=dict(type="p95", duration="5m")),
         assigned=[dict(name="assigned-pod-1", requests=G, limits=G, age_s=600)],
         metric=dict(update_age_s=0, report_interval_s=60, node_usage={"cpu": "0", "memory": "0Gi"},
                     pods_metric=[dict(name="assigned-pod-1", usage={"cpu": "1", "memory": "1Gi"})]),
         want=81),
    dict(name="score load node with just assigned pod", line=1300, pod=dict(requests=G, limits=G),
         assigned=[dict(requests=G, limits=G, age_s=0)],
         metric=dict(update_age_s=0, node_usage={"cpu": "32", "memory": "10Gi"}), want=63),
    dict(name="score load node with just assigned pod where after updateTime", line=1381, pod=dict(requests=G, limits=G),
         assigned=[dict(requests=G, limits=G, age_s=0)],
         metric=dict(update_age_s=10, node_usage={"cpu": "32", "memory": "10Gi"}), want=63),
    dict(name="score load node with just assigned pod where before updateTime", line=1462, pod=dict(requests=G, limits=G),
         assigned=[dict(requests=G, limits=G, age_s=10)],
         metric=dict(update_age_s=0, node_usage={"cpu": "32", "memory": "10Gi"}), want=63),
    dict(name="score batch Pod", line=1543,
         pod=dict(priority="koord-batch",
                  requests={"kubernetes.io/batch-cpu": "16000", "kubernetes.io/batch-memory": "32Gi"},
                  limits={"kubernetes.io/batch-cpu": "16000", "kubernetes.io/batch-memory": "32Gi"}),
         metric=dict(update_age_s=0), want=90),
    dict(name="score prod Pod", line=1588, args=dict(score_according_prod_usage=True),
         pod=dict(priority="koord-prod", requests={"cpu": "16000", "memory": "32Gi"},
                  limits={"cpu": "16000", "memory": "32Gi"}),
         assigned=[dict(name="assign-prod-pod-1", priority="koord-prod", requests=G, limits=G, age_s=0)],
         metric=dict(update_age_s=0, report_interval_s=60, pods_metric=[dict(name="assign-prod-pod-1", usage={"cpu": "30", "memory": "100Gi"})]),
         want=38),
    dict(name="score request less than limit", line=1676,
         pod=dict(requests={"cpu": "8", "memory": "16Gi"}, limits=G), metric=dict(update_age_s=0), want=88),
    dict(name="score empty pod", line=1720, pod=dict(), metric=dict(update_age_s=0), want=99),
]

EST = "pkg/scheduler/plugins/loadaware/estimator/default_estimator_test.go"
ESTIMATE_POD_CASES = [
    dict(name="estimate empty pod", line=41, pod=dict(), want={"cpu": 250, "memory": 209715200}),
    dict(name="estimate guaranteed pod", line=58, pod=dict(requests={"cpu": "4", "memory": "8Gi"},
                                                           limits={"cpu": "4", "memory": "8Gi"}),
         want={"cpu": 3400, "memory": 6012954214}),
    dict(name="estimate burstable pod", line=84, pod=dict(requests={"cpu": "4", "memory": "8Gi"},
                                                          limits={"cpu": "8", "memory": "8Gi"}),
         want={"cpu": 8000, "memory": 6012954214}),
    dict(name="estimate guaranteed pod and zoomed cpu factors", line=110, factors={"cpu": 110},
         pod=dict(requests={"cpu": "4", "memory": "8Gi"}, limits={"cpu": "4", "memory": "8Gi"}),
         want={"cpu": 4000, "memory": 6012954214}),
    dict(name="estimate guaranteed pod and zoomed memory factors", line=139, factors={"memory": 110},
         pod=dict(requests={"cpu": "4", "memory": "8Gi"}, limits={"cpu": "4", "memory": "8Gi"}),
         want={"cpu": 3400, "memory": 8589934592}),
    dict(name="estimate Batch pod", line=168,
         pod=dict(priority="koord-batch",
                  requests={"kubernetes.io/batch-cpu": "4000", "kubernetes.io/batch-memory": "8Gi"},
                  limits={"kubernetes.io/batch-cpu": "4000", "kubernetes.io/batch-memory": "8Gi"}),
         want={"cpu": 3400, "memory": 6012954214}),
    dict(name="estimate pod only has request", line=200, factors={"cpu": 80, "memory": 80},
         pod=dict(priority="koord-prod", requests={"cpu": "4", "memory": "8Gi"}),
         want={"cpu": 3200, "memory": 6871947674}),
]
ESTIMATE_NODE_CASES = [
    dict(name="estimate empty node", line=260, allocatable={"cpu": "32"}, raw=None, want={"cpu": "32"}),
    dict(name="estimate node with original allocatable", line=273, allocatable={"cpu": "32", "memory": "42Gi"},
         raw={"cpu": "28", "memory": "32Gi"}, want={"cpu": "28", "memory": "32Gi"}),
    dict(name="estimate node with original allocatable and sames", line=293, allocatable={"cpu": "32", "memory": "42Gi"},
         raw={"cpu": "32", "memory": "42Gi"}, want={"cpu": "32", "memory": "42Gi"}),
]


def _write(name, cases, source, extra=None):
    out = dict(source=source, generator="tests/golden/make_golden.py", cases=[])
    out.update(extra or {})
    for c in cases:
        c = dict(c)
        c["source_line"] = f"{source}:{c.pop('line')}"
        c.setdefault("scope", "core")
        out["cases"].append(c)
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
        f.write("\n")


def main():
    _write("loadaware_filter.json", FILTER_CASES, SRC, dict(node_allocatable=NODE, harness=f"{SRC}:806-908",
                                                            filter_expired_node_metrics=False))
    _write("loadaware_filter_expired.json", EXPIRED_CASES, SRC, dict(node_allocatable={}, harness=f"{SRC}:141-259",
                                                                      filter_expired_node_metrics=True))
    _write("loadaware_score.json", SCORE_CASES, SRC, dict(node_allocatable=NODE, harness=f"{SRC}:1754-1850"))
    _write("estimator_pod.json", ESTIMATE_POD_CASES, EST, dict(harness=f"{EST}:233-249"))
    _write("estimator_node.json", ESTIMATE_NODE_CASES, EST, dict(harness=f"{EST}:312-328"))


if __name__ == "__main__":
    main()
