/*
 * defaults.h — CPU restatement of the upstream default plugins a stock koord-scheduler profile keeps
 * (SURVEY §8f-2): TaintToleration, NodeAffinity and NodeResourcesBalancedAllocation.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h): tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it
 * as the checker; nothing under koordinator_amd/ links or calls it.
 *
 * The reference runs these plugins from k8s.io/kubernetes v1.24.15 (go.mod:57, replaced at go.mod:275), which is
 * not vendored under /root/reference and not importable here: the functions restate the published v1.24 algorithm
 * (pkg/scheduler/framework/plugins/{tainttoleration/taint_toleration.go, nodeaffinity/node_affinity.go,
 * noderesources/balanced_allocation.go, noderesources/resource_allocation.go, helper/normalize_score.go}).  The only
 * fixture the reference holds for them is frameworkext/debug_test.go:91-174 (already-computed per-plugin Scores
 * summed by the debug table), which pins the weighted sum, not the plugins: "parity unpinned" beyond the
 * hand-derived cases in tests/test_default_plugins.py.
 *
 * Label and taint matching is the caller's (kg_node_predicates): the functions take the bitmasks the engine takes.
 */
#ifndef KOORD_ORACLE_DEFAULTS_H_
#define KOORD_ORACLE_DEFAULTS_H_
#include <stdint.h>
#include "../include/koordgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* TaintToleration Filter: 1 = no untolerated NoSchedule / NoExecute taint (FindMatchingUntoleratedTaint). */
int or_taint_filter(const kg_node_predicates* n, const kg_pod* pod);
/* countIntolerableTaintsPreferNoSchedule. */
int64_t or_taint_count(const kg_node_predicates* n, const kg_pod* pod);
/* NodeAffinity Filter: RequiredNodeAffinity.Match (nodeSelector, then any required term). */
int or_affinity_filter(const kg_node_predicates* n, const kg_pod* pod);
/* NodeAffinity Score before normalisation: Σ weights of matching preferred terms. */
int64_t or_affinity_sum(const kg_node_predicates* n, const kg_pod* pod);
/* BalancedAllocation Score (useRequested = true) from Allocatable, Requested and the pod's request of cpu / memory;
 * `resources` bit 0 = cpu, bit 1 = memory listed. */
int64_t or_image_score(const kg_node_predicates* n, const kg_pod* pod);
int64_t or_balanced_score(int64_t alloc_cpu, int64_t alloc_mem, int64_t req_cpu, int64_t req_mem, int64_t pod_cpu,
                          int64_t pod_mem, int64_t resources);
/* DefaultNormalizeScore(MaxNodeScore, reverse) of one score against the maximum over the scored nodes. */
int64_t or_normalize_default(int64_t score, int64_t max_count, int reverse);

#ifdef __cplusplus
}
#endif
#endif
