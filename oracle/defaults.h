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

/* (ABI 12) PodTopologySpread / InterPodAffinity with topologyKey kubernetes.io/hostname or topology.kubernetes.io/zone
 * (k8s v1.24.15 podtopologyspread/{common,filtering,scoring}.go, interpodaffinity/{filtering,scoring}.go; not
 * vendored, restated as published — "parity unpinned" beyond tests/test_pod_groups.py's hand-derived cases).  With
 * the hostname key each node is its own topology domain, so the plugins' per-domain maps become per-node counters
 * over the caller's match groups; zone-keyed maps are sums of those counters over a zone's nodes. */
typedef struct or_group_node {
  int32_t cnt[KG_MAX_MATCH_GROUPS];     /* pods on the node matching group k (countPodsMatchSelector)        */
  int32_t anti[KG_MAX_MATCH_GROUPS];    /* required anti-affinity terms of group k held by the node's pods   */
  int32_t symw[KG_MAX_MATCH_GROUPS];    /* Σ symmetric weights of the node's pods' terms of group k          */
  int32_t anti_z[KG_MAX_MATCH_GROUPS];  /* the same two for the node's pods' zone-keyed terms               */
  int32_t symw_z[KG_MAX_MATCH_GROUPS];
} or_group_node;
/* InterPodAffinity's zone-keyed topologyToMatchedTermCount maps of one incoming pod (interpodaffinity PreFilter /
 * PreScore over every node carrying the zone label), indexed by zone − 1; entries = len(affinityCounts) ≠ 0. */
typedef struct or_ipa_zones {
  int64_t aff[KG_MAX_ZONES];      /* affinityCounts[zone]: pods matching every required affinity term          */
  int64_t anti_in[KG_MAX_ZONES];  /* antiAffinityCounts[zone] of the pod's zone-keyed required anti terms      */
  int64_t anti_ex[KG_MAX_ZONES];  /* existingAntiAffinityCounts[zone]: existing pods' zone anti terms vs pod   */
  int64_t score[KG_MAX_ZONES];    /* topologyScore[zone]                                                       */
  int64_t entries;                /* affinityCounts has a pair (hostname or zone)                              */
} or_ipa_zones;
/* Adds one valid node's counters (zone = 1 + zone id, 0 = no zone label) to `pod`'s maps (zeroed by the caller). */
void or_ipa_zones_add(or_ipa_zones* z, const or_group_node* g, int32_t zone, const kg_pod* pod);
/* NodeInfo.AddPod / RemovePod of `pod` (sign ±1) on one node's counters. */
void or_groups_apply(or_group_node* g, const kg_pod* pod, int sign, int64_t hard_weight);
/* PodTopologySpread constraints' node requirements (common.go nodeLabelsMatchSpreadConstraints + the PreFilter /
 * PreScore node selection): the pod's nodeSelector / required node affinity hold and the node carries every topology
 * key of the pod's constraints of that kind (hard = DoNotSchedule: the Filter's set; else ScheduleAnyway). */
int or_spread_node_ok(const kg_node_predicates* n, const kg_pod* pod, int hard);
/* 1 = the node carries every topology key of the pod's constraints of that kind. */
int or_spread_has_keys(const kg_node_predicates* n, const kg_pod* pod, int hard);
/* PodTopologySpread Score (scoring.go Score) before normalisation: Σ over the ScheduleAnyway constraints in the pod's
 * order of float64(cnt[c]) · w[c] + float64(maxSkew − 1), accumulated in float64 from 0, then int64(). */
/* (ABI 13) the pod's spread constraints are the plugin's system defaults: requireAllTopologies is false */
int or_spread_system_default(const kg_pod* pod);
/* (r5) Go's math.Log restated (amd64: no FMA contraction); the PodTopologySpread weight uses it. */
double or_go_log(double x);
int64_t or_spread_raw(const int64_t* cnt, const double* w, const kg_pod* pod);
/* PodTopologySpread NormalizeScore: MaxNodeScore · (max + min − s) / max, MaxNodeScore when max == 0. */
int64_t or_spread_normalize(int64_t raw, int64_t mn, int64_t mx);
/* InterPodAffinity Filter (filtering.go Filter): required affinity (the conjunction group, or the first pod of a
 * series: no pod in the cluster matches and the pod matches its own terms), required anti-affinity, existing pods'
 * anti-affinity; 1 = pass.  total[k] = pods in the cluster matching group k. */
int or_interpod_filter(const or_group_node* g, const kg_pod* pod, int32_t zone, const or_ipa_zones* z);
/* InterPodAffinity Score (scoring.go Score: the node's hostname pair plus its zone pair) before normalisation. */
int64_t or_interpod_raw(const or_group_node* g, const kg_pod* pod, int32_t zone, const or_ipa_zones* z);
/* InterPodAffinity NormalizeScore: int64(MaxNodeScore · float64(s − min) / float64(max − min)), 0 when max == min. */
int64_t or_interpod_normalize(int64_t raw, int64_t mn, int64_t mx);

#ifdef __cplusplus
}
#endif
#endif
