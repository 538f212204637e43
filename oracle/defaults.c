/* defaults.c — see defaults.h (TEST INFRASTRUCTURE ONLY). */
#include "defaults.h"

#include <math.h>

/* taint_toleration.go Filter: v1helper.FindMatchingUntoleratedTaint(node.Spec.Taints, pod.Spec.Tolerations,
 * effect ∈ {NoSchedule, NoExecute}); a taint id carries its effect, so "tolerated" is per id. */
int or_taint_filter(const kg_node_predicates* n, const kg_pod* pod) {
  return (n->taints_hard & ~pod->tolerated_taints) == 0;
}

/* taint_toleration.go countIntolerableTaintsPreferNoSchedule: PreferNoSchedule taints not tolerated by the pod's
 * tolerations of effect "" / PreferNoSchedule (a toleration of another effect never tolerates such a taint). */
int64_t or_taint_count(const kg_node_predicates* n, const kg_pod* pod) {
  int64_t c = 0;
  for (int t = 0; t < 64; t++)
    if (((n->taints_soft >> t) & 1u) && !((pod->tolerated_taints >> t) & 1u)) c++;
  return c;
}

/* component-helpers nodeaffinity nodeSelectorTerm.match: all requirements hold; no requirements = no match */
static int term_match(uint64_t pred, uint64_t term) {
  if (term == 0) return 0;
  for (int k = 0; k < 64; k++)
    if (((term >> k) & 1u) && !((pred >> k) & 1u)) return 0;
  return 1;
}

/* node_affinity.go Filter → RequiredNodeAffinity.Match: labels.SelectorFromSet(pod.Spec.NodeSelector) first, then
 * NodeSelector.Match (ORed terms) when RequiredDuringSchedulingIgnoredDuringExecution is set. */
int or_affinity_filter(const kg_node_predicates* n, const kg_pod* pod) {
  for (int k = 0; k < 64; k++)
    if (((pod->node_selector >> k) & 1u) && !((n->predicates >> k) & 1u)) return 0;
  if (pod->n_required_terms == 0) return 1;
  for (int64_t t = 0; t < pod->n_required_terms; t++)
    if (term_match(n->predicates, pod->required_terms[t])) return 1;
  return 0;
}

/* node_affinity.go Score: PreferredSchedulingTerms with weight 0 are skipped; matching ones add their weight. */
int64_t or_affinity_sum(const kg_node_predicates* n, const kg_pod* pod) {
  int64_t s = 0;
  for (int64_t t = 0; t < pod->n_preferred_terms; t++) {
    if (pod->preferred_weights[t] == 0) continue;
    if (term_match(n->predicates, pod->preferred_terms[t])) s += pod->preferred_weights[t];
  }
  return s;
}

/* balanced_allocation.go balancedResourceScorer over resource_allocation.go's requested / allocatable maps:
 * a resource enters only with a non-zero Allocatable; fraction = float64(req) / float64(alloc) capped at 1;
 * two fractions → std = |f0 − f1| / 2, fewer → 0; score = int64((1 − std) · MaxNodeScore). */
int64_t or_balanced_score(int64_t alloc_cpu, int64_t alloc_mem, int64_t req_cpu, int64_t req_mem, int64_t pod_cpu,
                          int64_t pod_mem, int64_t resources) {
  double f[2];
  int n = 0;
  if ((resources & 1) && alloc_cpu != 0) {
    double x = (double)(req_cpu + pod_cpu) / (double)alloc_cpu;
    f[n++] = x > 1 ? 1 : x;
  }
  if ((resources & 2) && alloc_mem != 0) {
    double x = (double)(req_mem + pod_mem) / (double)alloc_mem;
    f[n++] = x > 1 ? 1 : x;
  }
  double std = 0;
  if (n == 2) std = fabs((f[0] - f[1]) / 2);
  return (int64_t)((1 - std) * (double)100);
}

/* imagelocality/image_locality.go (v1.24.15): sumImageScores over pod.Spec.Containers — a container whose normalized
 * image the node holds adds its image's scaledImageScore (int64(float64(size) * spread), node-independent, computed
 * by the caller) — then calculatePriority: clamp to [23 MiB, 1000 MiB × #containers],
 * MaxNodeScore * (sum - minThreshold) / (maxThreshold - minThreshold) in int64. */
int64_t or_image_score(const kg_node_predicates* n, const kg_pod* pod) {
  const int64_t mb = 1024 * 1024, min_t = 23 * mb, max_t = 1000 * mb * pod->n_containers;
  int64_t sum = 0;
  for (int64_t c = 0; c < pod->n_containers; c++) {
    const int64_t b = pod->container_image_bit[c];
    if (b >= 0 && ((n->images >> b) & 1u)) sum += pod->container_image_score[c];
  }
  if (sum < min_t) sum = min_t;
  else if (sum > max_t) sum = max_t;
  return 100 * (sum - min_t) / (max_t - min_t);
}

/* helper/normalize_score.go DefaultNormalizeScore */
int64_t or_normalize_default(int64_t score, int64_t max_count, int reverse) {
  if (max_count == 0) return reverse ? 100 : score;
  int64_t s = 100 * score / max_count;
  return reverse ? 100 - s : s;
}
