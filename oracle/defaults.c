/* defaults.c — see defaults.h (TEST INFRASTRUCTURE ONLY). */
#include "defaults.h"

#include <math.h>
#include <string.h>

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

/* ---- (ABI 12) PodTopologySpread / InterPodAffinity, topologyKey kubernetes.io/hostname or zone -------------------- */

/* The counters a pod contributes to its node: countPodsMatchSelector (podtopologyspread/common.go, and the
 * interpodaffinity PreFilter / PreScore matches of existing pods against the incoming pod's terms) counts it in every
 * group it matches; its required anti-affinity terms feed existingAntiAffinityCounts (filtering.go
 * getExistingAntiAffinityCounts); its terms matched by a later incoming pod feed that pod's topologyScore
 * (scoring.go processExistingPod: required affinity × HardPodAffinityWeight when > 0, preferred ± weight). */
void or_groups_apply(or_group_node* g, const kg_pod* pod, int sign, int64_t hard_weight) {
  for (int k = 0; k < KG_MAX_MATCH_GROUPS; k++) {
    if ((pod->match_groups >> k) & 1) g->cnt[k] += sign;
    if ((pod->pod_anti_affinity >> k) & 1) g->anti[k] += sign;
    if ((pod->pod_anti_affinity_zone >> k) & 1) g->anti_z[k] += sign;
    if (hard_weight > 0 && ((pod->pod_affinity_terms >> k) & 1)) g->symw[k] += sign * (int32_t)hard_weight;
    if (hard_weight > 0 && ((pod->pod_affinity_terms_zone >> k) & 1)) g->symw_z[k] += sign * (int32_t)hard_weight;
  }
  for (int64_t t = 0; t < pod->n_pod_preferred; t++) {
    const int64_t k = pod->pod_preferred_group[t] - 1;
    if (k < 0 || k >= KG_MAX_MATCH_GROUPS) continue;
    int32_t* w = ((pod->pod_preferred_zone >> t) & 1) ? &g->symw_z[k] : &g->symw[k];
    *w += sign * (int32_t)pod->pod_preferred_weight[t];
  }
}

/* filtering.go getTPMapMatchingIncomingAffinityAntiAffinity / getExistingAntiAffinityCounts and scoring.go PreScore,
 * zone key: every existing pod on a node with the zone label adds its matches to the node's zone pair; a required
 * affinity match needs all the pod's terms (updateWithAffinityTerms); hostname terms make a pair on every node. */
void or_ipa_zones_add(or_ipa_zones* z, const or_group_node* g, int32_t zone, const kg_pod* pod) {
  const int64_t a = pod->pod_affinity_group - 1;
  if (a >= 0 && pod->pod_affinity_terms && g->cnt[a] > 0) z->entries = 1;  /* a hostname pair */
  if (zone <= 0) return;
  if (a >= 0 && pod->pod_affinity_terms_zone) {
    z->aff[zone - 1] += g->cnt[a];
    if (z->aff[zone - 1] > 0) z->entries = 1;
  }
  for (int k = 0; k < KG_MAX_MATCH_GROUPS; k++) {
    if ((pod->pod_anti_affinity_zone >> k) & 1) z->anti_in[zone - 1] += g->cnt[k];
    if ((pod->match_groups >> k) & 1) {
      z->anti_ex[zone - 1] += g->anti_z[k];
      z->score[zone - 1] += g->symw_z[k];
    }
  }
  for (int64_t t = 0; t < pod->n_pod_preferred; t++)
    if ((pod->pod_preferred_zone >> t) & 1)
      z->score[zone - 1] += pod->pod_preferred_weight[t] * (int64_t)g->cnt[pod->pod_preferred_group[t] - 1];
}

static int spread_needs_zone(const kg_pod* pod, int hard) {
  for (int64_t c = 0; c < pod->n_spread; c++)
    if (((pod->spread_flags[c] & KG_SPREAD_HARD) != 0) == (hard != 0) && (pod->spread_flags[c] & KG_SPREAD_ZONE))
      return 1;
  return 0;
}

int or_spread_has_keys(const kg_node_predicates* n, const kg_pod* pod, int hard) {
  return !spread_needs_zone(pod, hard) || n->zone > 0;  /* kubernetes.io/hostname: every node carries it */
}

/* (ABI 13) requireAllTopologies = len(pod.Spec.TopologySpreadConstraints) > 0 || !systemDefaulted (podtopologyspread
 * PreScore, k8s v1.24.15): false when the pod's constraints are the plugin's system defaults */
int or_spread_system_default(const kg_pod* pod) {
  return pod->n_spread > 0 && (pod->spread_flags[0] & KG_SPREAD_SYSTEM_DEFAULT) != 0;
}

int or_spread_node_ok(const kg_node_predicates* n, const kg_pod* pod, int hard) {
  return or_affinity_filter(n, pod) && or_spread_has_keys(n, pod, hard);
}

/* scoring.go: scoreForCount = float64(cnt)·weight + float64(maxSkew − 1), summed over the constraints from 0 and
 * truncated by int64() (no fused multiply-add: -ffp-contract=off); weight = log(size + 2), the caller's per constraint */
/* (r5) Go's math.Log (go1.18+ src/math/log.go `log`, the FreeBSD e_log.c algorithm; on amd64 `archLog` in log_amd64.s
 * evaluates the same expression in the same order with SSE2 scalar ops, and the Go compiler never contracts a*b+c
 * into an FMA on amd64), restated here in plain IEEE double arithmetic (-ffp-contract=off).  PodTopologySpread's
 * topologyNormalizingWeight(size) = math.Log(float64(size + 2)) (podtopologyspread/scoring.go, k8s v1.24.15) feeds
 * int64(cnt·w + maxSkew − 1), so a one-ulp difference from glibc's log() could move a truncation: the oracle and the
 * engine both compute the weight with this function (tests/test_go_log.py compares it with glibc over [0, 1M]). */
double or_go_log(double x) {
  static const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10;
  static const double L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01, L3 = 2.857142874366239149e-01,
                      L4 = 2.222219843214978396e-01, L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01,
                      L7 = 1.479819860511658591e-01;
  if (isnan(x) || isinf(x)) return x > 0 || isnan(x) ? x : NAN;
  if (x < 0) return NAN;
  if (x == 0) return -INFINITY;
  int ki = 0;
  double f1 = frexp(x, &ki); /* Go's Frexp: f1 in [0.5, 1), the same for every finite non-zero x (subnormals too) */
  if (f1 < 0.70710678118654752440 /* math.Sqrt2 / 2 as a float64 constant */) {
    f1 *= 2;
    ki--;
  }
  const double f = f1 - 1, k = (double)ki;
  const double s = f / (2 + f), s2 = s * s, s4 = s2 * s2;
  const double t1 = s2 * (L1 + s4 * (L3 + s4 * (L5 + s4 * L7)));
  const double t2 = s4 * (L2 + s4 * (L4 + s4 * L6));
  const double R = t1 + t2, hfsq = 0.5 * f * f;
  return k * Ln2Hi - ((hfsq - (s * (hfsq + R) + k * Ln2Lo)) - f);
}

int64_t or_spread_raw(const int64_t* cnt, const double* w, const kg_pod* pod) {
  double s = 0;
  for (int64_t c = 0; c < pod->n_spread; c++) {
    if (pod->spread_flags[c] & KG_SPREAD_HARD) continue;
    if (cnt[c] < 0) continue; /* (ABI 13) Score: `if tpVal, ok := node.Labels[c.TopologyKey]; ok` — no label, no term */
    s += (double)cnt[c] * w[c] + (double)(pod->spread_max_skew[c] - 1);
  }
  return (int64_t)s;
}

int64_t or_spread_normalize(int64_t raw, int64_t mn, int64_t mx) {
  if (mx == 0) return 100;
  return 100 * (mx + mn - raw) / mx;
}

int or_interpod_filter(const or_group_node* g, const kg_pod* pod, int32_t zone, const or_ipa_zones* z) {
  const int64_t a = pod->pod_affinity_group - 1;
  if (a >= 0) {  /* satisfyPodAffinity: every term's topology key on the node, then each term's pair count */
    if (pod->pod_affinity_terms_zone && zone <= 0) return 0;
    int exist = 1;
    if (pod->pod_affinity_terms && g->cnt[a] <= 0) exist = 0;
    if (pod->pod_affinity_terms_zone && z->aff[zone - 1] <= 0) exist = 0;
    if (!exist && !(!z->entries && ((pod->match_groups >> a) & 1))) return 0;
  }
  for (int k = 0; k < KG_MAX_MATCH_GROUPS; k++) {
    if (((pod->pod_anti_affinity >> k) & 1) && g->cnt[k] > 0) return 0;  /* satisfyPodAntiAffinity */
    if (((pod->match_groups >> k) & 1) && g->anti[k] > 0) return 0;      /* satisfyExistingPodsAntiAffinity */
  }
  if (zone > 0 && (z->anti_in[zone - 1] > 0 || z->anti_ex[zone - 1] > 0)) return 0;  /* the zone pairs */
  return 1;
}

int64_t or_interpod_raw(const or_group_node* g, const kg_pod* pod, int32_t zone, const or_ipa_zones* z) {
  int64_t s = zone > 0 ? z->score[zone - 1] : 0;
  for (int64_t t = 0; t < pod->n_pod_preferred; t++) {
    const int64_t k = pod->pod_preferred_group[t] - 1;
    if (k >= 0 && k < KG_MAX_MATCH_GROUPS && !((pod->pod_preferred_zone >> t) & 1))
      s += pod->pod_preferred_weight[t] * (int64_t)g->cnt[k];
  }
  for (int k = 0; k < KG_MAX_MATCH_GROUPS; k++)
    if ((pod->match_groups >> k) & 1) s += g->symw[k];
  return s;
}

int64_t or_interpod_normalize(int64_t raw, int64_t mn, int64_t mx) {
  const int64_t d = mx - mn;
  if (d <= 0) return 0;
  return (int64_t)(100.0 * ((double)(raw - mn) / (double)d));
}
