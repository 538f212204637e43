/*
 * oracle.c — plain-C restatement of the koord-scheduler Filter/Score/selectHost/assume path.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Build: oracle/Makefile (gcc -O2 -ffp-contract=off, no fast-math,
 * so float64 expressions round exactly like Go's).  Every function cites the reference file:line it restates
 * (paths relative to /root/reference).
 */
#define _GNU_SOURCE
#include "oracle.h"
#include "numa.h"
#include "deviceshare.h"
#include "reservation.h"

#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>
#include <sched.h>

#define MAX_NODE_SCORE 100 /* framework.MaxNodeScore (k8s v1.24.15) */
#define DEFAULT_MILLI_CPU_REQUEST 250LL                 /* estimator/default_estimator.go:36 */
#define DEFAULT_MEMORY_REQUEST (200LL * 1024 * 1024)     /* estimator/default_estimator.go:38 */

static int is_cpu_like(int r) { return r == KG_RES_CPU; }

/* Quantity.MilliValue() of the value stored in slot r (cpu is stored in milli already). */
static int64_t milli_of(int r, int64_t v) { return is_cpu_like(r) ? v : v * 1000; }

/* apis/extension/resource.go:53-58 TranslateResourceNameByPriorityClass; -1 = "" (no such resource). */
static int translate_resource(int64_t prio, int r) {
  if (prio == KG_PRIO_PROD || prio == KG_PRIO_NONE) return r;
  if (prio == KG_PRIO_BATCH) {
    if (r == KG_RES_CPU) return KG_RES_BATCH_CPU;
    if (r == KG_RES_MEMORY) return KG_RES_BATCH_MEMORY;
    return -1;
  }
  if (prio == KG_PRIO_MID) {
    if (r == KG_RES_CPU) return KG_RES_MID_CPU;
    if (r == KG_RES_MEMORY) return KG_RES_MID_MEMORY;
    return -1;
  }
  return -1; /* PriorityFree: ResourceNameMap has no entry → "" */
}

/* estimator/default_estimator.go:73-108 estimatedUsedByResource */
int64_t or_estimated_used_by_resource(const kg_pod* pod, int real, int64_t scaling_factor) {
  int64_t limit = real >= 0 ? pod->limits[real] : 0;
  int64_t request = real >= 0 ? pod->requests[real] : 0;
  int64_t q;
  if (limit > request) { /* limitQuantity.Cmp(requestQuantity) > 0 */
    scaling_factor = 100;
    q = limit;
  } else {
    q = request;
  }
  if (q == 0) {
    if (real == KG_RES_CPU || real == KG_RES_BATCH_CPU) return DEFAULT_MILLI_CPU_REQUEST;
    if (real == KG_RES_MEMORY || real == KG_RES_BATCH_MEMORY) return DEFAULT_MEMORY_REQUEST;
    return 0;
  }
  /* case cpu: MilliValue; default: Value — slot values already carry exactly that unit */
  volatile double prod = (double)q * (double)scaling_factor; /* float64(q) * float64(f), rounded */
  int64_t est = (int64_t)round(prod / 100.0);
  if (limit > 0 && est > limit) est = limit;
  return est;
}

/* estimator/default_estimator.go:57-70 estimatedPodUsed, for the weight keys cpu and memory */
void or_estimate_pod(const kg_config* cfg, const kg_pod* pod, int64_t out[2]) {
  for (int r = 0; r < 2; r++) {
    out[r] = 0;
    if (cfg->la_resource_weights[r] == 0) continue; /* only resources in ResourceWeights are estimated */
    int real = translate_resource(pod->priority_class, r);
    out[r] = or_estimated_used_by_resource(pod, real, cfg->la_estimated_scaling_factors[r]);
  }
}

/* estimator/default_estimator.go:110-129 EstimateNode: raw-allocatable keys override node.Status.Allocatable */
int64_t or_estimate_node(const kg_node* node, int r) {
  if ((node->flags & KG_NODE_HAS_RAW_ALLOCATABLE) && node->raw_allocatable_present[r]) return node->raw_allocatable[r];
  return node->allocatable[r];
}

/* loadaware/helper.go:36-41 isNodeMetricExpired */
static int node_metric_expired(const kg_node_metric* m, int64_t expiration_seconds, int64_t now) {
  if (!m->present || !m->has_update_time) return 1;
  return expiration_seconds > 0 && (now - m->update_time_unix_nano) >= expiration_seconds * 1000000000LL;
}

/* loadaware/helper.go:102-140 generateUsageThresholdsFilterProfile (non-aggregated part). */
/* Custom maps replace the args' maps when non-empty (len counts zero-valued keys; -1 = key absent).  Args
 * maps encode "absent" as 0, which the threshold loop skips anyway (load_aware.go:186,235). */
static void usage_threshold_profile(const kg_config* cfg, const kg_node* node, int64_t thr[KG_RES_MAX],
                                    int64_t prod_thr[KG_RES_MAX], int* n_thr, int* n_prod) {
  int custom = (node->flags & KG_NODE_HAS_CUSTOM_THRESHOLDS) != 0;
  int nc = 0, ncp = 0, nargs = 0, nargs_prod = 0;
  for (int r = 0; r < KG_RES_MAX; r++) {
    if (custom && node->custom_usage_thresholds[r] >= 0) nc++;
    if (custom && node->custom_prod_usage_thresholds[r] >= 0) ncp++;
    if (cfg->la_usage_thresholds[r] != 0) nargs++;
    if (cfg->la_prod_usage_thresholds[r] != 0) nargs_prod++;
  }
  for (int r = 0; r < KG_RES_MAX; r++) {
    thr[r] = nc > 0 ? (node->custom_usage_thresholds[r] > 0 ? node->custom_usage_thresholds[r] : 0)
                    : cfg->la_usage_thresholds[r];
    prod_thr[r] = ncp > 0 ? (node->custom_prod_usage_thresholds[r] > 0 ? node->custom_prod_usage_thresholds[r] : 0)
                          : cfg->la_prod_usage_thresholds[r];
  }
  *n_thr = nc > 0 ? nc : nargs;
  *n_prod = ncp > 0 ? ncp : nargs_prod;
}

/* loadaware/helper.go:58-92 getTargetAggregatedUsage: index of the AggregatedNodeUsages entry read, -1 = nil */
static int target_aggregated(const kg_node_metric* m, int64_t dur_ns, int64_t type) {
  if (!m->has_node_metric || m->agg_count <= 0 || type < 1 || type > KG_AGG_TYPES) return -1;
  const int n = m->agg_count < KG_MAX_AGG ? (int)m->agg_count : KG_MAX_AGG;
  if (dur_ns == 0) { /* "the maximum period recorded by NodeMetrics will be used by default" */
    int64_t max_d = 0;
    int max_i = 0;
    for (int i = 0; i < n; i++)
      if (m->agg_duration_ns[i] > max_d) { max_d = m->agg_duration_ns[i]; max_i = i; }
    return m->agg_present[max_i][type - 1] ? max_i : -1; /* len(usage.ResourceList) > 0 */
  }
  for (int i = 0; i < n; i++)
    if (m->agg_duration_ns[i] == dur_ns && m->agg_present[i][type - 1]) return i;
  return -1;
}

static int64_t aggregated_value(const kg_node_metric* m, int i, int64_t type, int r) {
  return (r < 2 && ((m->agg_present[i][type - 1] >> r) & 1)) ? m->agg_usage[i][type - 1][r] : 0;
}

/* generateUsageThresholdsFilterProfile's AggregatedUsage (helper.go:102-140): the annotation's when it has
 * thresholds and a type, else the args' when filterWithAggregation (helper.go:94-96).  Returns 0 for nil. */
static int aggregated_filter_profile(const kg_config* cfg, const kg_node* node, int64_t thr[KG_RES_MAX],
                                     int64_t* type, int64_t* dur) {
  int nargs = 0, ncust = 0;
  for (int r = 0; r < KG_RES_MAX; r++) {
    if (cfg->la_agg_usage_thresholds[r] != 0) nargs++;
    if (node->custom_agg_thresholds[r] >= 0) ncust++;
  }
  if ((node->flags & KG_NODE_HAS_CUSTOM_THRESHOLDS) && ncust > 0 && node->custom_agg_type != KG_AGG_NONE) {
    for (int r = 0; r < KG_RES_MAX; r++) thr[r] = node->custom_agg_thresholds[r] > 0 ? node->custom_agg_thresholds[r] : 0;
    *type = node->custom_agg_type;
    *dur = node->custom_agg_duration_ns;
    return 1;
  }
  if (nargs > 0 && cfg->la_agg_usage_type != KG_AGG_NONE) {
    for (int r = 0; r < KG_RES_MAX; r++) thr[r] = cfg->la_agg_usage_thresholds[r];
    *type = cfg->la_agg_usage_type;
    *dur = cfg->la_agg_usage_duration_ns;
    return 1;
  }
  return 0;
}

/* loadaware/load_aware.go:123-171 Filter (+ filterNodeUsage :173-224, filterProdUsage :226-254) */
int or_loadaware_filter(const kg_config* cfg, const kg_node* node, const kg_node_metric* m, const kg_pod* pod,
                        int64_t now) {
  if (pod->flags & KG_POD_DAEMONSET) return 0;            /* :129-131 */
  if (!m->present) return 0;                               /* :133-140 NotFound → skip */
  if (cfg->la_filter_expired_node_metrics && cfg->la_node_metric_expiration_seconds >= 0 &&
      node_metric_expired(m, cfg->la_node_metric_expiration_seconds, now))
    return 0;                                              /* :144-147 */
  int64_t thr[KG_RES_MAX], pthr[KG_RES_MAX];
  int n_thr, n_prod;
  usage_threshold_profile(cfg, node, thr, pthr, &n_thr, &n_prod);
  if (n_prod > 0 && pod->priority_class == KG_PRIO_PROD) { /* :150-154 → filterProdUsage :226-254 */
    if (m->pods_metric_count == 0) return 0;               /* :227-229 */
    for (int r = 0; r < KG_RES_MAX; r++) {
      if (pthr[r] == 0) continue;                          /* :235-237 */
      int64_t total = or_estimate_node(node, r);
      if (total == 0) continue;                            /* :243-246 */
      volatile double q = (double)milli_of(r, m->prod_pods_usage[r]) / (double)milli_of(r, total);
      volatile double pct = q * 100.0;
      if ((int64_t)round(pct) >= pthr[r]) return 1;        /* :248-251 */
    }
    return 0;
  }
  int64_t athr[KG_RES_MAX], atype = 0, adur = 0;
  const int agg = aggregated_filter_profile(cfg, node, athr, &atype, &adur); /* :157-161 */
  if (agg) {
    n_thr = 0;
    for (int r = 0; r < KG_RES_MAX; r++) n_thr += athr[r] != 0;
    for (int r = 0; r < KG_RES_MAX; r++) thr[r] = athr[r];
  }
  if (n_thr == 0) return 0;
  if (!m->has_node_metric) return 0;                       /* :174-176 */
  const int ai = agg ? target_aggregated(m, adur, atype) : -1;
  for (int r = 0; r < KG_RES_MAX; r++) {                   /* :185-222 */
    if (thr[r] == 0) continue;
    int64_t total = or_estimate_node(node, r);
    if (total == 0) continue;
    if (agg && ai < 0) continue;                           /* :198-209 nodeUsage == nil */
    int64_t used = agg ? aggregated_value(m, ai, atype, r) : (m->node_usage_present[r] ? m->node_usage[r] : 0);
    volatile double q = (double)milli_of(r, used) / (double)milli_of(r, total);
    volatile double pct = q * 100.0;
    int64_t usage = (int64_t)round(pct);
    if (usage >= thr[r]) return 1;
  }
  return 0;
}

/* loadaware/load_aware.go:388-397 leastRequestedScore */
int64_t or_least_requested_score(int64_t requested, int64_t capacity) {
  if (capacity == 0) return 0;
  if (requested > capacity) return 0;
  return ((capacity - requested) * MAX_NODE_SCORE) / capacity;
}

/* NodeUsage (or the aggregated score usage) of the all-pods view, per resource present: load_aware.go:307-320 */
static void score_node_usage(const kg_config* cfg, const kg_node_metric* m, int64_t u[2], int present[2]) {
  u[0] = u[1] = 0;
  present[0] = present[1] = 0;
  if (!m->has_node_metric) return;
  if (cfg->la_agg_score_type != KG_AGG_NONE) {
    const int i = target_aggregated(m, cfg->la_agg_score_duration_ns, cfg->la_agg_score_type);
    if (i < 0) return;
    for (int r = 0; r < 2; r++) {
      u[r] = aggregated_value(m, i, cfg->la_agg_score_type, r);
      present[r] = 1;
    }
    return;
  }
  for (int r = 0; r < 2; r++)
    if (m->node_usage_present[r]) {
      u[r] = m->node_usage[r];
      present[r] = 1;
    }
}

/* estimatedAssignedPodUsed (load_aware.go:337-376), sumPodUsages (helper.go:172-186) and the two views of
 * Score (:296-326).  view 1 = buildPodMetricMap with filterProdPod and the prod-filtered assign cache. */
void or_la_node_terms(const kg_config* cfg, const kg_node_metric* m, const kg_pod_metric* pm, int64_t n_pm,
                      const or_assigned* as, int64_t n_as, int64_t out[4]) {
  int64_t nu[2];
  int present[2];
  score_node_usage(cfg, m, nu, present);
  const int64_t upd = m->has_update_time ? m->update_time_unix_nano : INT64_MIN;
  const int64_t interval = m->report_interval_ns > 0 ? m->report_interval_ns : 60LL * 1000000000LL; /* helper.go:43-48 */
  const int agg_nil = cfg->la_agg_score_type != KG_AGG_NONE &&
                      target_aggregated(m, cfg->la_agg_score_duration_ns, cfg->la_agg_score_type) < 0;
  for (int view = 0; view < 2; view++) {
    int64_t used[2] = {0, 0};       /* Σ over estimated pods of (counted value − EstimatePod) − Σ non-estimated EstimatePod */
    int64_t est_pods_usage[2] = {0, 0}, pods_usage[2] = {0, 0};
    char* estimated = (char*)calloc(n_pm > 0 ? (size_t)n_pm : 1, 1); /* estimatedPods, indexed like pm */
    if (!estimated) return;
    for (int64_t a = 0; a < n_as; a++) {
      if (view == 1 && !as[a].prod) continue;                                          /* :350-352 */
      int64_t hit = -1;
      for (int64_t q = 0; as[a].uid != 0 && q < n_pm; q++)
        if (pm[q].uid == as[a].uid && (view == 0 || pm[q].prod)) { hit = q; break; }   /* podMetrics[podName] */
      const int has_usage = hit >= 0 && (pm[hit].usage_present & 3) != 0;              /* len(podUsage) != 0 */
      const int missed = as[a].time > upd;                                             /* helper.go:50-52 */
      const int still = as[a].time < upd && upd - as[a].time < interval;               /* helper.go:54-56 */
      if (!has_usage || missed || still || agg_nil) {                                  /* :355-359 */
        for (int r = 0; r < 2; r++) {
          int64_t v = as[a].est[r];
          if (hit >= 0 && ((pm[hit].usage_present >> r) & 1) && pm[hit].usage[r] > v) v = pm[hit].usage[r]; /* :364-369 */
          used[r] += v - as[a].est[r];
        }
        if (hit >= 0) estimated[hit] = 1;                                              /* estimatedPods.Insert */
      } else {
        for (int r = 0; r < 2; r++) used[r] -= as[a].est[r];  /* counted through the reported usages instead */
      }
    }
    for (int64_t q = 0; q < n_pm; q++) {
      if (view == 1 && !pm[q].prod) continue;
      for (int r = 0; r < 2; r++)
        if ((pm[q].usage_present >> r) & 1) (estimated[q] ? est_pods_usage : pods_usage)[r] += pm[q].usage[r];
    }
    free(estimated);
    if (view == 1) {                                                                   /* :302-305 */
      for (int r = 0; r < 2; r++) out[2 + r] = pods_usage[r] + used[r];
    } else {                                                                           /* :306-326 */
      for (int r = 0; r < 2; r++) {
        int64_t q = nu[r];
        if (present[r] && est_pods_usage[r] != 0 && q >= est_pods_usage[r]) q -= est_pods_usage[r];
        out[r] = (present[r] ? q : 0) + used[r];
      }
    }
  }
}

/* loadaware/load_aware.go:269-335 Score (+ estimatedAssignedPodUsed :337-376, scorer :378-386).
 * Without PodsMetric (helper.go:153-156 → nil map) every assigned pod is estimated (:354) and no pod usage is
 * subtracted from NodeUsage (:317); with it, the state carries or_la_node_terms. */
int64_t or_loadaware_score(const kg_config* cfg, const kg_node* node, const kg_node_metric* m,
                           const or_node_state* st, const kg_pod* pod, int64_t now) {
  if (!m->present) return 0;                                                          /* :278-284 */
  if (cfg->la_node_metric_expiration_seconds >= 0 &&
      node_metric_expired(m, cfg->la_node_metric_expiration_seconds, now))
    return 0;                                                                         /* :287-289 */
  if (m->pods_metric_count != 0 && !st->has_la_term) return -1;
  int prod_pod = pod->priority_class == KG_PRIO_PROD && cfg->la_score_according_prod_usage; /* :291 */
  int64_t est[2];
  or_estimate_pod(cfg, pod, est);                                                     /* :294 */
  int64_t used[2];
  for (int r = 0; r < 2; r++) used[r] = est[r] + (prod_pod ? st->la_est_prod[r] : st->la_est_all[r]); /* :298-301 */
  if (st->has_la_term) {
    for (int r = 0; r < 2; r++) used[r] += st->la_term[(prod_pod ? 2 : 0) + r];
  } else if (!prod_pod && m->has_node_metric) {                                       /* :307-326 */
    if (cfg->la_agg_score_type != KG_AGG_NONE) { /* scoreWithAggregation: the aggregated usage, nil → none */
      const int i = target_aggregated(m, cfg->la_agg_score_duration_ns, cfg->la_agg_score_type);
      if (i >= 0)
        for (int r = 0; r < 2; r++) used[r] += aggregated_value(m, i, cfg->la_agg_score_type, r);
    } else {
      for (int r = 0; r < 2; r++)
        if (m->node_usage_present[r]) used[r] += m->node_usage[r];
    }
  }
  int64_t node_score = 0, weight_sum = 0;                                             /* :378-386 */
  for (int r = 0; r < 2; r++) {
    int64_t w = cfg->la_resource_weights[r];
    if (w == 0) continue;
    node_score += or_least_requested_score(used[r], or_estimate_node(node, r)) * w;
    weight_sum += w;
  }
  if (weight_sum == 0) return -1; /* Go would divide by zero; validation forbids it */
  return node_score / weight_sum;
}

/* k8s v1.24.15 noderesources/fit.go fitsRequest (restated in-tree by reservation/plugin.go:433-482). */
int or_fit_filter(const kg_node* node, const or_node_state* st, const kg_pod* pod) {
  int reasons = 0;
  if (st->num_pods + 1 > node->allowed_pods) reasons |= KG_REJECT_FIT_PODS;
  int zero = 1;
  for (int r = 0; r < KG_RES_MAX; r++) zero &= pod->requests[r] == 0;
  if (zero) return reasons;
  if (pod->requests[KG_RES_CPU] > node->allocatable[KG_RES_CPU] - st->requested[KG_RES_CPU])
    reasons |= KG_REJECT_FIT_CPU;
  if (pod->requests[KG_RES_MEMORY] > node->allocatable[KG_RES_MEMORY] - st->requested[KG_RES_MEMORY])
    reasons |= KG_REJECT_FIT_MEMORY;
  /* ephemeral-storage for every pod with a non-zero request (reservation/plugin.go:469-471: compared unconditionally,
   * so an overcommitted node rejects a pod without an ephemeral request too), then the scalar (batch / mid cpu /
   * memory) resources the pod requests (:472-479 `for rName, rQuant := range podRequest.ScalarResources`): a scalar
   * the pod does not request (0) is not a key of its request map. */
  if (pod->requests[KG_RES_EPHEMERAL] > node->allocatable[KG_RES_EPHEMERAL] - st->requested[KG_RES_EPHEMERAL])
    reasons |= KG_REJECT_FIT_OTHER;
  for (int r = KG_RES_EPHEMERAL + 1; r <= KG_RES_MID_MEMORY; r++)
    if (pod->requests[r] != 0 && pod->requests[r] > node->allocatable[r] - st->requested[r])
      reasons |= KG_REJECT_FIT_OTHER;
  return reasons;
}

/* k8s v1.24.15 noderesources resource_allocation.go score + least_allocated.go leastResourceScorer with
 * useRequested=false (NonZeroRequested); restated in-tree by nodenumaresource/scoring.go:191-230 and
 * least_allocated.go:30-58.  Only cpu/memory keys (non-scalar) are restated. */
int64_t or_fit_score(const kg_config* cfg, const kg_node* node, const or_node_state* st, const kg_pod* pod) {
  int64_t node_score = 0, weight_sum = 0;
  for (int r = 0; r < 2; r++) {
    int64_t w = cfg->fit_resource_weights[r];
    if (w == 0) continue;                           /* not a key of resourceToWeightMap */
    int64_t alloc = node->allocatable[r];
    if (alloc == 0) continue;                       /* "Only fill the extended resource entry when it's non-zero" */
    int64_t req = st->nonzero[r] + pod->nonzero_requests[r];
    node_score += or_least_requested_score(req, alloc) * w;
    weight_sum += w;
  }
  if (weight_sum == 0) return 0;
  return node_score / weight_sum;
}

/* upstream NodeInfo.AddPod/RemovePod + podAssignCache.assign/unAssign (pod_assign_cache.go:53-80) with the estimate
 * taken at Score time (load_aware.go:359).  informer = 1: the pod informer's add / delete (OnAdd / OnDelete), which a
 * reserve pod never reaches (a Reservation is not a Pod object); 0: LoadAware Reserve / Unreserve
 * (load_aware.go:260-267), which assign / unAssign every scheduled pod, a reserve pod included. */
static void apply_pod(const kg_config* cfg, or_node_state* st, const kg_pod* pod, int sign, int informer) {
  for (int r = 0; r < KG_RES_MAX; r++) st->requested[r] += sign * pod->requests[r];
  st->nonzero[0] += sign * pod->nonzero_requests[0];
  st->nonzero[1] += sign * pod->nonzero_requests[1];
  st->num_pods += sign;
  if (informer && (pod->flags & KG_POD_RESERVE)) return;
  int64_t est[2];
  or_estimate_pod(cfg, pod, est);
  for (int r = 0; r < 2; r++) {
    st->la_est_all[r] += sign * est[r];
    if (pod->priority_class == KG_PRIO_PROD) st->la_est_prod[r] += sign * est[r];
  }
}

void or_apply_pod(const kg_config* cfg, or_node_state* st, const kg_pod* pod, int sign) { apply_pod(cfg, st, pod, sign, 1); }
void or_assume_pod(const kg_config* cfg, or_node_state* st, const kg_pod* pod, int sign) { apply_pod(cfg, st, pod, sign, 0); }

void or_states_init(int64_t n_nodes, or_node_state* st) { memset(st, 0, sizeof(*st) * (size_t)n_nodes); }

int or_states_add_pods(const kg_config* cfg, int64_t n_nodes, or_node_state* st, int64_t n, const kg_pod* pods,
                       const int32_t* node_idx) {
  for (int64_t i = 0; i < n; i++) {
    if (node_idx[i] < 0 || node_idx[i] >= n_nodes) return KG_E_INVALID;
    or_apply_pod(cfg, &st[node_idx[i]], &pods[i], +1);
  }
  return 0;
}

/* ---------------------------------------------------------------------------------------------------
 * Scheduling loop.  Per pod: Filter pass over all nodes, Score pass over feasible nodes, weighted sum,
 * selectHost with lowest-index tie-break, assume.  Parallel passes mirror the reference Parallelizer:
 * 16 workers by default, chunk = max(1, min(sqrt(n), n/16+1)) (pkg/util/parallelize/parallelism.go:29-49).
 * ------------------------------------------------------------------------------------------------- */
typedef struct sched_ctx {
  const kg_config* cfg;
  int64_t n_nodes;
  const kg_node* nodes;
  const kg_node_metric* metrics;
  or_node_state* st;
  int64_t now;
  const kg_pod* pod;
  or_numa_node* numa;     /* per node NodeNUMAResource state (NULL: plugin not in the profile) */
  or_numa_pod numa_pod;   /* the pod's NodeNUMAResource preFilterState                          */
  or_hint* affinity;      /* per node: the topology manager's stored affinity (Filter → Score/Reserve) */
  kg_node_device* dev;    /* per node DeviceShare state (NULL: plugin not in the profile)       */
  or_ds_pod ds_pod;       /* the pod's DeviceShare preFilterState                               */
  int64_t* ds_raw;        /* per node: DeviceShare Score before NormalizeScore                  */
  int32_t* feasible;      /* per node: 1 feasible, 0 not, -1 unsupported */
  int64_t* total;         /* weighted score per node                     */
  int64_t chunk;
  atomic_long next;       /* work counter for the current phase          */
  int phase;              /* 0 filter, 1 score                           */
  int n_threads;
  atomic_int arrive;
  atomic_int generation;
  atomic_int stop;
} sched_ctx;

static void eval_filter(sched_ctx* c, int64_t i) {
  const kg_config* cfg = c->cfg;
  if (!(c->nodes[i].flags & KG_NODE_VALID)) { c->feasible[i] = 0; return; }
  int ok = 1;
  if (cfg->fit_filter && or_fit_filter(&c->nodes[i], &c->st[i], c->pod) != 0) ok = 0;
  if (ok && cfg->la_filter) {
    int s = or_loadaware_filter(cfg, &c->nodes[i], &c->metrics[i], c->pod, c->now);
    if (s < 0) { c->feasible[i] = -1; return; }
    if (s != 0) ok = 0;
  }
  if (c->numa) c->affinity[i] = (or_hint){1, 0, 0, 0};
  if (ok && cfg->numa_filter && c->numa && !or_numa_filter(cfg, &c->numa[i], &c->numa_pod, &c->affinity[i],
                                                            c->st[i].requested[KG_RES_CPU],
                                                            c->nodes[i].allocatable[KG_RES_CPU])) ok = 0;
  if (ok && cfg->ds_filter && c->dev && !or_ds_filter(&c->dev[i], &c->ds_pod)) ok = 0;
  c->feasible[i] = ok;
}

static void eval_score(sched_ctx* c, int64_t i) {
  const kg_config* cfg = c->cfg;
  if (c->feasible[i] != 1) return;
  int64_t t = 0;
  if (cfg->fit_score) t += cfg->weight_fit * or_fit_score(cfg, &c->nodes[i], &c->st[i], c->pod);
  if (cfg->la_score) {
    int64_t s = or_loadaware_score(cfg, &c->nodes[i], &c->metrics[i], &c->st[i], c->pod, c->now);
    if (s < 0) { c->feasible[i] = -1; return; }
    t += cfg->weight_loadaware * s;
  }
  if (cfg->numa_score && c->numa)
    t += cfg->weight_numa * or_numa_score(cfg, &c->numa[i], &c->numa_pod, &c->affinity[i], c->st[i].requested[KG_RES_CPU],
                                          c->st[i].requested[KG_RES_MEMORY], c->nodes[i].allocatable[KG_RES_CPU],
                                          c->nodes[i].allocatable[KG_RES_MEMORY]);
  if (c->dev) c->ds_raw[i] = cfg->ds_score ? or_ds_score(&c->dev[i], &c->ds_pod, (int)cfg->ds_scoring_strategy,
                                                         cfg->ds_scoring_weights) +
                                                 or_dsx_score(&c->dev[i], &c->ds_pod, (int)cfg->ds_scoring_strategy,
                                                              cfg->ds_scoring_weights_x)
                                           : 0;
  c->total[i] = t;
}

static void run_chunks(sched_ctx* c) {
  for (;;) {
    int64_t start = atomic_fetch_add(&c->next, c->chunk);
    if (start >= c->n_nodes) break;
    int64_t end = start + c->chunk < c->n_nodes ? start + c->chunk : c->n_nodes;
    for (int64_t i = start; i < end; i++) {
      if (c->phase == 0) eval_filter(c, i);
      else eval_score(c, i);
    }
  }
}

/* sense-reversing barrier over n_threads (workers + the main thread) */
static void barrier_wait(sched_ctx* c) {
  int gen = atomic_load(&c->generation);
  if (atomic_fetch_add(&c->arrive, 1) == c->n_threads - 1) {
    atomic_store(&c->arrive, 0);
    atomic_fetch_add(&c->generation, 1);
  } else {
    int spins = 0;
    while (atomic_load(&c->generation) == gen) {
      if (++spins > 256) { sched_yield(); spins = 0; }
    }
  }
}

static void* worker(void* arg) {
  sched_ctx* c = (sched_ctx*)arg;
  for (;;) {
    barrier_wait(c); /* phase start */
    if (atomic_load(&c->stop)) break;
    run_chunks(c);
    barrier_wait(c); /* phase end */
  }
  return NULL;
}

static void run_phase(sched_ctx* c, int phase) {
  c->phase = phase;
  atomic_store(&c->next, 0);
  if (c->n_threads <= 1) { run_chunks(c); return; }
  barrier_wait(c);
  run_chunks(c);
  barrier_wait(c);
}

int or_schedule(const kg_config* cfg, int64_t n_nodes, const kg_node* nodes, const kg_node_metric* metrics,
                or_node_state* st, int64_t n_pods, const kg_pod* pods, int64_t now, int n_threads,
                int32_t* out_node, int64_t* out_score) {
  return or_schedule_numa(cfg, n_nodes, nodes, metrics, st, NULL, n_pods, pods, now, n_threads, out_node, out_score,
                          NULL);
}

int or_schedule_numa(const kg_config* cfg, int64_t n_nodes, const kg_node* nodes, const kg_node_metric* metrics,
                     or_node_state* st, void* numa_states, int64_t n_pods, const kg_pod* pods, int64_t now,
                     int n_threads, int32_t* out_node, int64_t* out_score, uint64_t* out_cpus) {
  return or_schedule_full(cfg, n_nodes, nodes, metrics, st, numa_states, NULL, NULL, 0, n_pods, pods, now, n_threads,
                          out_node, out_score, out_cpus, NULL, NULL);
}

/* The pod's quota request over the KG_QUOTA_RES resources (PodRequestsAndLimits: cpu, memory, the device
 * resources) and which of them are keys of it: cpu / memory per the request-key flags, devices by value. */
static void quota_request(const kg_pod* p, int64_t req[KG_QUOTA_RES], int key[KG_QUOTA_RES]) {
  req[0] = p->requests[KG_RES_CPU];
  req[1] = p->requests[KG_RES_MEMORY];
  key[0] = or_pod_cpu_key(p);
  key[1] = or_pod_mem_key(p);
  for (int k = 0; k < KG_QUOTA_RES - 2; k++) {
    req[2 + k] = p->device_requests[k];
    key[2 + k] = p->device_requests[k] != 0;
  }
}

/* ElasticQuota PreFilter (elasticquota/plugin.go:211-256): Mask(Add(request, used), ResourceNames(request)) ≤
 * usedLimit, and for non-preemptible pods (extension.IsPodNonPreemptible) the same against min with the
 * non-preemptible used. */
int or_quota_admit(const kg_quota* q, const kg_pod* p) {
  int64_t req[KG_QUOTA_RES];
  int key[KG_QUOTA_RES];
  quota_request(p, req, key);
  /* quotav1.LessThanOrEqual(a, b) walks the keys of b and compares those a has: a limit of -1 (absent) is free */
  int ok = 1;
  for (int d = 0; d < KG_QUOTA_RES; d++)
    if (key[d] && q->used_limit[d] >= 0 && q->used[d] + req[d] > q->used_limit[d]) ok = 0;
  if (p->flags & KG_POD_NON_PREEMPTIBLE)
    for (int d = 0; d < KG_QUOTA_RES; d++)
      if (key[d] && q->min[d] >= 0 && q->non_preemptible_used[d] + req[d] > q->min[d]) ok = 0;
  return ok;
}

/* Reserve → GroupQuotaManager.ReservePod → updatePodUsedNoLock (core/group_quota_manager.go:613-648, 791-797) */
void or_quota_charge(kg_quota* q, const kg_pod* p) {
  int64_t req[KG_QUOTA_RES];
  int key[KG_QUOTA_RES];
  quota_request(p, req, key);
  for (int d = 0; d < KG_QUOTA_RES; d++) {
    q->used[d] += req[d];
    if (p->flags & KG_POD_NON_PREEMPTIBLE) q->non_preemptible_used[d] += req[d];
  }
}

int or_unreserve(const kg_config* cfg, or_node_state* st, void* numa_states, kg_node_device* dev,
                 kg_node_reservations* rsv, kg_quota* quotas, int64_t n_quotas, const kg_pod* pod, int32_t node,
                 const uint64_t* cpus, const int64_t* numa_alloc, int32_t minors, int32_t slot) {
  if (node < 0) return 0;
  if (pod->quota_id > n_quotas) return KG_E_INVALID;
  or_assume_pod(cfg, &st[node], pod, -1); /* NodeInfo.RemovePod + LoadAware Unreserve (unAssign) */
  if (numa_states && (cfg->numa_filter || cfg->numa_score) && cpus && numa_alloc) {
    if (rsv) or_numa_rsv_refs(&((or_numa_node*)numa_states)[node], &rsv[node]);
    or_cpuset cs;
    for (int w = 0; w < OR_CPUSET_WORDS; w++) cs.w[w] = cpus[w];
    or_numa_release(&((or_numa_node*)numa_states)[node], &cs, numa_alloc); /* nodenumaresource/plugin.go:417-425 */
  }
  if (dev && (cfg->ds_filter || cfg->ds_score) && minors) { /* deviceshare/plugin.go:440-455 */
    or_ds_pod dsp;
    if (or_ds_pod_init(pod, &dsp) != 0) return KG_E_INVALID;
    or_ds_release(&dev[node], &dsp, minors);
    /* (ABI 13) the pod leaves the reservation's AssignedPods: its allocation on the reservation's minors leaves the
     * restore's `allocated` (deviceshare/reservation.go:150-155) */
    if (rsv && slot >= 0) or_ds_rsv_assign(&rsv[node], slot, &dev[node], &dsp, minors, -1);
  }
  if (rsv && slot >= 0) or_rsv_forget(&rsv[node], slot, pod); /* reservation/plugin.go:561-583 */
  if (rsv && slot >= 0 && cpus) /* (ABI 15) the pod leaves the reservation's AssignedPods: its cpus are reserved again */
    for (int w = 0; w < OR_CPUSET_WORDS; w++) rsv[node].cpus_assigned[slot][w] &= ~cpus[w];
  if (quotas && pod->quota_id > 0) { /* elasticquota/plugin.go:348-360 → UnreservePod (addUsedNonNegativeNoLock) */
    kg_quota* q = &quotas[pod->quota_id - 1];
    int64_t req[KG_QUOTA_RES];
    int key[KG_QUOTA_RES];
    quota_request(pod, req, key);
    for (int d = 0; d < KG_QUOTA_RES; d++) {
      q->used[d] = q->used[d] - req[d] > 0 ? q->used[d] - req[d] : 0;
      if (pod->flags & KG_POD_NON_PREEMPTIBLE)
        q->non_preemptible_used[d] = q->non_preemptible_used[d] - req[d] > 0 ? q->non_preemptible_used[d] - req[d] : 0;
    }
  }
  return 0;
}

int or_schedule_full(const kg_config* cfg, int64_t n_nodes, const kg_node* nodes, const kg_node_metric* metrics,
                     or_node_state* st, void* numa_states, kg_node_device* dev, kg_quota* quotas, int64_t n_quotas,
                     int64_t n_pods, const kg_pod* pods, int64_t now, int n_threads, int32_t* out_node,
                     int64_t* out_score, uint64_t* out_cpus, int32_t* out_minors, int64_t* out_numa) {
  or_numa_node* numa = (or_numa_node*)numa_states;
  sched_ctx c;
  memset(&c, 0, sizeof(c));
  c.cfg = cfg; c.n_nodes = n_nodes; c.nodes = nodes; c.metrics = metrics; c.st = st; c.now = now;
  const int numa_on = numa && (cfg->numa_filter || cfg->numa_score);
  c.numa = numa_on ? numa : NULL;
  c.affinity = numa_on ? (or_hint*)calloc((size_t)(n_nodes > 0 ? n_nodes : 1), sizeof(or_hint)) : NULL;
  const int ds_on = dev && (cfg->ds_filter || cfg->ds_score);
  c.dev = ds_on ? dev : NULL;
  c.ds_raw = ds_on ? (int64_t*)calloc((size_t)(n_nodes > 0 ? n_nodes : 1), sizeof(int64_t)) : NULL;
  c.feasible = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n_nodes > 0 ? n_nodes : 1));
  c.total = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n_nodes > 0 ? n_nodes : 1));
  if (!c.feasible || !c.total) { free(c.feasible); free(c.total); return KG_E_NOMEM; }
  if (n_threads < 1) n_threads = 1;
  c.n_threads = n_threads;
  /* chunkSizeFor (parallelism.go:35-46) with parallelism = n_threads */
  int64_t s = (int64_t)sqrt((double)n_nodes);
  int64_t r = n_nodes / n_threads + 1;
  if (s > r) s = r; else if (s < 1) s = 1;
  c.chunk = s;
  pthread_t* th = NULL;
  if (n_threads > 1) {
    th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)(n_threads - 1));
    for (int t = 0; t < n_threads - 1; t++) pthread_create(&th[t], NULL, worker, &c);
  }
  int rc = 0;
  for (int64_t p = 0; p < n_pods && rc == 0; p++) {
    c.pod = &pods[p];
    kg_quota* quota = NULL;
    if (pods[p].quota_id > 0) {
      if (pods[p].quota_id > n_quotas) { rc = KG_E_INVALID; break; }
      quota = &quotas[pods[p].quota_id - 1];
      if (!or_quota_admit(quota, &pods[p])) { /* PreFilter Unschedulable: no node search, nothing reserved */
        out_node[p] = -1;
        out_score[p] = 0;
        if (out_minors) out_minors[p] = 0;
        if (out_cpus)
          for (int w = 0; w < OR_CPUSET_WORDS; w++) out_cpus[p * OR_CPUSET_WORDS + w] = 0;
        if (out_numa) memset(&out_numa[p * OR_NUMA_ALLOC_WORDS], 0, sizeof(int64_t) * OR_NUMA_ALLOC_WORDS);
        continue;
      }
    }
    if (c.numa) or_numa_pod_init(cfg, c.pod, &c.numa_pod);
    if (c.dev) {
      or_ds_pod_init(c.pod, &c.ds_pod);
      if (c.ds_pod.unsupported) { rc = KG_E_UNSUPPORTED; break; }
    }
    run_phase(&c, 0);
    run_phase(&c, 1);
    if (c.dev && cfg->ds_score) {
      /* RunScorePlugins: DeviceShare NormalizeScore = DefaultNormalizeScore over the feasible nodes' scores,
       * then × weight (scoring.go:95-97) */
      int64_t mx = 0;
      for (int64_t i = 0; i < n_nodes; i++)
        if (c.feasible[i] == 1 && c.ds_raw[i] > mx) mx = c.ds_raw[i];
      if (mx > 0)
        for (int64_t i = 0; i < n_nodes; i++)
          if (c.feasible[i] == 1) c.total[i] += cfg->weight_deviceshare * (100 * c.ds_raw[i] / mx);
    }
    /* selectHost: max total, ties → lowest snapshot index (BASELINE determinism pin) */
    int64_t best = -1, best_score = 0;
    for (int64_t i = 0; i < n_nodes; i++) {
      if (c.feasible[i] < 0) { rc = KG_E_UNSUPPORTED; break; }
      if (c.feasible[i] == 1 && (best < 0 || c.total[i] > best_score)) { best = i; best_score = c.total[i]; }
    }
    if (rc) break;
    /* Reserve: NodeNUMAResource allocates the cpuset / NUMA resources; a failure un-assumes the pod
     * (RunReservePluginsUnreserve + ForgetPod): it is not placed this cycle */
    or_cpuset cpus;
    memset(&cpus, 0, sizeof(cpus));
    int64_t nalloc[OR_NUMA_ALLOC_WORDS] = {0};
    or_numa_node numa_save;
    if (best >= 0 && c.numa) {
      numa_save = c.numa[best];
      if (or_numa_reserve(cfg, &c.numa[best], &c.numa_pod, &c.affinity[best], &cpus, nalloc) != 0) best = -1;
    }
    int32_t minors = 0;
    if (best >= 0 && c.dev) {
      minors = or_ds_reserve(&c.dev[best], &c.ds_pod, (int)cfg->ds_scoring_strategy, cfg->ds_scoring_weights);
      if (minors >= 0) { /* (ABI 17) the RDMA / FPGA types: all of them or none (the GPU part is given back) */
        const int32_t xm = or_dsx_reserve(&c.dev[best], &c.ds_pod, (int)cfg->ds_scoring_strategy,
                                          cfg->ds_scoring_weights_x);
        if (xm < 0) {
          or_ds_release(&c.dev[best], &c.ds_pod, minors);
          minors = -1;
        } else {
          minors |= xm;
        }
      }
      if (minors < 0) {
        /* DeviceShare Reserve failed: RunReservePluginsUnreserve releases NodeNUMAResource's allocation too */
        minors = 0;
        if (c.numa) {
          c.numa[best] = numa_save;
          memset(&cpus, 0, sizeof(cpus));
          memset(nalloc, 0, sizeof(nalloc));
        }
        best = -1;
      }
    }
    if (out_numa) memcpy(&out_numa[p * OR_NUMA_ALLOC_WORDS], nalloc, sizeof(nalloc));
    if (out_minors) out_minors[p] = minors;
    if (out_cpus)
      for (int w = 0; w < OR_CPUSET_WORDS; w++) out_cpus[p * OR_CPUSET_WORDS + w] = cpus.w[w];
    out_node[p] = (int32_t)best;
    out_score[p] = best >= 0 ? best_score : 0;
    if (best >= 0) or_assume_pod(cfg, &st[best], &pods[p], +1); /* assume + Reserve */
    if (best >= 0 && quota) or_quota_charge(quota, &pods[p]);
  }
  if (n_threads > 1) {
    atomic_store(&c.stop, 1);
    barrier_wait(&c);
    for (int t = 0; t < n_threads - 1; t++) pthread_join(th[t], NULL);
    free(th);
  }
  free(c.feasible);
  free(c.total);
  free(c.affinity);
  free(c.ds_raw);
  return rc;
}

int or_node_keys(const kg_config* cfg, const kg_node* nodes, const kg_node_metric* metrics,
                 const or_node_state* st, const kg_pod* pod, int64_t now, int64_t lo, int64_t hi,
                 uint64_t* out_keys) {
  sched_ctx c;
  memset(&c, 0, sizeof(c));
  c.cfg = cfg; c.nodes = nodes; c.metrics = metrics; c.st = (or_node_state*)st; c.now = now; c.pod = pod;
  c.feasible = (int32_t*)calloc((size_t)(hi > 0 ? hi : 1), sizeof(int32_t)); /* indexed by node, like or_schedule */
  c.total = (int64_t*)calloc((size_t)(hi > 0 ? hi : 1), sizeof(int64_t));
  if (!c.feasible || !c.total) { free(c.feasible); free(c.total); return KG_E_NOMEM; }
  int rc = 0;
  for (int64_t i = lo; i < hi && rc == 0; i++) {
    eval_filter(&c, i);
    if (c.feasible[i] == 1) eval_score(&c, i);
    if (c.feasible[i] < 0) { rc = KG_E_UNSUPPORTED; break; }
    out_keys[i - lo] = c.feasible[i] == 1
                           ? (((uint64_t)(uint32_t)c.total[i] << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)i))
                           : 0;
  }
  free(c.feasible);
  free(c.total);
  return rc;
}
