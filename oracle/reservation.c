/*
 * reservation.c — CPU restatement of the Reservation plugin (TEST INFRASTRUCTURE ONLY; see reservation.h).
 * Resources are cpu (milli) and memory (bytes); a reservation's allocatable of 0 means the key is absent
 * (ResourceNames ⊆ {cpu, memory}: cpu-only and memory-only reservations).
 */
#include "reservation.h"

#include "defaults.h"
#include "numa.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "deviceshare.h"

#define OR_DEFAULT_MILLI_CPU 100LL             /* schedutil.DefaultMilliCPURequest */
#define OR_DEFAULT_MEMORY (200LL * 1024 * 1024) /* schedutil.DefaultMemoryRequest   */

static int slot_usable(const kg_node_reservations* r, int s) {
  /* forEachAvailableReservationOnNode + IsAvailable/ParseError + AllocateOnce skip (transformer.go:101-110) */
  if (!r->available[s]) return 0;
  if (r->allocate_once[s] && r->assigned[s] > 0) return 0;
  return 1;
}

/* RequiredReservationAffinity.Match (pkg/util/reservation/reservation.go:476-489) on matchReservation's fakeNode — the
 * node's labels overlaid with the reservation's (transformer.go:353-369) — as the caller's predicate bits of the slot:
 * the ReservationSelector's predicates all hold, and one ReservationSelectorTerm holds when any are given (an empty
 * term matches nothing, nodeaffinity.NodeSelector) */
static int affinity_matches(const kg_pod* pod, uint64_t pred) {
  if (!(pod->reservation_flags & KG_POD_RSV_AFFINITY)) return 1;
  if ((pred & pod->reservation_selector) != pod->reservation_selector) return 0;
  if (pod->n_reservation_terms <= 0) return 1;
  for (int64_t t = 0; t < pod->n_reservation_terms && t < KG_MAX_AFF_TERMS; t++) {
    const uint64_t term = pod->reservation_terms[t];
    if (term != 0 && (pred & term) == term) return 1;
  }
  return 0;
}

static int pod_matches(const kg_pod* pod, const kg_node_reservations* r, int s) {
  /* matchReservation (transformer.go:348-372): ReservationInfo.Match → MatchReservationOwners
   * (reservation_info.go:231-236) decoded per owner group — bit g of the pod's mask —, !IsUnschedulable
   * (transformer.go:112), and the pod's required reservation affinity on the slot's labels */
  const int64_t g = r->owner[s];
  if (pod->flags & KG_POD_RESERVE) return 0; /* isReservedPod: a reserve pod matches no reservation (:112) */
  return g >= 0 && g < KG_MAX_OWNER_GROUPS && (((uint64_t)pod->reservation_owner_mask >> g) & 1u) &&
         !r->unschedulable[s] && affinity_matches(pod, r->predicates[s]);
}

/* Reservation.Filter of a reserve pod or a pod in reservation operating mode (reservation/plugin.go:324-350): the
 * reservation's node name, then forEachAvailableReservationOnNode — Default coexists with no other allocate policy
 * (a reserve pod brings its reservation's policy, operating mode Aligned).  1 = pass. */
int or_rsv_policy_filter(const kg_pod* pod, int64_t node_idx, const kg_node_reservations* r) {
  const int reserve = (pod->flags & KG_POD_RESERVE) != 0;
  if (!reserve && !(pod->reservation_flags & KG_POD_RSV_OPERATING)) return 1;
  int64_t pol = KG_RSV_POLICY_ALIGNED;
  if (reserve) {
    if (pod->reserve_node > 0 && pod->reserve_node - 1 != node_idx) return 0;
    pol = pod->reserve_allocate_policy;
  }
  if (!r) return 1;
  for (int64_t s = 0; s < r->n; s++) {
    if (!r->available[s]) continue;
    if ((pol == KG_RSV_POLICY_DEFAULT || r->policy[s] == KG_RSV_POLICY_DEFAULT) && pol != r->policy[s]) return 0;
  }
  return 1;
}

/* GetNonzeroRequests of the reserve pod (requests = Allocatable): an absent key takes the default */
static int64_t nz_cpu_of(const kg_node_reservations* r, int s) {
  return r->allocatable_cpu[s] > 0 ? r->allocatable_cpu[s] : OR_DEFAULT_MILLI_CPU;
}
static int64_t nz_mem_of(const kg_node_reservations* r, int s) {
  return r->allocatable_mem[s] > 0 ? r->allocatable_mem[s] : OR_DEFAULT_MEMORY;
}

static int64_t sub_nn(int64_t a, int64_t b) { return a - b > 0 ? a - b : 0; } /* SubtractWithNonNegativeResult */

void or_rsv_restore(const kg_node_reservations* r, const or_node_state* st, const kg_pod* pod, or_rsv_node* out) {
  memset(out, 0, sizeof(*out));
  out->requested[0] = st->requested[KG_RES_CPU];
  out->requested[1] = st->requested[KG_RES_MEMORY];
  out->nonzero[0] = st->nonzero[0];
  out->nonzero[1] = st->nonzero[1];
  out->num_pods = st->num_pods;
  if (!r) return;
  int32_t* unmatched = out->unmatched;
  int n_unmatched = 0;
  for (int s = 0; s < (int)r->n; s++) {
    if (!slot_usable(r, s)) continue;
    if (pod_matches(pod, r, s)) out->matched[out->n_matched++] = s;
    else if (r->assigned[s] > 0) unmatched[n_unmatched++] = s;
  }
  out->n_unmatched = n_unmatched;
  if (out->n_matched == 0 && n_unmatched == 0) return;
  /* reservationAffinity != nil && no matched: the node is not processed (transformer.go:134-136) */
  if ((pod->reservation_flags & KG_POD_RSV_AFFINITY) && out->n_matched == 0) return;
  out->has_state = 1;
  /* restoreUnmatchedReservations (transformer.go:265-291): the reserve pod (requests = allocatable, both keys
   * present so NonZero = requests) leaves; its remainder returns when non-zero */
  for (int k = 0; k < n_unmatched; k++) {
    const int s = unmatched[k];
    out->requested[0] -= r->allocatable_cpu[s];
    out->requested[1] -= r->allocatable_mem[s];
    out->nonzero[0] -= nz_cpu_of(r, s);
    out->nonzero[1] -= nz_mem_of(r, s);
    const int64_t rc = sub_nn(r->allocatable_cpu[s], r->allocated_cpu[s]);
    const int64_t rm = sub_nn(r->allocatable_mem[s], r->allocated_mem[s]);
    if (rc != 0 || rm != 0) {
      /* the remainder pod's requests carry the reservation's keys (even a zero value): a present key keeps its
       * value in GetNonzeroRequests, an absent one takes the default */
      out->requested[0] += rc;
      out->requested[1] += rm;
      out->nonzero[0] += r->allocatable_cpu[s] > 0 ? rc : OR_DEFAULT_MILLI_CPU;
      out->nonzero[1] += r->allocatable_mem[s] > 0 ? rm : OR_DEFAULT_MEMORY;
    }
  }
  out->pod_requested[0] = out->requested[0];
  out->pod_requested[1] = out->requested[1];
  /* restoreMatchedReservation (transformer.go:240-263): NodeInfo.RemovePod(reserve pod) */
  for (int k = 0; k < out->n_matched; k++) {
    const int s = out->matched[k];
    out->requested[0] -= r->allocatable_cpu[s];
    out->requested[1] -= r->allocatable_mem[s];
    out->nonzero[0] -= nz_cpu_of(r, s);
    out->nonzero[1] -= nz_mem_of(r, s);
    out->num_pods -= 1;
    out->r_allocated[0] += r->allocated_cpu[s];
    out->r_allocated[1] += r->allocated_mem[s];
  }
}

/* reservationCache.forgetPod → ReservationInfo.RemoveAssignedPod (reservation_info.go:328-339): Allocated −=
 * Mask(requests, ResourceNames) with a non-negative result, and the pod leaves AssignedPods */
void or_rsv_forget(kg_node_reservations* r, int s, const kg_pod* pod) {
  if (s < 0 || s >= (int)r->n || r->assigned[s] <= 0) return;
  if (r->allocatable_cpu[s] > 0) r->allocated_cpu[s] = sub_nn(r->allocated_cpu[s], pod->requests[KG_RES_CPU]);
  if (r->allocatable_mem[s] > 0) r->allocated_mem[s] = sub_nn(r->allocated_mem[s], pod->requests[KG_RES_MEMORY]);
  r->assigned[s] -= 1;
}

int or_rsv_fits_node(const kg_pod* pod, int64_t allowed_pods, const int64_t alloc[2], const or_rsv_node* ns,
                     const kg_node_reservations* r, int s) {
  if (ns->num_pods - ns->n_matched + 1 > allowed_pods) return 0;
  const int64_t pc = pod->requests[KG_RES_CPU], pm = pod->requests[KG_RES_MEMORY];
  if (pc == 0 && pm == 0) return 1;
  int64_t rc = 0, rm = 0;
  if (s >= 0) {
    rc = sub_nn(r->allocatable_cpu[s], r->allocated_cpu[s]);
    rm = sub_nn(r->allocatable_mem[s], r->allocated_mem[s]);
  }
  if (pc > alloc[0] - (ns->pod_requested[0] - rc - ns->r_allocated[0])) return 0;
  if (pm > alloc[1] - (ns->pod_requested[1] - rm - ns->r_allocated[1])) return 0;
  return 1;
}

int or_rsv_filter_with(const kg_pod* pod, int64_t allowed_pods, const int64_t alloc[2], const or_rsv_node* ns,
                       const kg_node_reservations* r, const int32_t* slots, int n_slots, int required) {
  const int64_t pc = pod->requests[KG_RES_CPU], pm = pod->requests[KG_RES_MEMORY];
  const int kc = or_pod_cpu_key(pod), km = or_pod_mem_key(pod);
  int satisfied = 0;
  for (int k = 0; k < n_slots && !satisfied; k++) {
    const int s = slots[k];
    const int hc = r->allocatable_cpu[s] > 0, hm = r->allocatable_mem[s] > 0;
    if (!((kc && hc) || (km && hm))) continue; /* Intersection(ResourceNames, pod request names) empty */
    const int fits = or_rsv_fits_node(pod, allowed_pods, alloc, ns, r, s);
    if (r->policy[s] == KG_RSV_POLICY_RESTRICTED) {
      /* LessThanOrEqual(podRequests, rRemained): the reservation's keys the pod requests */
      const int64_t rc = sub_nn(r->allocatable_cpu[s], r->allocated_cpu[s]);
      const int64_t rm = sub_nn(r->allocatable_mem[s], r->allocated_mem[s]);
      if ((!hc || !kc || pc <= rc) && (!hm || !km || pm <= rm) && fits) satisfied = 1;
    } else if (fits) {
      satisfied = 1;
    }
  }
  return (!satisfied && required) ? 0 : 1;
}

int or_rsv_filter(const kg_pod* pod, int64_t allowed_pods, const int64_t alloc[2], const or_rsv_node* ns,
                  const kg_node_reservations* r) {
  if (pod->flags & KG_POD_RESERVE) return 1; /* the matched-reservation part skips reserve pods (plugin.go:357) */
  const int required = (pod->reservation_flags & KG_POD_RSV_AFFINITY) != 0;
  if (ns->n_matched == 0 || !ns->has_state) return required ? 0 : 1;
  return or_rsv_filter_with(pod, allowed_pods, alloc, ns, r, ns->matched, ns->n_matched, required);
}

int64_t or_rsv_score_slot(const kg_pod* pod, const kg_node_reservations* r, int s) {
  const int64_t req[2] = {pod->requests[KG_RES_CPU] + r->allocated_cpu[s],
                          pod->requests[KG_RES_MEMORY] + r->allocated_mem[s]};
  const int64_t cap[2] = {r->allocatable_cpu[s], r->allocatable_mem[s]};
  int64_t w = 0, sc = 0;
  for (int k = 0; k < 2; k++) {
    if (cap[k] == 0) continue; /* RemoveZeros */
    w++;
    if (req[k] <= cap[k]) sc += 100 * req[k] / cap[k]; /* MaxNodeScore · MilliValue / MilliValue */
  }
  return w > 0 ? sc / w : 0;
}

int64_t or_rsv_node_order(const or_rsv_node* ns, const kg_node_reservations* r) {
  int64_t best = INT64_MAX;
  for (int k = 0; k < ns->n_matched; k++) {
    const int64_t o = r->order[ns->matched[k]];
    if (o != 0 && best > o) best = o;
  }
  return best;
}

int or_rsv_nominate(const kg_pod* pod, int64_t allowed_pods, const int64_t alloc[2], const or_rsv_node* ns,
                    const kg_node_reservations* r) {
  return or_rsv_nominate_ds(pod, allowed_pods, alloc, ns, r, NULL, NULL, NULL, 0, NULL);
}

int or_rsv_nominate_ds(const kg_pod* pod, int64_t allowed_pods, const int64_t alloc[2], const or_rsv_node* ns,
                       const kg_node_reservations* r, const kg_node_device* dev, const struct or_ds_pod* dsp,
                       const struct or_ds_rsv* dst, int strategy, const int64_t w[3]) {
  if (pod->flags & KG_POD_RESERVE) return -1; /* NominateReservation: none for a reserve pod (nominator.go:77) */
  if (!ns->has_state || ns->n_matched == 0) return -1;
  const int ds = dev && dsp && dst && !dsp->skip;
  int32_t cand[KG_MAX_RSV_SLOTS];
  int n = 0;
  for (int k = 0; k < ns->n_matched; k++) {
    const int s = ns->matched[k];
    /* FilterReservation (plugin.go:492-519): AllocateOnce already excluded; filterWithReservations([s], true) */
    const int32_t one = s;
    if (!or_rsv_filter_with(pod, allowed_pods, alloc, ns, r, &one, 1, 1)) continue;
    /* (ABI 13) DeviceShare.FilterReservation (deviceshare/plugin.go:333-380) */
    if (ds && !or_ds_filter_reservation(dev, dsp, r, dst, s)) continue;
    cand[n++] = s;
  }
  if (n == 0) return -1;
  int64_t best_order = INT64_MAX;
  int pick = -1;
  for (int k = 0; k < n; k++) {
    const int64_t o = r->order[cand[k]];
    if (o != 0 && best_order > o) { best_order = o; pick = cand[k]; }
  }
  if (pick >= 0) return pick;
  /* prioritizeReservations: Σ over the reservation score plugins — Reservation (no normalizer) + DeviceShare
   * (scoreWithNominatedReservation, then DefaultReservationNormalizeScore: 100·s / max over the candidates) */
  int64_t dsc[KG_MAX_RSV_SLOTS] = {0}, dmax = 0;
  if (ds)
    for (int k = 0; k < n; k++) {
      dsc[k] = or_ds_score_slot(dev, dsp, r, dst, cand[k], strategy, w);
      if (dsc[k] > dmax) dmax = dsc[k];
    }
  int64_t best = -1;
  for (int k = 0; k < n; k++) {
    const int64_t sc = or_rsv_score_slot(pod, r, cand[k]) + (dmax > 0 ? 100 * dsc[k] / dmax : 0);
    if (sc > best) { best = sc; pick = cand[k]; } /* sort.Slice unstable → pinned: lowest slot on ties */
  }
  return pick;
}

void or_rsv_case_flat(const kg_pod* pod, int64_t allowed_pods, const int64_t alloc[2], int64_t num_pods,
                      const int64_t pod_requested[2], const int64_t r_allocated[2], int has_state,
                      const kg_node_reservations* r, int64_t* out) {
  or_rsv_node ns;
  memset(&ns, 0, sizeof(ns));
  ns.has_state = has_state;
  for (int s = 0; s < (int)r->n; s++) ns.matched[ns.n_matched++] = s; /* the tests place every slot in matched */
  ns.num_pods = num_pods;
  for (int k = 0; k < 2; k++) { ns.pod_requested[k] = pod_requested[k]; ns.r_allocated[k] = r_allocated[k]; }
  out[0] = or_rsv_filter(pod, allowed_pods, alloc, &ns, r);
  const int nom = or_rsv_nominate(pod, allowed_pods, alloc, &ns, r);
  out[1] = nom;
  out[2] = nom >= 0 ? or_rsv_score_slot(pod, r, nom) : 0;
}

int or_schedule_resv(const kg_config* cfg, int64_t n_nodes, const kg_node* nodes, const kg_node_metric* metrics,
                     or_node_state* st, kg_node_reservations* rsv, int64_t n_pods, const kg_pod* pods, int64_t now,
                     int32_t* out_node, int64_t* out_score, int32_t* out_slot) {
  return or_schedule_resv_full(cfg, n_nodes, nodes, metrics, st, rsv, NULL, NULL, 0, n_pods, pods, now, 1, out_node,
                               out_score, out_slot, NULL, NULL, NULL, NULL, NULL, NULL);
}

int or_schedule_resv_full(const kg_config* cfg, int64_t n_nodes, const kg_node* nodes, const kg_node_metric* metrics,
                          or_node_state* st, kg_node_reservations* rsv, kg_node_device* dev, kg_quota* quotas,
                          int64_t n_quotas, int64_t n_pods, const kg_pod* pods, int64_t now, int n_threads,
                          int32_t* out_node, int64_t* out_score, int32_t* out_slot, int32_t* out_minors,
                          void* numa_states, uint64_t* out_cpus, int64_t* out_numa, const kg_node_predicates* preds,
                          void* groups) {
  const size_t nn = (size_t)(n_nodes > 0 ? n_nodes : 1);
  or_group_node* grp = (or_group_node*)groups;
  const int spread_on = grp && (cfg->spread_filter || cfg->spread_score);
  const int ipa_on = grp && (cfg->interpod_filter || cfg->interpod_score);
  int64_t* scnt = (int64_t*)calloc(nn, sizeof(int64_t)); /* PodTopologySpread: the soft constraint's count */
  int64_t* iraw = (int64_t*)calloc(nn, sizeof(int64_t)); /* InterPodAffinity raw Score */
  if (!scnt || !iraw) { free(scnt); free(iraw); return KG_E_NOMEM; }
  or_numa_node* numa = (or_numa_node*)numa_states;
  const int numa_on = numa && (cfg->numa_filter || cfg->numa_score);
  or_hint* aff = numa_on ? (or_hint*)calloc(nn, sizeof(or_hint)) : NULL;
  if (numa_on && !aff) return KG_E_NOMEM;
  int8_t* feas = (int8_t*)malloc(nn);
  int64_t* base = (int64_t*)malloc(nn * sizeof(int64_t));
  int64_t* raw = (int64_t*)malloc(nn * sizeof(int64_t));
  int64_t* dsraw = (int64_t*)malloc(nn * sizeof(int64_t));
  int64_t* order = (int64_t*)malloc(nn * sizeof(int64_t));
  int32_t* nom = (int32_t*)malloc(nn * sizeof(int32_t));
  int64_t* tcnt = (int64_t*)calloc(nn, sizeof(int64_t));
  int64_t* asum = (int64_t*)calloc(nn, sizeof(int64_t));
  if (!feas || !base || !raw || !dsraw || !order || !nom || !tcnt || !asum) {
    free(feas); free(base); free(raw); free(dsraw); free(order); free(nom); free(aff); free(tcnt); free(asum);
    return KG_E_NOMEM;
  }
  /* TaintToleration / NodeAffinity / BalancedAllocation (defaults.c); a NULL table = no predicates, no taints */
  const kg_node_predicates zero_pred = {0, 0, 0, 0, 0, 0, 0};
  const int rsv_on = cfg->reservation_filter || cfg->reservation_score;
  const int ds_on = dev && (cfg->ds_filter || cfg->ds_score);
  /* (r6) the cpus a reservation and one of its assigned pods both hold have RefCount 2 in NodeAllocation */
  if (numa_on && rsv_on)
    for (int64_t i = 0; i < n_nodes; i++) or_numa_rsv_refs(&numa[i], &rsv[i]);
  if (n_threads < 1) n_threads = 1;
  /* chunkSizeFor (pkg/util/parallelize/parallelism.go:35-46) with parallelism = n_threads */
  int64_t chunk = (int64_t)sqrt((double)n_nodes), lim = n_nodes / n_threads + 1;
  if (chunk > lim) chunk = lim;
  if (chunk < 1) chunk = 1;
  int rc = 0;
  for (int64_t p = 0; p < n_pods && rc == 0; p++) {
    const kg_pod* pod = &pods[p];
    if (out_slot) out_slot[p] = -1;
    if (out_minors) out_minors[p] = 0;
    if (out_cpus) memset(&out_cpus[p * OR_CPUSET_WORDS], 0, sizeof(uint64_t) * OR_CPUSET_WORDS);
    if (out_numa) memset(&out_numa[p * OR_NUMA_ALLOC_WORDS], 0, sizeof(int64_t) * OR_NUMA_ALLOC_WORDS);
    /* ElasticQuota PreFilter: a rejected pod is Unschedulable without a node search */
    kg_quota* quota = NULL;
    if (pod->quota_id > 0) {
      if (pod->quota_id > n_quotas || !quotas) { rc = KG_E_INVALID; break; }
      quota = &quotas[pod->quota_id - 1];
      if (!or_quota_admit(quota, pod)) {
        out_node[p] = -1;
        out_score[p] = 0;
        continue;
      }
    }
    or_ds_pod dsp;
    memset(&dsp, 0, sizeof(dsp));
    dsp.skip = 1;
    if (ds_on) {
      or_ds_pod_init(pod, &dsp);
      if (dsp.unsupported) { rc = KG_E_UNSUPPORTED; break; }
    }
    /* (ABI 13) DeviceShare with reservations holding GPUs: the plugin's restore per node (or_ds_rsv_init over the
     * Reservation restore's matched / unmatched slots), its Filter / FilterReservation / ScoreReservation / Score /
     * Reserve (deviceshare.c) */
    const int ds_rsv = ds_on && !dsp.skip;
    const int required_from_rsv = (pod->reservation_flags & KG_POD_RSV_AFFINITY) != 0;
    or_numa_pod npod;
    if (numa_on) or_numa_pod_init(cfg, pod, &npod);
    /* PodTopologySpread PreFilter (common.go calPreFilterState) over the nodes passing the pod's nodeSelector /
     * required node affinity and carrying every DoNotSchedule key: per constraint, TpPairToMatchNum — each such node's
     * own count (hostname) or its zone's sum (zone) — and the minimum over those pairs (MaxInt32 when none);
     * InterPodAffinity PreFilter / PreScore: the pod's topology-pair maps (or_ipa_zones: the zone pairs and whether
     * affinityCounts has any pair) */
    int64_t min_match[KG_MAX_SPREAD], zsum_f[KG_MAX_SPREAD][KG_MAX_ZONES];
    uint64_t zpres_f[KG_MAX_SPREAD] = {0};
    or_ipa_zones ipz;
    memset(&ipz, 0, sizeof(ipz));
    memset(zsum_f, 0, sizeof(zsum_f));
    for (int c = 0; c < KG_MAX_SPREAD; c++) min_match[c] = INT32_MAX;
    if (spread_on || ipa_on) {
      for (int64_t i = 0; i < n_nodes; i++) {
        if (!(nodes[i].flags & KG_NODE_VALID)) continue;
        const kg_node_predicates* np = preds ? &preds[i] : &zero_pred;
        if (ipa_on) or_ipa_zones_add(&ipz, &grp[i], np->zone, pod);
        if (!spread_on || !or_spread_node_ok(np, pod, 1)) continue;
        for (int64_t c = 0; c < pod->n_spread; c++) {
          if (!(pod->spread_flags[c] & KG_SPREAD_HARD)) continue;
          const int64_t v = grp[i].cnt[pod->spread_group[c] - 1];
          if (pod->spread_flags[c] & KG_SPREAD_ZONE) {
            zsum_f[c][np->zone - 1] += v;
            zpres_f[c] |= 1ull << (np->zone - 1);
          } else if (v < min_match[c]) {
            min_match[c] = v;
          }
        }
      }
      for (int64_t c = 0; c < pod->n_spread; c++)
        if (pod->spread_flags[c] & KG_SPREAD_ZONE)
          for (int z = 0; z < KG_MAX_ZONES; z++)
            if (((zpres_f[c] >> z) & 1) && zsum_f[c][z] < min_match[c]) min_match[c] = zsum_f[c][z];
    }
    int err = 0;
#pragma omp parallel for schedule(dynamic, chunk) num_threads(n_threads) reduction(min : err)
    for (int64_t i = 0; i < n_nodes; i++) {
      feas[i] = 0;
      const kg_node* nd = &nodes[i];
      if (!(nd->flags & KG_NODE_VALID)) continue;
      const kg_node_predicates* np = preds ? &preds[i] : &zero_pred;
      if (cfg->taint_filter && !or_taint_filter(np, pod)) continue;
      if (cfg->affinity_filter && !or_affinity_filter(np, pod)) continue;
      or_rsv_node ns;
      or_rsv_restore(rsv_on ? &rsv[i] : NULL, &st[i], pod, &ns);
      or_node_state rs = st[i];
      rs.requested[KG_RES_CPU] = ns.requested[0];
      rs.requested[KG_RES_MEMORY] = ns.requested[1];
      rs.nonzero[0] = ns.nonzero[0];
      rs.nonzero[1] = ns.nonzero[1];
      rs.num_pods = ns.num_pods;
      const int64_t alloc[2] = {nd->allocatable[KG_RES_CPU], nd->allocatable[KG_RES_MEMORY]};
      if (cfg->fit_filter && or_fit_filter(nd, &rs, pod) != 0) continue;
      if (cfg->la_filter) {
        const int f = or_loadaware_filter(cfg, nd, &metrics[i], pod, now);
        if (f < 0) { err = f; continue; }
        if (f != 0) continue;
      }
      if (cfg->reservation_filter && !or_rsv_policy_filter(pod, i, rsv_on ? &rsv[i] : NULL)) continue;
      if (cfg->reservation_filter && !or_rsv_filter(pod, nd->allowed_pods, alloc, &ns, &rsv[i])) continue;
      or_ds_rsv dst;
      memset(&dst, 0, sizeof(dst));
      if (ds_rsv && rsv_on && ns.has_state)
        or_ds_rsv_init(&rsv[i], ns.matched, ns.n_matched, ns.unmatched, ns.n_unmatched, &dst);
      if (ds_on && cfg->ds_filter && !or_ds_filter_rsv(&dev[i], &dsp, rsv_on ? &rsv[i] : NULL, &dst, required_from_rsv))
        continue;
      /* NodeNUMAResource Filter (nodenumaresource/plugin.go:276-334) on the restored NodeInfo; the reserve pods hold
       * no cpuset, so its RestoreReservation (nodenumaresource/reservation.go) restores nothing */
      if (numa_on) {
        aff[i] = (or_hint){1, 0, 0, 0};
        if (cfg->numa_filter &&
            !or_numa_filter(cfg, &numa[i], &npod, &aff[i], rs.requested[KG_RES_CPU], nd->allocatable[KG_RES_CPU]))
          continue;
      }
      if (spread_on && cfg->spread_filter) { /* filtering.go Filter */
        int ok = 1;
        const int elig = or_spread_node_ok(np, pod, 1);
        for (int64_t c = 0; c < pod->n_spread && ok; c++) {
          if (!(pod->spread_flags[c] & KG_SPREAD_HARD)) continue;
          const int64_t g = pod->spread_group[c] - 1;
          int64_t match;
          if (pod->spread_flags[c] & KG_SPREAD_ZONE) {
            if (np->zone <= 0) { ok = 0; break; } /* the node lacks the constraint's key */
            match = ((zpres_f[c] >> (np->zone - 1)) & 1) ? zsum_f[c][np->zone - 1] : 0;
          } else {
            match = elig ? grp[i].cnt[g] : 0;
          }
          const int64_t self = (pod->match_groups >> g) & 1;
          if (match + self - min_match[c] > pod->spread_max_skew[c]) ok = 0;
        }
        if (!ok) continue;
      }
      if (ipa_on && cfg->interpod_filter && !or_interpod_filter(&grp[i], pod, np->zone, &ipz)) continue;
      feas[i] = 1;
      iraw[i] = ipa_on ? or_interpod_raw(&grp[i], pod, np->zone, &ipz) : 0;
      int64_t t = 0;
      if (cfg->fit_score) t += cfg->weight_fit * or_fit_score(cfg, nd, &rs, pod);
      if (cfg->la_score) {
        const int64_t sc = or_loadaware_score(cfg, nd, &metrics[i], &st[i], pod, now);
        if (sc < 0) { err = (int)sc; continue; }
        t += cfg->weight_loadaware * sc;
      }
      int64_t nsc = 0;
      if (numa_on && cfg->numa_score) { /* scoring.go:55-93 on the restored NodeInfo with the stored affinity */
        nsc = or_numa_score(cfg, &numa[i], &npod, &aff[i], rs.requested[KG_RES_CPU], rs.requested[KG_RES_MEMORY],
                            nd->allocatable[KG_RES_CPU], nd->allocatable[KG_RES_MEMORY]);
        t += cfg->weight_numa * nsc;
      }
      if (cfg->balanced_score)
        t += cfg->weight_balanced * or_balanced_score(nd->allocatable[KG_RES_CPU], nd->allocatable[KG_RES_MEMORY],
                                                      rs.requested[KG_RES_CPU], rs.requested[KG_RES_MEMORY],
                                                      pod->requests[KG_RES_CPU], pod->requests[KG_RES_MEMORY],
                                                      cfg->balanced_resources);
      if (cfg->image_score) t += cfg->weight_image * or_image_score(np, pod);
      tcnt[i] = cfg->taint_score ? or_taint_count(np, pod) : 0;
      asum[i] = cfg->affinity_score ? or_affinity_sum(np, pod) : 0;
      base[i] = t;
      nom[i] = rsv_on ? or_rsv_nominate_ds(pod, nd->allowed_pods, alloc, &ns, &rsv[i], ds_on ? &dev[i] : NULL,
                                           ds_on ? &dsp : NULL, ds_on ? &dst : NULL, (int)cfg->ds_scoring_strategy,
                                           cfg->ds_scoring_weights)
                      : -1;
      raw[i] = nom[i] >= 0 ? or_rsv_score_slot(pod, &rsv[i], nom[i]) : 0;
      /* (r6) NodeNUMAResource Score after the PreScore nomination: getResourceOptions offers the nominated
       * reservation's reserved cpus (getReservationReservedCPUs, plugin.go:513-535; RestoreReservation
       * reservation.go:76-113, skipped unless AllowUseCPUSet) as preferredCPUs / reusable NUMA cpu */
      if (numa_on && cfg->numa_score && nom[i] >= 0 && npod.allow_cpuset && !(pod->flags & KG_POD_RESERVE)) {
        const or_cpuset pref = or_numa_rsv_reserved(&rsv[i], nom[i]);
        const int64_t psc = or_numa_score_pref(cfg, &numa[i], &npod, &aff[i], &pref, rs.requested[KG_RES_CPU],
                                               rs.requested[KG_RES_MEMORY], nd->allocatable[KG_RES_CPU],
                                               nd->allocatable[KG_RES_MEMORY]);
        base[i] += cfg->weight_numa * (psc - nsc);
      }
      order[i] = ns.has_state ? or_rsv_node_order(&ns, &rsv[i]) : INT64_MAX;
      dsraw[i] = (ds_on && cfg->ds_score && !dsp.skip)
                     ? or_ds_score_rsv(&dev[i], &dsp, rsv_on ? &rsv[i] : NULL, &dst, nom[i],
                                       (int)cfg->ds_scoring_strategy, cfg->ds_scoring_weights) +
                           or_dsx_score(&dev[i], &dsp, (int)cfg->ds_scoring_strategy, cfg->ds_scoring_weights_x)
                     : 0;
    }
    if (err) { rc = err; break; }
    /* PreScore preferredNode (scoring.go:89-99): smallest order, first (lowest index) feasible node */
    int64_t pref = -1, best_order = INT64_MAX;
    for (int64_t i = 0; i < n_nodes; i++)
      if (feas[i] && order[i] != 0 && best_order > order[i]) { best_order = order[i]; pref = i; }
    int64_t mx = 0, mds = 0, mt = 0, ma = 0;
    /* PodTopologySpread PreScore (scoring.go initPreScoreState, processAllNode): filtered nodes lacking a
     * ScheduleAnyway key are IgnoredNodes; the hostname weight is log(|filtered| − |ignored| + 2), a zone constraint's
     * log(#zones of the non-ignored filtered nodes + 2); a zone's count sums the pods of every node passing the pod's
     * node affinity and carrying every ScheduleAnyway key.  Score per node, then NormalizeScore's extremes over the
     * non-ignored filtered nodes; InterPodAffinity's extremes over the filtered nodes */
    /* (ABI 13) a system-defaulted pod (requireAllTopologies false) ignores no node: a filtered node without the zone
     * label adds the empty zone value as one more domain of a zone constraint (zone_empty) */
    const int sysdef = spread_on && or_spread_system_default(pod);
    int64_t n_feas = 0, n_ign = 0, smin = INT64_MAX, smax = INT64_MIN, imin = INT64_MAX, imax = INT64_MIN;
    int zone_empty = 0;
    uint64_t zpres_s = 0;
    for (int64_t i = 0; i < n_nodes; i++) {
      if (!feas[i]) continue;
      n_feas++;
      if (iraw[i] < imin) imin = iraw[i];
      if (iraw[i] > imax) imax = iraw[i];
      if (!spread_on) continue;
      const kg_node_predicates* np = preds ? &preds[i] : &zero_pred;
      if (!sysdef && !or_spread_has_keys(np, pod, 0)) { n_ign++; continue; }
      if (np->zone > 0) zpres_s |= 1ull << (np->zone - 1);
      else zone_empty = 1;
    }
    int64_t zsum_s[KG_MAX_SPREAD][KG_MAX_ZONES];
    double sw[KG_MAX_SPREAD] = {0};
    memset(zsum_s, 0, sizeof(zsum_s));
    if (spread_on) {
      int has_zone = 0;
      for (int64_t c = 0; c < pod->n_spread; c++) {
        if (pod->spread_flags[c] & KG_SPREAD_HARD) continue;
        if (pod->spread_flags[c] & KG_SPREAD_ZONE) {
          has_zone = 1;
          sw[c] = or_go_log((double)(__builtin_popcountll(zpres_s) + (sysdef ? zone_empty : 0) + 2));
        } else {
          sw[c] = or_go_log((double)(n_feas - n_ign + 2));
        }
      }
      if (has_zone)
        for (int64_t i = 0; i < n_nodes; i++) {
          if (!(nodes[i].flags & KG_NODE_VALID)) continue;
          const kg_node_predicates* np = preds ? &preds[i] : &zero_pred;
          if (np->zone <= 0 || !((zpres_s >> (np->zone - 1)) & 1) || !or_spread_node_ok(np, pod, 0)) continue;
          for (int64_t c = 0; c < pod->n_spread; c++)
            if ((pod->spread_flags[c] & (KG_SPREAD_HARD | KG_SPREAD_ZONE)) == KG_SPREAD_ZONE)
              zsum_s[c][np->zone - 1] += grp[i].cnt[pod->spread_group[c] - 1];
        }
      for (int64_t i = 0; i < n_nodes; i++) {
        scnt[i] = INT64_MIN; /* ignored */
        if (!feas[i]) continue;
        const kg_node_predicates* np = preds ? &preds[i] : &zero_pred;
        if (!sysdef && !or_spread_has_keys(np, pod, 0)) continue;
        int64_t cnt[KG_MAX_SPREAD] = {0};
        for (int64_t c = 0; c < pod->n_spread; c++)
          cnt[c] = (pod->spread_flags[c] & KG_SPREAD_ZONE) ? (np->zone > 0 ? zsum_s[c][np->zone - 1] : -1)
                                                           : grp[i].cnt[pod->spread_group[c] - 1];
        scnt[i] = or_spread_raw(cnt, sw, pod);
        if (scnt[i] < smin) smin = scnt[i];
        if (scnt[i] > smax) smax = scnt[i];
      }
    }
    for (int64_t i = 0; i < n_nodes; i++) {
      if (!feas[i]) continue;
      if (tcnt[i] > mt) mt = tcnt[i];
      if (asum[i] > ma) ma = asum[i];
      const int64_t sc = (i == pref) ? 1000 : raw[i]; /* mostPreferredScore */
      raw[i] = sc;
      if (sc > mx) mx = sc;
      if (dsraw[i] > mds) mds = dsraw[i];
    }
    /* RunScorePlugins: DefaultNormalizeScore (Reservation scoring.go:126-131, DeviceShare scoring.go:95-97) × weight */
    int64_t win = -1, win_total = -1;
    for (int64_t i = 0; i < n_nodes; i++) {
      if (!feas[i]) continue;
      int64_t t = base[i];
      if (cfg->reservation_score && mx > 0) t += cfg->weight_reservation * (100 * raw[i] / mx);
      if (ds_on && cfg->ds_score && mds > 0) t += cfg->weight_deviceshare * (100 * dsraw[i] / mds);
      /* TaintToleration NormalizeScore (reverse) and NodeAffinity NormalizeScore × weight */
      if (cfg->taint_score) t += cfg->weight_taint * or_normalize_default(tcnt[i], mt, 1);
      if (cfg->affinity_score) t += cfg->weight_affinity * or_normalize_default(asum[i], ma, 0);
      if (spread_on && cfg->spread_score) /* NormalizeScore: an ignored node scores 0 */
        t += cfg->weight_spread * (scnt[i] == INT64_MIN ? 0 : or_spread_normalize(scnt[i], smin, smax));
      if (ipa_on && cfg->interpod_score) t += cfg->weight_interpod * or_interpod_normalize(iraw[i], imin, imax);
      if (t > win_total) { win_total = t; win = i; }
    }
    /* Reserve in the profile's order (scheduler-config.yaml:92-98): NodeNUMAResource (the exact cpuset), then
     * DeviceShare (the minors); any failure un-assumes the pod and RunReservePluginsUnreserve releases what the earlier
     * plugins took (nodenumaresource/plugin.go:417-425), so nothing stays placed */
    or_numa_node numa_save;
    or_cpuset cpus;
    memset(&cpus, 0, sizeof(cpus));
    int64_t nalloc[OR_NUMA_ALLOC_WORDS] = {0};
    if (win >= 0 && numa_on) {
      numa_save = numa[win];
      /* (r6) the nominated reservation's reserved cpus are Reserve's preferredCPUs too (getResourceOptions) */
      or_cpuset pref;
      memset(&pref, 0, sizeof(pref));
      if (rsv_on && nom[win] >= 0 && npod.allow_cpuset && !(pod->flags & KG_POD_RESERVE))
        pref = or_numa_rsv_reserved(&rsv[win], nom[win]);
      if (or_numa_reserve_pref(cfg, &numa[win], &npod, &aff[win], &pref, &cpus, nalloc) != 0) {
        numa[win] = numa_save;
        win = -1;
      }
    }
    int32_t minors = 0;
    if (win >= 0 && ds_on && !dsp.skip) {
      /* the winner's DeviceShare restore again (the per-node state of the Filter pass above) */
      or_rsv_node wns;
      or_ds_rsv wdst;
      memset(&wdst, 0, sizeof(wdst));
      if (rsv_on) {
        or_rsv_restore(&rsv[win], &st[win], pod, &wns);
        if (wns.has_state) or_ds_rsv_init(&rsv[win], wns.matched, wns.n_matched, wns.unmatched, wns.n_unmatched, &wdst);
      }
      minors = or_ds_reserve_rsv(&dev[win], &dsp, rsv_on ? &rsv[win] : NULL, &wdst, rsv_on ? nom[win] : -1,
                                 (int)cfg->ds_scoring_strategy, cfg->ds_scoring_weights);
      if (minors >= 0) { /* (ABI 17) the RDMA / FPGA types: all of them or none */
        const int32_t xm = or_dsx_reserve(&dev[win], &dsp, (int)cfg->ds_scoring_strategy, cfg->ds_scoring_weights_x);
        if (xm < 0) {
          or_ds_release(&dev[win], &dsp, minors);
          minors = -1;
        } else {
          minors |= xm;
        }
      }
      if (minors < 0) {
        minors = 0;
        if (numa_on) numa[win] = numa_save;
        win = -1;
      }
    }
    if (win >= 0 && out_cpus) memcpy(&out_cpus[p * OR_CPUSET_WORDS], cpus.w, sizeof(uint64_t) * OR_CPUSET_WORDS);
    if (win >= 0 && out_numa) memcpy(&out_numa[p * OR_NUMA_ALLOC_WORDS], nalloc, sizeof(nalloc));
    out_node[p] = (int32_t)win;
    out_score[p] = win >= 0 ? win_total : 0;
    if (out_minors) out_minors[p] = minors;
    if (win >= 0) {
      or_assume_pod(cfg, &st[win], pod, 1); /* assume + LoadAware Reserve (a reserve pod too) */
      if (rsv_on && nom[win] >= 0) {
        /* Reserve → reservationCache.assumePod → AddAssignedPod (reservation_info.go:317-326) */
        kg_node_reservations* r = &rsv[win];
        const int s = nom[win];
        /* Allocated += quotav1.Mask(requests, ResourceNames): only the reservation's own keys (0 = absent) */
        if (r->allocatable_cpu[s] > 0) r->allocated_cpu[s] += pod->requests[KG_RES_CPU];
        if (r->allocatable_mem[s] > 0) r->allocated_mem[s] += pod->requests[KG_RES_MEMORY];
        r->assigned[s] += 1;
        /* (ABI 13) the reservation's allocated GPUs: the pod's allocation on the reservation's minors */
        if (ds_on && minors > 0) or_ds_rsv_assign(r, s, &dev[win], &dsp, minors, 1);
        /* (ABI 15) an assigned pod's cpus leave the reservation's reserved cpus at the next RestoreReservation */
        int holds = 0;
        for (int w = 0; w < OR_CPUSET_WORDS; w++) holds |= r->cpus[s][w] != 0;
        if (numa_on && holds)
          for (int w = 0; w < OR_CPUSET_WORDS; w++) r->cpus_assigned[s][w] |= cpus.w[w];
        if (out_slot) out_slot[p] = nom[win];
      }
      if (quota) or_quota_charge(quota, pod);
      if (grp) or_groups_apply(&grp[win], pod, 1, cfg->hard_pod_affinity_weight);
    }
  }
  free(feas); free(base); free(raw); free(dsraw); free(order); free(nom); free(aff); free(tcnt); free(asum);
  free(scnt); free(iraw);
  return rc;
}

/* Test hook: BeforePreFilter's restore of one node (or_rsv_restore) as flat values: [0] has_state, [1] matched slot
 * mask, [2..3] restored Requested cpu / memory, [4..5] NonZeroRequested, [6] pod count, [7..8] podRequested,
 * [9..10] Σ matched Allocated.  Pins transformer.go's restore with transformer_test.go's tables. */
void or_rsv_restore_flat(const kg_node_reservations* r, const or_node_state* st, const kg_pod* pod, int64_t* out) {
  or_rsv_node ns;
  or_rsv_restore(r, st, pod, &ns);
  int64_t m = 0;
  for (int k = 0; k < ns.n_matched; k++) m |= 1LL << ns.matched[k];
  out[0] = ns.has_state;
  out[1] = m;
  out[2] = ns.requested[0], out[3] = ns.requested[1];
  out[4] = ns.nonzero[0], out[5] = ns.nonzero[1];
  out[6] = ns.num_pods;
  out[7] = ns.pod_requested[0], out[8] = ns.pod_requested[1];
  out[9] = ns.r_allocated[0], out[10] = ns.r_allocated[1];
}

/* The preemption dry run's per-candidate state: the restored NodeInfo copy minus the removed victims and the
 * Reservation plugin's preemptible maps (PreFilterExtensions RemovePod / AddPod, reservation/plugin.go:253-310: a
 * non-reserve victim with non-zero requests adds (RemovePod) or subtracts (AddPod) its requests — every resource, so
 * ephemeral-storage and the scalars too — to state.preemptible[node] or preemptibleInRRs[node][its reservation]; either
 * call sets the map entry, which then stays non-empty).  (r6) DeviceShare's preemptibleDevices[node] per minor. */
typedef struct {
  or_node_state rs;   /* the NodeInfo copy the Filters see */
  or_rsv_node ns;     /* nodeReservationState (restore-time podRequested / rAllocated, untouched by the victims) */
  int64_t pre[KG_RES_MAX], pre_rr[KG_MAX_RSV_SLOTS][KG_RES_MAX];
  int pre_set, pre_rr_set;
  const or_pre_ext* x;
  or_ds_pod dsp;                        /* the preemptor's DeviceShare preFilterState */
  int64_t dpre[KG_MAX_MINORS][3];       /* preemptibleDevices[node]: gpu-core, gpu-memory, gpu-memory-ratio */
  int64_t xpre[KG_DEV_XTYPES][KG_MAX_MINORS]; /* (ABI 17) its RDMA / FPGA part */
  or_numa_node nn;                      /* the node's NodeAllocation (victims' cpusets kept) */
  or_numa_pod np;
} pre_node;

static void pre_node_init(pre_node* S, const kg_config* cfg, const or_node_state* st, const kg_node_reservations* rsv,
                          const kg_pod* pod, const or_pre_ext* x) {
  const int rsv_on = cfg->reservation_filter || cfg->reservation_score;
  memset(S, 0, sizeof(*S));
  or_rsv_restore(rsv_on ? rsv : NULL, st, pod, &S->ns);
  S->rs = *st;
  S->rs.requested[KG_RES_CPU] = S->ns.requested[0];
  S->rs.requested[KG_RES_MEMORY] = S->ns.requested[1];
  S->rs.nonzero[0] = S->ns.nonzero[0];
  S->rs.nonzero[1] = S->ns.nonzero[1];
  S->rs.num_pods = S->ns.num_pods;
  S->x = x;
  S->dsp.skip = 1;
  if (x && x->dev) or_ds_pod_init(pod, &S->dsp);
  if (x && x->numa) {
    or_numa_node_init(&S->nn, x->numa);
    or_numa_pod_init(cfg, pod, &S->np);
  }
}

/* sign +1: NodeInfo.RemovePod + RemovePod; -1: NodeInfo.AddPodInfo + AddPod */
static void pre_node_apply(pre_node* S, const kg_pod* v, int slot, int32_t minors, int64_t sign) {
  /* (r6) DeviceShare AddPod / RemovePod: reserve pods and state.skip return first; no allocation on the node
   * (getUsed empty) returns; a victim allocated from a reservation goes to preemptibleInRRs */
  if (S->x && S->x->dev && !S->dsp.skip && minors != 0 && !(v->flags & KG_POD_RESERVE) && slot < 0) {
    or_ds_pod vp;
    or_ds_pod_init(v, &vp);
    const or_ds_inst in = (minors & 0xFF) && !vp.nogpu ? or_ds_instance(S->x->dev, &vp) : (or_ds_inst){0, 0, 0, 0, 0};
    if (in.ok)
      for (int m = 0; m < KG_MAX_MINORS; m++)
        if ((minors >> m) & 1) {
          S->dpre[m][0] += sign * in.core;
          S->dpre[m][1] += sign * in.mem;
          S->dpre[m][2] += sign * in.ratio;
        }
    /* (ABI 17) its RDMA / FPGA minors (bytes 1 and 2 of the packed mask): the per-instance request on each */
    for (int t = 0; t < KG_DEV_XTYPES; t++) {
      const int32_t xm = (int32_t)(((uint32_t)minors >> (8 * (t + 1))) & 0xFFu);
      if (!xm || !vp.xq[t]) continue;
      const int64_t q = vp.xq[t], per = (q > 100 && q % 100 == 0) ? 100 : q;
      for (int m = 0; m < KG_MAX_MINORS; m++)
        if ((xm >> m) & 1) S->xpre[t][m] += sign * per;
    }
  }
  for (int q = 0; q < KG_RES_MAX; q++) S->rs.requested[q] -= sign * v->requests[q];
  S->rs.nonzero[0] -= sign * v->nonzero_requests[0];
  S->rs.nonzero[1] -= sign * v->nonzero_requests[1];
  S->rs.num_pods -= sign;
  int nz = 0; /* !quotav1.IsZero(podRequests): every requested resource counts, not only cpu / memory */
  for (int q = 0; q < KG_RES_MAX; q++) nz |= v->requests[q] != 0;
  if (!nz) return;
  if (v->flags & KG_POD_RESERVE) return; /* RemovePod / AddPod (plugin.go:254,286): a reserve pod is never preemptible */
  if (slot >= 0 && slot < KG_MAX_RSV_SLOTS) {
    for (int q = 0; q < KG_RES_MAX; q++) S->pre_rr[slot][q] += sign * v->requests[q];
    S->pre_rr_set |= 1 << slot;
  } else {
    for (int q = 0; q < KG_RES_MAX; q++) S->pre[q] += sign * v->requests[q];
    S->pre_set = 1;
  }
}

/* fitsNode (plugin.go:433-482) with rInfo = slot s (s < 0: nil) and a preemptible amount over every resource.  `np` =
 * len(NodeInfo.Pods) of the NodeInfo the Filter sees (victims removed); podRequested / rAllocated are
 * nodeReservationState's, which the victims' removal does not touch (a node without state has none: zero).  A
 * reservation holds cpu / memory only, so its remained / allocated amounts of the other resources are 0, and
 * podRequested's are the node's Requested at restore time (`st0`). */
static int fits_node_pre(const kg_pod* pod, const kg_node* node, const or_node_state* st0, const or_rsv_node* ns,
                         int64_t np, const kg_node_reservations* r, int s, const int64_t pre[KG_RES_MAX]) {
  if (np - ns->n_matched + 1 > node->allowed_pods) return 0;
  int zero = 1;
  for (int q = 0; q < KG_RES_MAX; q++) zero &= pod->requests[q] == 0;
  if (zero) return 1;
  int64_t rc = 0, rm = 0;
  if (s >= 0) {
    rc = sub_nn(r->allocatable_cpu[s], r->allocated_cpu[s]);
    rm = sub_nn(r->allocatable_mem[s], r->allocated_mem[s]);
  }
  const int64_t prc = ns->has_state ? ns->pod_requested[0] : 0, prm = ns->has_state ? ns->pod_requested[1] : 0;
  if (pod->requests[KG_RES_CPU] > node->allocatable[KG_RES_CPU] - (prc - rc - ns->r_allocated[0] - pre[KG_RES_CPU]))
    return 0;
  if (pod->requests[KG_RES_MEMORY] > node->allocatable[KG_RES_MEMORY] - (prm - rm - ns->r_allocated[1] - pre[KG_RES_MEMORY]))
    return 0;
  /* EphemeralStorage always (:471), then `for rName, rQuant := range podRequest.ScalarResources` (:475-479) */
  for (int q = KG_RES_EPHEMERAL; q <= KG_RES_MID_MEMORY; q++) {
    if (q > KG_RES_EPHEMERAL && pod->requests[q] == 0) continue;
    const int64_t pr = ns->has_state ? st0->requested[q] : 0;
    if (pod->requests[q] > node->allocatable[q] - (pr - pre[q])) return 0;
  }
  return 1;
}

/* the pod's Filters on the candidate's current NodeInfo copy: 0, KG_REJECT_* bits, or < 0 (an oracle error) */
static int64_t pre_node_filter(const kg_config* cfg, const kg_node* node, const kg_node_metric* metric,
                               const or_node_state* st0, const kg_node_reservations* rsv, const kg_pod* pod,
                               const pre_node* S, int64_t now) {
  const int rsv_on = cfg->reservation_filter || cfg->reservation_score;
  int64_t rej = 0;
  if (cfg->fit_filter) rej |= or_fit_filter(node, &S->rs, pod);
  if (cfg->la_filter) {
    const int f = or_loadaware_filter(cfg, node, metric, pod, now);
    if (f < 0) return f;
    if (f) rej |= KG_REJECT_LOADAWARE;
  }
  if (rsv_on && cfg->reservation_filter) {
    const or_rsv_node* ns = &S->ns;
    const int required = (pod->reservation_flags & KG_POD_RSV_AFFINITY) != 0;
    int ok = 1;
    if (ns->n_matched == 0 || !ns->has_state) {
      if (required) ok = 0;
      else if (S->pre_set || S->pre_rr_set) ok = fits_node_pre(pod, node, st0, ns, S->rs.num_pods, rsv, -1, S->pre);
    } else {
      const int64_t pc = pod->requests[KG_RES_CPU], pm = pod->requests[KG_RES_MEMORY];
      const int kc = or_pod_cpu_key(pod), km = or_pod_mem_key(pod);
      int satisfied = 0;
      for (int k = 0; k < ns->n_matched && !satisfied; k++) {
        const int s = ns->matched[k];
        const int hc = rsv->allocatable_cpu[s] > 0, hm = rsv->allocatable_mem[s] > 0;
        if (!((kc && hc) || (km && hm))) continue;
        int64_t p2[KG_RES_MAX]; /* framework.NewResource(preemptibleInRR) + preemptible[node] */
        for (int q = 0; q < KG_RES_MAX; q++) p2[q] = S->pre_rr[s][q] + S->pre[q];
        const int fits = fits_node_pre(pod, node, st0, ns, S->rs.num_pods, rsv, s, p2);
        if (rsv->policy[s] == KG_RSV_POLICY_RESTRICTED) {
          /* Allocated − preemptibleInRR (non-negative, masked to the reservation's keys) when that map is set */
          int64_t ac = rsv->allocated_cpu[s], am = rsv->allocated_mem[s];
          if ((S->pre_rr_set >> s) & 1) {
            ac = hc ? sub_nn(ac, S->pre_rr[s][KG_RES_CPU]) : 0;
            am = hm ? sub_nn(am, S->pre_rr[s][KG_RES_MEMORY]) : 0;
          }
          const int64_t rc = sub_nn(rsv->allocatable_cpu[s], ac), rm = sub_nn(rsv->allocatable_mem[s], am);
          if ((!hc || !kc || pc <= rc) && (!hm || !km || pm <= rm) && fits) satisfied = 1;
        } else if (fits) {
          satisfied = 1;
        }
      }
      ok = satisfied || !required;
    }
    if (!ok) rej |= KG_REJECT_RESERVATION;
  }
  const or_pre_ext* x = S->x;
  if (x && x->pred) {
    if (cfg->taint_filter && !or_taint_filter(x->pred, pod)) rej |= KG_REJECT_TAINT;
    if (cfg->affinity_filter && !or_affinity_filter(x->pred, pod)) rej |= KG_REJECT_NODE_AFFINITY;
  }
  if (x && x->numa && cfg->numa_filter) {
    or_hint aff;
    if (!or_numa_filter(cfg, &S->nn, &S->np, &aff, S->rs.requested[KG_RES_CPU], node->allocatable[KG_RES_CPU]))
      rej |= KG_REJECT_NUMA;
  }
  if (x && x->dev && cfg->ds_filter && !S->dsp.skip) {
    /* Filter without GPU-holding reservations: Allocate(nil, nil, nil, preemptibleDevices[node]); a node without a
     * Device object rejects a device pod (NodeResourcesFit on the device resources, as or_ds_filter) */
    const int ok = !S->dsp.error && x->dev->has_device &&
                   or_ds_allocate(x->dev, &S->dsp, 0, 0, 0, NULL, (const int64_t(*)[3])S->dpre, 0, 0, NULL) >= 0 &&
                   or_dsx_filter(x->dev, &S->dsp, (const int64_t(*)[KG_MAX_MINORS])S->xpre);
    if (!ok) rej |= KG_REJECT_DEVICE;
  }
  return rej;
}

int64_t or_filter_preemption(const kg_config* cfg, const kg_node* node, const kg_node_metric* metric,
                             const or_node_state* st, const kg_node_reservations* rsv, const kg_pod* pod,
                             const kg_pod* victims, const int32_t* victim_slot, int64_t n_victims, int64_t now,
                             const or_pre_ext* ext) {
  if (!(node->flags & KG_NODE_VALID)) return KG_REJECT_INVALID_NODE;
  pre_node S;
  pre_node_init(&S, cfg, st, rsv, pod, ext);
  const int32_t* vm = ext ? ext->victim_minors : NULL;
  for (int64_t k = 0; k < n_victims; k++)
    pre_node_apply(&S, &victims[k], victim_slot ? victim_slot[k] : -1, vm ? vm[k] : 0, 1);
  return pre_node_filter(cfg, node, metric, st, rsv, pod, &S, now);
}

/* SelectVictimsOnNode (elasticquota/preempt.go:111-215; k8s defaultpreemption) of one candidate node, the potential
 * victims given in reprieve order (PDB-violating first, each group by util.MoreImportantPod — the caller's sort and
 * filterPodsWithPDBViolation): remove them all, Filter (none: "No victims found" → KG_REJECT_NO_VICTIMS), then
 * reprieve each in order — add it back, Filter, remove it again as a victim when the pod no longer fits (:175-213).
 * out_victim[k] = 1 for a victim kept; *out_violating = the PDB-violating victims kept.  Returns the first Filter's
 * status (0 = a candidate), or < 0 on an oracle error. */
int64_t or_select_victims(const kg_config* cfg, const kg_node* node, const kg_node_metric* metric,
                          const or_node_state* st, const kg_node_reservations* rsv, const kg_pod* pod,
                          const kg_pod* victims, const int32_t* victim_slot, const uint8_t* violating,
                          int64_t n_victims, int64_t now, uint8_t* out_victim, int32_t* out_violating,
                          const or_pre_ext* ext) {
  for (int64_t k = 0; k < n_victims; k++) out_victim[k] = 0;
  *out_violating = 0;
  if (!(node->flags & KG_NODE_VALID)) return KG_REJECT_INVALID_NODE;
  if (n_victims == 0) return KG_REJECT_NO_VICTIMS;
  pre_node S;
  pre_node_init(&S, cfg, st, rsv, pod, ext);
  const int32_t* vm = ext ? ext->victim_minors : NULL;
  for (int64_t k = 0; k < n_victims; k++)
    pre_node_apply(&S, &victims[k], victim_slot ? victim_slot[k] : -1, vm ? vm[k] : 0, 1);
  const int64_t rej = pre_node_filter(cfg, node, metric, st, rsv, pod, &S, now);
  if (rej != 0) return rej;
  for (int64_t k = 0; k < n_victims; k++) {
    const int slot = victim_slot ? victim_slot[k] : -1;
    const int32_t mk = vm ? vm[k] : 0;
    pre_node_apply(&S, &victims[k], slot, mk, -1);
    const int64_t f = pre_node_filter(cfg, node, metric, st, rsv, pod, &S, now);
    if (f < 0) return f;
    if (f != 0) {
      pre_node_apply(&S, &victims[k], slot, mk, 1);
      out_victim[k] = 1;
      if (violating && violating[k]) *out_violating += 1;
    }
  }
  return 0;
}
