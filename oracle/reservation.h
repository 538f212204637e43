/*
 * reservation.h — CPU restatement of the Reservation plugin on the hot path (SURVEY §8a A15–A18).
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h): tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it
 * as the checker / CPU baseline; nothing under koordinator_amd/ links or calls it.
 *
 * Pinning: golden cases transcribed from reservation/scoring_test.go (TestScore :40, TestPreScore nomination
 * :392-729) and plugin_test.go (Test_filterWithReservations :670) into tests/golden/reservation.json
 * (script tests/golden/make_golden_resv.py).  The BeforePreFilter restore arithmetic (transformer.go:49-346)
 * and the full-cycle composition (Filter → PreScore → Score → NormalizeScore → Reserve) are restated from the
 * source; no reference test drives the whole cycle on a cluster, so those parts are "parity unpinned" beyond
 * the per-function cases.
 */
#ifndef KOORD_ORACLE_RESERVATION_H_
#define KOORD_ORACLE_RESERVATION_H_
#include <stdint.h>
#include "../include/koordgpu.h"
#include "oracle.h"

#ifdef __cplusplus
extern "C" {
#endif

/* nodeReservationState (transformer.go:180-187) of one (pod, node) plus the restored NodeInfo fields. */
typedef struct or_rsv_node {
  int32_t has_state;                 /* the node is in state.nodeReservationStates                         */
  int32_t n_matched;
  int32_t matched[KG_MAX_RSV_SLOTS]; /* slot indices, reservation order                                     */
  int64_t pod_requested[2];          /* Requested after the unmatched trim (cpu milli, memory)              */
  int64_t r_allocated[2];            /* Σ matched Allocated                                                 */
  int64_t requested[2], nonzero[2];  /* restored NodeInfo.Requested / NonZeroRequested                      */
  int64_t num_pods;                  /* restored len(NodeInfo.Pods)                                         */
  int32_t n_unmatched;               /* (ABI 13) the restore's unmatched list (usable, not matched, assigned) */
  int32_t unmatched[KG_MAX_RSV_SLOTS];
} or_rsv_node;

/* BeforePreFilter for one node (transformer.go:100-189). */
void or_rsv_forget(kg_node_reservations* r, int s, const kg_pod* pod);
void or_rsv_restore(const kg_node_reservations* r, const or_node_state* st, const kg_pod* pod, or_rsv_node* out);
/* fitsNode (plugin.go:433-482) with rInfo = slot s (s < 0: nil), preemptible = 0. */
int or_rsv_fits_node(const kg_pod* pod, int64_t allowed_pods, const int64_t alloc[2], const or_rsv_node* ns,
                     const kg_node_reservations* r, int s);
/* filterWithReservations over the given slots (plugin.go:384-428): 1 = Success, 0 = Unschedulable. */
int or_rsv_filter_with(const kg_pod* pod, int64_t allowed_pods, const int64_t alloc[2], const or_rsv_node* ns,
                       const kg_node_reservations* r, const int32_t* slots, int n_slots, int required);
/* Filter for a non-reserve pod (plugin.go:357-378, preemption maps empty). */
/* (ABI 12) Reservation.Filter of a reserve pod / reservation operating mode (plugin.go:324-350): 1 = pass */
int or_rsv_policy_filter(const kg_pod* pod, int64_t node_idx, const kg_node_reservations* r);
int or_rsv_filter(const kg_pod* pod, int64_t allowed_pods, const int64_t alloc[2], const or_rsv_node* ns,
                  const kg_node_reservations* r);
/* scoreReservation (scoring.go:183-203) of slot s. */
int64_t or_rsv_score_slot(const kg_pod* pod, const kg_node_reservations* r, int s);
/* NominateReservation (nominator.go:76-134) with FilterReservation (plugin.go:492-519) as the only reservation
 * filter and ScoreReservation as the only reservation scorer; ties on score → lowest slot.  Returns slot or -1. */
int or_rsv_nominate(const kg_pod* pod, int64_t allowed_pods, const int64_t alloc[2], const or_rsv_node* ns,
                    const kg_node_reservations* r);
/* (ABI 13) NominateReservation with DeviceShare as a reservation filter / score plugin (plugin.go:333-380,
 * scoring.go:99-127): a pod with device requests may be nominated only to a GPU-holding reservation DeviceShare can
 * allocate from; the prioritization sums Reservation's ScoreReservation and DeviceShare's, the latter normalized by
 * DefaultReservationNormalizeScore (frameworkext/framework_extender.go:379-432).  dsp / dev / dst NULL = no DeviceShare. */
struct or_ds_pod;
struct or_ds_rsv;
int or_rsv_nominate_ds(const kg_pod* pod, int64_t allowed_pods, const int64_t alloc[2], const or_rsv_node* ns,
                       const kg_node_reservations* r, const kg_node_device* dev, const struct or_ds_pod* dsp,
                       const struct or_ds_rsv* dst, int strategy, const int64_t w[3]);
/* findMostPreferredReservationByOrder over the matched slots (scoring.go:162-181): INT64_MAX if none. */
int64_t or_rsv_node_order(const or_rsv_node* ns, const kg_node_reservations* r);

/* Sequential FIFO scheduling with NodeResourcesFit + LoadAwareScheduling + Reservation (one pod at a time,
 * ties → lowest index).  `st` and `rsv` are updated by Reserve; out_slot (nullable) = the slot each pod was
 * assumed into (-1 = none). */
int or_schedule_resv(const kg_config* cfg, int64_t n_nodes, const kg_node* nodes, const kg_node_metric* metrics,
                     or_node_state* st, kg_node_reservations* rsv, int64_t n_pods, const kg_pod* pods, int64_t now,
                     int32_t* out_node, int64_t* out_score, int32_t* out_slot);

/* The exact per-pod cycle (C5, the shipped profile, TaintToleration / NodeAffinity / BalancedAllocation when the
 * config enables them, over `preds`, NULL = no predicates / taints; (ABI 12) PodTopologySpread / InterPodAffinity over
 * `groups` = or_group_node[n_nodes] (defaults.h), NULL = none — mutated by Reserve): NodeResourcesFit + LoadAwareScheduling + Reservation + DeviceShare (+ ElasticQuota admission when
 * pods carry quota_id).  `dev` / `quotas` may be NULL.  The node loop of every pod runs on n_threads OpenMP threads
 * (Parallelizer chunking); reductions and Reserve are sequential.  out_minors (nullable) = DeviceShare's minors. */
int or_schedule_resv_full(const kg_config* cfg, int64_t n_nodes, const kg_node* nodes, const kg_node_metric* metrics,
                          or_node_state* st, kg_node_reservations* rsv, kg_node_device* dev, kg_quota* quotas,
                          int64_t n_quotas, int64_t n_pods, const kg_pod* pods, int64_t now, int n_threads,
                          int32_t* out_node, int64_t* out_score, int32_t* out_slot, int32_t* out_minors,
                          void* numa_states, uint64_t* out_cpus, int64_t* out_numa, const kg_node_predicates* preds,
                          void* groups);

/* Golden-case entry (flat): explicit nodeReservationState (pod_requested, r_allocated, restored pod count) as the
 * reference tests build it.  out[0] = filter pass, out[1] = nominated slot, out[2] = Score (before normalize). */
void or_rsv_case_flat(const kg_pod* pod, int64_t allowed_pods, const int64_t alloc[2], int64_t num_pods,
                      const int64_t pod_requested[2], const int64_t r_allocated[2], int has_state,
                      const kg_node_reservations* r, int64_t* out);

void or_rsv_restore_flat(const kg_node_reservations* r, const or_node_state* st, const kg_pod* pod, int64_t* out);

/* (r6) The dry run's other Filters (NULL members: the plugin has no data for the node / is not in the profile):
 *   numa  the node's NodeNUMAResource view — no PreFilterExtensions (nodenumaresource/plugin.go:272-274): the victims'
 *         cpusets stay allocated; the Filter (plugin.go:276-334) reads the victim-free NodeInfo.Requested cpu;
 *   dev   the node's GPUs — DeviceShare's RemovePod / AddPod (deviceshare/plugin.go:163-278) append / subtract a victim's
 *         allocation (victim_minors[k], its per-instance share) to state.preemptibleDevices[node] unless it is a reserve
 *         pod, requests nothing the preemptor's state tracks (state.skip) or was allocated from a reservation (its GPUs
 *         go to preemptibleInRRs, which only GPU-holding reservations read); Filter (:280-330) allocates with free =
 *         total − max(0, used − preemptible) (calcFreeWithPreemptible, device_cache.go:314-342);
 *   pred  the node's taints / labels — TaintToleration and NodeAffinity Filters (node-static). */
typedef struct or_pre_ext {
  const kg_node_numa* numa;
  const kg_node_device* dev;
  const kg_node_predicates* pred;
  const int32_t* victim_minors;
} or_pre_ext;

/* Preemption dry run (defaultpreemption SelectVictimsOnNode → RunFilterPluginsWithNominatedPods on a NodeInfo copy
 * with the victims removed): NodeInfo.RemovePod of each victim, and Reservation's PreFilterExtensions.RemovePod
 * (plugin.go:284-310) adding each victim's requests to state.preemptible[node] (victim_slot[k] < 0) or to
 * state.preemptibleInRRs[node][slot] — a victim with all-zero requests is skipped.  Then the pod's Filters on that
 * node: NodeResourcesFit (cpu / memory / pods / ephemeral-storage / scalars), LoadAwareScheduling, and the Reservation Filter (plugin.go:357-428)
 * with the preemptible amounts in fitsNode (:433-482) and the Restricted policy's Allocated (:404-413); (r6) with `ext`
 * NodeNUMAResource, DeviceShare, TaintToleration and NodeAffinity as or_pre_ext says.  Returns the KG_REJECT_* bits
 * (0 = every Filter passes). */
int64_t or_filter_preemption(const kg_config* cfg, const kg_node* node, const kg_node_metric* metric,
                             const or_node_state* st, const kg_node_reservations* rsv, const kg_pod* pod,
                             const kg_pod* victims, const int32_t* victim_slot, int64_t n_victims, int64_t now,
                             const or_pre_ext* ext);
/* (r5) SelectVictimsOnNode of one candidate (elasticquota/preempt.go:111-215): the potential victims in reprieve
 * order are removed, the Filters run (none: KG_REJECT_NO_VICTIMS), then each victim is reprieved in order (added
 * back, kept as a victim when the pod no longer fits).  out_victim[k], *out_violating as kg_pods_select_victims. */
int64_t or_select_victims(const kg_config* cfg, const kg_node* node, const kg_node_metric* metric,
                          const or_node_state* st, const kg_node_reservations* rsv, const kg_pod* pod,
                          const kg_pod* victims, const int32_t* victim_slot, const uint8_t* violating,
                          int64_t n_victims, int64_t now, uint8_t* out_victim, int32_t* out_violating,
                          const or_pre_ext* ext);

#ifdef __cplusplus
}
#endif
#endif
