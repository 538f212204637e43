// Reservation plugin on the device (SURVEY §8a A15–A18), composed with DeviceShare (A19–A21) and ElasticQuota
// admission (A24) for config C5: per-node reservation slots in HBM and the per-pod pass that restores NodeInfo for
// matched / unmatched reservations (BeforePreFilter, transformer.go:49-346), runs NodeResourcesFit + LoadAware on the
// restored row, the Reservation Filter (plugin.go:357-428), the DeviceShare Filter (deviceshare/plugin.go:280-330),
// the nomination (nominator.go:76-134) and both Scores (reservation/scoring.go:103-203, deviceshare/scoring.go:34-89)
// with the PreScore preferred node and DefaultNormalizeScore, then Reserve (reservation/plugin.go:521-559,
// deviceshare/plugin.go:385-438, elasticquota/plugin.go:332-346).
//
// One pod per pass, two kernels (wide pass, normalise + argmax pass); pod j's Reserve runs in pod j+1's wide-pass
// prologue by the thread owning the winner row.  A group of kRsvGroup pods is captured in one hipGraph, closed by
// a one-wave kernel that reserves the group's last pod and advances the device cursor.
//
// (r3) The same pass is the engine's exact path for every plugin combination the round engines do not cover, in
// particular the reference's shipped profile (config/manager/scheduler-config.yaml:66-117: LoadAwareScheduling +
// NodeNUMAResource + DeviceShare + Reservation [+ ElasticQuota]): NodeNUMAResource Filter + Score run per node on the
// restored NodeInfo (nodenumaresource/plugin.go:276-334, scoring.go:55-93) and its Reserve (plugin.go:375-415, the
// exact cpuset) runs in the winner's owner thread before DeviceShare's, in the profile's Reserve order; a later
// Reserve failure leaves the earlier plugins' state untouched (RunReservePluginsUnreserve).  Reserve pods hold no
// cpuset here, so NodeNUMAResource's RestoreReservation (nodenumaresource/reservation.go) has nothing to restore.
//
// Reservations here hold cpu / memory (an allocatable of 0 = the key is absent).  DeviceShare restores device state
// only for reservations whose reserve pod holds devices (deviceshare/reservation.go:132-150), so for these it keeps
// no reservation state: its Filter / Score are the node-level ones, and its FilterReservation rejects every
// reservation for a pod that requests devices (plugin.go:462-486) — such a pod is never nominated into one.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/koordgpu.h"
#include "defaults_dev.h"
#include "ds_dev.h"
#include "groups_dev.h"
#include "kernels.h"
#include "numa_dev.h"

namespace kg {

constexpr int kRsvSlots = KG_MAX_RSV_SLOTS;
constexpr uint32_t RS_AVAIL = 1u << 0, RS_ONCE = 1u << 1, RS_UNSCHED = 1u << 2;  // policy in bits 4..5
constexpr uint32_t RS_GPU = 1u << 3;  // (ABI 13) the reservation holds GPUs: its RsvGpu row is live
constexpr uint32_t RS_CPUS = 1u << 6;  // (ABI 15) the reservation holds a cpuset: its RsvCpu row is live
constexpr uint32_t RP_AFFINITY = 1u << 0, RP_RESERVE = 1u << 1, RP_OPERATING = 1u << 2, RP_SEL = 1u << 3;
constexpr int RP_POLICY_SHIFT = 8;  // flags bits 8..9: the allocate policy of a reserve / operating-mode pod
constexpr int64_t kDefaultMilliCpu = 100, kDefaultMemory = 200ll << 20;  // schedutil.GetNonzeroRequests defaults

struct RsvNode {  // 192 B: one node's slots, read only for nodes with slots (rsv_n[i] > 0)
  int64_t alloc_cpu[kRsvSlots], alloc_mem[kRsvSlots];    // ReservationInfo.Allocatable (0 = key absent)
  int64_t allocd_cpu[kRsvSlots], allocd_mem[kRsvSlots];  // ReservationInfo.Allocated
  int32_t owner[kRsvSlots], assigned[kRsvSlots], order[kRsvSlots];  // owner group 0..63
  uint32_t meta[kRsvSlots];
};
static_assert(sizeof(RsvNode) == 192, "RsvNode layout");
// (ABI 12) the slots' fakeNode predicate bits live in their own [cap][kRsvSlots] array (RsvExt::rsv_pred), read only
// for a pod whose reservation affinity has a selector or terms: the slot record the resolvers copy stays 192 B

struct RsvPod {  // 16 B: what every evaluation of the pod reads
  uint64_t owner_mask;  // bit g: the pod matches the owners of owner group g
  uint32_t flags;       // RP_* | allocate policy << RP_POLICY_SHIFT
  int32_t aux;          // RP_RESERVE: the node GetReservePodNodeName names (-1 = none); RP_SEL: its RsvSel index
};
// (ABI 12) a required reservation affinity's selector / terms, read only by pods with RP_SEL (RsvExt::rsv_sel)
struct RsvSel {  // 48 B
  uint64_t sel;     // ReservationSelector predicates (all must hold)
  uint64_t terms[KG_MAX_AFF_TERMS];
  uint32_t nterms;  // ReservationSelectorTerms (0 = absent)
  uint32_t pad;
};

// RequiredReservationAffinity.Match (pkg/util/reservation/reservation.go:476-489) on a slot's fakeNode labels
__device__ __forceinline__ bool rsv_affinity_match(const RsvSel& c, uint64_t pred) {
  if ((pred & c.sel) != c.sel) return false;
  if (c.nterms == 0) return true;
  bool any = false;
#pragma unroll
  for (int k = 0; k < KG_MAX_AFF_TERMS; ++k) any |= k < (int)c.nterms && c.terms[k] != 0 && (pred & c.terms[k]) == c.terms[k];
  return any;
}

struct RsvParams {
  int32_t filter, score, weight, pad;
};

// (ABI 13) One reservation's GPU holding (deviceshare/reservation.go:133-160): the reserve pod's allocation per minor
// (the reservation's allocatable) and the allocations of its assigned pods on those minors (appendAllocatedByHints).
// 272 B per slot, [cap][kRsvSlots]; read only for a pod with device requests on a node with an RS_GPU slot.
struct RsvGpu {
  int32_t acore[kMinors], aratio[kMinors];  // allocatable: gpu-core, gpu-memory-ratio
  int32_t dcore[kMinors], dratio[kMinors];  // allocated by the assigned pods
  int64_t amem[kMinors], dmem[kMinors];     // gpu-memory bytes
  uint32_t minors;                          // the reserve pod's minors
  uint32_t pad[3];
};
static_assert(sizeof(RsvGpu) == 272, "RsvGpu layout");
struct RsvGpuNode {  // one node's slots (the upsert's scatter row)
  RsvGpu s[kRsvSlots];
};
__device__ __forceinline__ int64_t rg_a(const RsvGpu& g, int m, int q) {
  return q == 0 ? (int64_t)g.acore[m] : (q == 1 ? g.amem[m] : (int64_t)g.aratio[m]);
}
__device__ __forceinline__ int64_t rg_d(const RsvGpu& g, int m, int q) {
  return q == 0 ? (int64_t)g.dcore[m] : (q == 1 ? g.dmem[m] : (int64_t)g.dratio[m]);
}

// (ABI 15) One reservation's cpuset (NodeNUMAResource): `r` = GetAllocatedCPUSet(node, reservation UID), `u` = the union
// of its assigned pods' cpusets.  RestoreReservation's reserved cpus are r − u (nodenumaresource/reservation.go:76-113).
// 64 B per slot, [cap][kRsvSlots]; read only for a cpuset-capable pod nominated into an RS_CPUS slot, and by Unreserve.
struct RsvCpu {
  uint64_t r[kCpuWords];
  uint64_t u[kCpuWords];
};
static_assert(sizeof(RsvCpu) == 64, "RsvCpu layout");
struct RsvCpuNode {  // one node's slots (the upsert's scatter row)
  RsvCpu s[kRsvSlots];
};
__device__ __forceinline__ CpuSet rsv_reserved_cpus(const RsvCpu& c) {
  CpuSet p;
#pragma unroll
  for (int w = 0; w < kCpuWords; ++w) p.w[w] = c.r[w] & ~c.u[w];
  return p;
}

// DeviceShare + ElasticQuota context of the C5 pass (ds = nullptr: no DeviceShare in the profile; nq = 0: no quotas)
struct RsvExt {
  const DsNode* __restrict__ ds;       // [cap] node devices (deviceUsed updated by Reserve)
  DsXNode* __restrict__ dsx;           // (ABI 17) [cap] RDMA / FPGA devices (per-pod pass only)
  const DsPod* __restrict__ dpods;     // [pods] DeviceShare preFilterState
  DsParams DP;
  QuotaRow* __restrict__ quotas;       // [nq]
  const int64_t* __restrict__ qdev;    // [pods][kQuotaRes] device requests (quota dims 2..7)
  int32_t* __restrict__ out_minors;    // [pods]
  int nq;
  // NodeNUMAResource (ns = nullptr: not in the profile)
  const NumaStatic* __restrict__ ns;   // [cap] TopologyOptions
  NumaMut* __restrict__ nm;            // [cap] NodeAllocation (Reserve updates it)
  const NumaPod* __restrict__ npods;   // [pods] preFilterState
  NumaParams NP;
  uint32_t* __restrict__ aff;          // [cap] the affinity NUMA Filter stored for the pass's pod: mask | nil << 8
  uint64_t* __restrict__ out_cpus;     // [pods][kCpuWords] the cpuset Reserve allocated
  int64_t* __restrict__ out_nrec;      // [pods][kNumaRecWords] the pod's NUMA allocation record
  // NodeResourcesFit over ephemeral-storage / scalar resources (P_AUX pods): [pods][kAux] requests
  const int64_t* __restrict__ paux;
  // TaintToleration / NodeAffinity / NodeResourcesBalancedAllocation (defp = nullptr: none in the profile)
  const NodePred* __restrict__ pred;   // [cap]
  const DefPod* __restrict__ defp;     // [pods]
  DefParams DF;
  uint32_t* __restrict__ val2;         // [cap] raw TaintToleration count << 24 | raw NodeAffinity sum (scores on)
  // (ABI 12) PodTopologySpread / InterPodAffinity, hostname key (gpods = nullptr: neither in the profile)
  GroupTable G;                        // per-node group counters
  const GroupPod* __restrict__ gpods;  // [pods]
  GroupParams GP;
  const double* __restrict__ logw;     // [cap + 1]: log(F + 2), the host's libm
  uint64_t* __restrict__ gval;         // [cap] InterPodAffinity raw << 32 | PodTopologySpread raw (+ 2^31; 0 = ignored)
  int32_t* __restrict__ gz;            // [2 parities][kZoneSumWords] the zone sums (ZoneSums)
  const uint64_t* __restrict__ rsv_pred;  // [cap][kRsvSlots] the slots' fakeNode predicates (reservation affinity)
  const RsvSel* __restrict__ rsv_sel;     // [pods] the RP_SEL pods' selectors / terms (RsvPod::aux)
  uint64_t* __restrict__ gzm;          // [2 parities] the present zones
  // (ABI 13) reservations holding GPUs (rgpu = nullptr: none in the cluster, or DeviceShare / Reservation off); the
  // Reserve re-runs the winner's restore, so it needs the pod's Reservation view and the slot counts
  RsvGpu* __restrict__ rgpu;           // [cap][kRsvSlots]
  const RsvPod* __restrict__ rpods;    // [pods]
  const int32_t* __restrict__ rsv_n;   // [cap]
  // (ABI 15) reservations holding cpusets (rcpu = nullptr: none in the cluster, or NodeNUMAResource / Reservation off)
  RsvCpu* __restrict__ rcpu;           // [cap][kRsvSlots]
};
// pod j's zone sums (double-buffered by parity: group_pre(j) accumulates, rsv_select(j) clears j + 1's)
__device__ __forceinline__ ZoneSums zone_sums(const RsvExt& X, int64_t j) {
  int32_t* b = X.gz + (size_t)(j & 1) * kZoneSumWords;
  return ZoneSums{b, b + kSpread * kZones, b + 2 * kSpread * kZones, X.gzm + (j & 1)};
}

struct RsvOut {
  bool feas;
  int64_t base;   // Fit + LoadAware weighted total
  int32_t raw;    // Reservation Score of the nominated slot (0 = none)
  int32_t nom;    // nominated slot, -1 = none
  int32_t order;  // findMostPreferredReservationByOrder over matched (INT32_MAX = none)
  int32_t dsraw;  // DeviceShare raw Score
  int32_t tcnt;   // TaintToleration raw Score (intolerable PreferNoSchedule taints)
  int32_t asum;   // NodeAffinity raw Score
};

__device__ __forceinline__ int64_t rsv_nn(int64_t a, int64_t b) { return a - b > 0 ? a - b : 0; }
// GetNonzeroRequests of the reserve pod (requests = Allocatable): an absent key takes the default
__device__ __forceinline__ int64_t rsv_nz_cpu(const RsvNode& rn, int s) {
  return rn.alloc_cpu[s] > 0 ? rn.alloc_cpu[s] : kDefaultMilliCpu;
}
__device__ __forceinline__ int64_t rsv_nz_mem(const RsvNode& rn, int s) {
  return rn.alloc_mem[s] > 0 ? rn.alloc_mem[s] : kDefaultMemory;
}

// scoreReservation (scoring.go:183-203): MostAllocated over the reservation's non-zero allocatable.  Division-free:
// 100·r / a for 0 ≤ r ≤ a is most_requested64 (float estimate + one exact int64 correction each way), and Σ / #r
// divides by 1 or 2 (a non-negative sum: a shift).
__device__ __forceinline__ int32_t rsv_score_slot(const RsvNode& rn, int s, const DevPod& p) {
  const int64_t rc = p.req_cpu + rn.allocd_cpu[s], rm = p.req_mem + rn.allocd_mem[s];
  int64_t w = 0, sc = 0;
  if (rn.alloc_cpu[s] != 0) {
    ++w;
    if (rc <= rn.alloc_cpu[s]) sc += rc >= 0 ? most_requested64(rc, rn.alloc_cpu[s]) : 100 * rc / rn.alloc_cpu[s];
  }
  if (rn.alloc_mem[s] != 0) {
    ++w;
    if (rm <= rn.alloc_mem[s]) sc += rm >= 0 ? most_requested64(rm, rn.alloc_mem[s]) : 100 * rm / rn.alloc_mem[s];
  }
  if (w == 2) return (int32_t)(sc >= 0 ? sc >> 1 : sc / 2);
  return (int32_t)sc;
}

// Per-node outputs kg_pods_evaluate_reservation reports besides RsvOut (nullptr in the scheduling pass)
struct RsvDbg {
  uint32_t matched;       // the slots in nodeReservationState.matched
  int32_t has_state;      // a nodeReservationState exists (BeforePreFilter restored the node)
  int64_t req_cpu, req_mem, nz_cpu, nz_mem, num_pods;  // the restored NodeInfo
  int64_t pod_req_cpu, pod_req_mem;                    // nodeReservationState.podRequested
};

// BeforePreFilter's restore of one node for one pod (transformer.go:100-189): the matched slots' reserve pods leave
// NodeInfo (restoreMatchedReservation :240-263), the unmatched assigned ones leave and return as their remainders
// (restoreUnmatchedReservations :265-291); pr_* = nodeReservationState.podRequested, ra_* = Σ matched Allocated.
// kExt = false (the batched exact rounds, which never see reserve / operating-mode / selector pods): owner groups only
template <bool kExt = true>
__device__ __forceinline__ void rsv_restore(const RsvNode& rn, int ns, const RsvPod& rp, const uint64_t* pred_row,
                                            const RsvSel* sel, Row& r, uint32_t& mm, int& nm,
                                            int64_t& pr_c, int64_t& pr_m, int64_t& ra_c, int64_t& ra_m,
                                            bool& has_state, uint32_t* um_out = nullptr) {
  uint32_t um = 0;
#pragma unroll
  for (int s = 0; s < kRsvSlots; ++s) {
    if (s >= ns) break;
    const uint32_t m = rn.meta[s];
    if (!(m & RS_AVAIL) || ((m & RS_ONCE) && rn.assigned[s] > 0)) continue;  // transformer.go:101-110
    // ReservationInfo.Match → MatchReservationOwners, decoded per owner group into the pod's mask
    // a reserve pod matches no reservation (transformer.go:112 isReservedPod)
    bool match = ((rp.owner_mask >> (rn.owner[s] & 63)) & 1u) && !(m & RS_UNSCHED);
    if (kExt)
      match = match && !(rp.flags & RP_RESERVE) &&
              (!(rp.flags & RP_AFFINITY) || !(rp.flags & RP_SEL) ||
               (sel && rsv_affinity_match(*sel, pred_row ? pred_row[s] : 0ull)));
    if (match) mm |= 1u << s;
    else if (rn.assigned[s] > 0) um |= 1u << s;
  }
  has_state = (mm | um) != 0 && !((rp.flags & RP_AFFINITY) && mm == 0);  // transformer.go:127-136
  if (um_out) *um_out = has_state ? um : 0u;
  if (!has_state) return;
#pragma unroll
  for (int s = 0; s < kRsvSlots; ++s)
    if (um >> s & 1) {  // restoreUnmatchedReservations (transformer.go:265-291)
      r.req_cpu -= rn.alloc_cpu[s];
      r.req_mem -= rn.alloc_mem[s];
      r.nz_cpu -= rsv_nz_cpu(rn, s);
      r.nz_mem -= rsv_nz_mem(rn, s);
      const int64_t rc = rsv_nn(rn.alloc_cpu[s], rn.allocd_cpu[s]), rm = rsv_nn(rn.alloc_mem[s], rn.allocd_mem[s]);
      if (rc != 0 || rm != 0) {  // the remainder pod carries the reservation's keys
        r.req_cpu += rc;
        r.req_mem += rm;
        r.nz_cpu += rn.alloc_cpu[s] > 0 ? rc : kDefaultMilliCpu;
        r.nz_mem += rn.alloc_mem[s] > 0 ? rm : kDefaultMemory;
      }
    }
  pr_c = r.req_cpu;
  pr_m = r.req_mem;
#pragma unroll
  for (int s = 0; s < kRsvSlots; ++s)
    if (mm >> s & 1) {  // restoreMatchedReservation: NodeInfo.RemovePod(reserve pod) (transformer.go:240-263)
      r.req_cpu -= rn.alloc_cpu[s];
      r.req_mem -= rn.alloc_mem[s];
      r.nz_cpu -= rsv_nz_cpu(rn, s);
      r.nz_mem -= rsv_nz_mem(rn, s);
      r.num_pods -= 1;
      ra_c += rn.allocd_cpu[s];
      ra_m += rn.allocd_mem[s];
      ++nm;
    }
}

// ---- (ABI 13) DeviceShare with reservations holding GPUs --------------------------------------------------------
// The plugin's restore of one node for one pod (RestoreReservation + mergeReservationAllocations, reservation.go:84-171)
// over the GPU-holding slots of the Reservation restore's matched (mt) / unmatched (um) lists.  The preemptible maps it
// builds are evaluated per (minor, resource) where used instead of materialized:
//   node view   (Filter fallback, Score / Reserve without a nominated GPU reservation):
//               mergedUnmatchedUsed + mergedMatchedAllocatable
//   slot view s (tryAllocateFromReservation / scoreWithReservation of matched slot s):
//               mergedUnmatchedUsed + mergedMatchedAllocated + remained(s)
// with mergedUnmatchedUsed = Σ_unmatched min(allocatable, allocated) (allocatable − remained), remained =
// SubtractWithNonNegativeResult(allocatable, allocated).  calcFreeWithPreemptible (device_cache.go:314-342) then gives
// free = total − max(0, used − preemptible), non-negative, on every minor; a Restricted slot's second Allocate sees only
// its own minors with their remained resources (requiredDeviceResources, calcRequiredDeviceResources).
struct DsrCtx {
  const RsvGpu* g;  // the node's [kRsvSlots] rows
  uint32_t um, mt;  // GPU-holding unmatched / matched slots
};
__device__ __forceinline__ int64_t dsr_pre(const DsrCtx& c, int m, int q, int slot) {
  int64_t v = 0;
#pragma unroll
  for (int s = 0; s < kRsvSlots; ++s) {
    if (!(((c.um | c.mt) >> s) & 1u)) continue;
    const int64_t A = rg_a(c.g[s], m, q), a = rg_d(c.g[s], m, q);
    if ((c.um >> s) & 1u) v += A < a ? A : a;
    else v += slot < 0 ? A : a;
  }
  if (slot >= 0) v += rsv_nn(rg_a(c.g[slot], m, q), rg_d(c.g[slot], m, q));
  return v;
}
__device__ __forceinline__ int64_t ds_tot(const DsNode& d, int m, int q) {
  return q == 0 ? (int64_t)d.tcore[m] : (q == 1 ? d.tmem[m] : (int64_t)d.tratio[m]);
}
__device__ __forceinline__ int64_t ds_used(const DsNode& d, int m, int q) {
  return q == 0 ? (int64_t)d.ucore[m] : (q == 1 ? d.umem[m] : (int64_t)d.uratio[m]);
}
// the free resources of minor m in a view (slot < 0: the node view; rr: a Restricted slot's required view)
__device__ __forceinline__ void dsr_free(const DsNode& d, const DsrCtx& c, int m, int slot, bool rr, int64_t f[3]) {
#pragma unroll
  for (int q = 0; q < 3; ++q)
    f[q] = rr ? rsv_nn(rg_a(c.g[slot], m, q), rg_d(c.g[slot], m, q))
              : rsv_nn(ds_tot(d, m, q), rsv_nn(ds_used(d, m, q), dsr_pre(c, m, q, slot)));
}
struct DsrView {
  bool any;    // some minor of the view has free resources (nodeDevice.filter keeps the GPU type)
  int nfit;    // minors the per-instance request fits (within `req` when set)
  int64_t T[3], F[3];
};
__device__ __forceinline__ DsrView dsr_view(const DsNode& d, const DsInst& in, const DsrCtx& c, int slot, bool rr,
                                           uint32_t req) {
  DsrView v{false, 0, {0, 0, 0}, {0, 0, 0}};
  const uint32_t minors = rr ? c.g[slot].minors & (uint32_t)d.present : (uint32_t)d.present;
  for (int m = 0; m < kMinors; ++m) {
    if (!((minors >> m) & 1u)) continue;
    int64_t f[3];
    dsr_free(d, c, m, slot, rr, f);
    const bool nz = (f[0] | f[1] | f[2]) != 0;
    v.any |= nz;
    v.nfit += (nz && (!req || ((req >> m) & 1u)) && in.core <= f[0] && in.mem <= f[1] && in.ratio <= f[2]) ? 1 : 0;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      v.T[q] += ds_tot(d, m, q);
      v.F[q] += f[q];
    }
  }
  return v;
}
__device__ __forceinline__ int64_t dsr_score(const DsrView& v, const DsInst& in, const DsParams& P) {
  if (!v.any) return 0;
  int64_t num = 0, ws = 0;
  const bool most = P.most != 0;
  ds_term(P.w_core, v.T[0], v.F[0], in.core, num, ws, most);
  ds_term(P.w_mem, v.T[1], v.F[1], in.mem, num, ws, most);
  ds_term(P.w_ratio, v.T[2], v.F[2], in.ratio, num, ws, most);
  return ws ? div_small(num, ws) : 0;
}
// tryAllocateFromReservation([s]) feasibility (reservation.go:196-236): Default / Aligned — Allocate(nil, preferred,
// nil, preemptible); Restricted — with required = preferred = the slot's minors, then again on its remained resources
__device__ __forceinline__ bool dsr_slot_ok(const DsNode& d, const DsInst& in, const DsrCtx& c, int s, bool restricted) {
  if (!restricted) {
    const DsrView v = dsr_view(d, in, c, s, false, 0u);
    return v.any && v.nfit >= in.count;
  }
  const uint32_t req = c.g[s].minors;
  const DsrView v1 = dsr_view(d, in, c, s, false, req);
  if (!(v1.any && v1.nfit >= in.count)) return false;
  const DsrView v2 = dsr_view(d, in, c, s, true, req);
  return v2.any && v2.nfit >= in.count;
}
// scoreWithReservation of slot s (reservation.go:246-272): the required view for Restricted, else the slot view
__device__ __forceinline__ int64_t dsr_slot_score(const DsNode& d, const DsInst& in, const DsrCtx& c, int s,
                                                  bool restricted, const DsParams& P) {
  return dsr_score(dsr_view(d, in, c, s, restricted, 0u), in, P);
}

// kSlotsInRegs = false: the slot record is read where used (the wide exact pass, register-bound); kExt = false: no
// reserve-pod / operating-mode / reservation-selector logic (the batched exact rounds; the host routes queues holding
// such pods to the per-pod pass); kXF = false: no RDMA / FPGA evaluation and no reserved-cpus NodeNUMAResource Score
// (the host picks it when the queue holds no RDMA / FPGA request and no reservation holds cpus: fewer registers)
template <bool kSlotsInRegs = true, bool kExt = true, bool kXF = true, bool kNuma = true, bool kDs = true>
__device__ __forceinline__ RsvOut rsv_eval_node(const DevTable& T, const RsvNode* __restrict__ RN,
                                                const int32_t* __restrict__ rsv_n, int64_t i, const DevPod& p,
                                                const RsvPod& rp, const EvalParams& P, const RsvParams& RP,
                                                const RsvExt& X, const DsPod* dp, const NumaPod* np = nullptr,
                                                RsvDbg* dbg = nullptr, const int64_t* aux_req = nullptr,
                                                const DefPod* df = nullptr) {
  RsvOut o{false, 0, 0, -1, 0x7fffffff, 0, 0, 0};
  NodePred npd{0, 0, 0, 0};
  if (df) {  // TaintToleration / NodeAffinity Filter: node-static, so first
    npd = X.pred[i];
    if (!dbg && !defaults_filter(npd, *df, X.DF)) return o;
  }
  Row r = load_row(T, i);
  const int ns = rsv_n[i];
  uint32_t mm = 0;  // matched slots
  uint32_t um = 0;  // unmatched slots with assigned pods (the restore's unmatched list)
  int nm = 0;
  int64_t pr_c = 0, pr_m = 0, ra_c = 0, ra_m = 0;
  bool has_state = false;
  // xr_eval reads the slot record where used instead of copying it: a 192-B copy live across the Fit / NUMA /
  // DeviceShare evaluation cost that pass a wave per SIMD (shipped profile: 256 VGPRs + AGPR spills → 239, occupancy
  // 1 → 2); the single-wave resolvers keep the copy (one batch of loads on their serial path)
  RsvNode rn_copy;
  if (kSlotsInRegs && ns > 0) rn_copy = RN[i];
  const RsvNode& rn = kSlotsInRegs ? rn_copy : RN[i];
  if (ns > 0)
    rsv_restore<kExt>(rn, ns, rp, X.rsv_pred ? X.rsv_pred + (size_t)i * kRsvSlots : nullptr,
                (rp.flags & RP_SEL) && X.rsv_sel ? X.rsv_sel + rp.aux : nullptr, r, mm, nm, pr_c, pr_m, ra_c, ra_m,
                has_state, &um);
  if (dbg) {
    dbg->matched = mm;
    dbg->has_state = has_state ? 1 : 0;
    dbg->req_cpu = r.req_cpu, dbg->req_mem = r.req_mem, dbg->nz_cpu = r.nz_cpu, dbg->nz_mem = r.nz_mem;
    dbg->num_pods = r.num_pods;
    dbg->pod_req_cpu = has_state ? pr_c : 0, dbg->pod_req_mem = has_state ? pr_m : 0;
  }
  if (dbg && df && !defaults_filter(npd, *df, X.DF)) return o;
  // Reservation.Filter of a reserve pod / a pod in reservation operating mode (plugin.go:324-350): the reservation's
  // node, and no available reservation whose allocate policy conflicts (Default coexists with no other policy)
  if (kExt && RP.filter && (rp.flags & (RP_RESERVE | RP_OPERATING))) {
    if ((rp.flags & RP_RESERVE) && rp.aux >= 0 && i != rp.aux) return o;
    const int32_t pol = (int32_t)((rp.flags >> RP_POLICY_SHIFT) & 3);
#pragma unroll
    for (int s = 0; s < kRsvSlots; ++s) {
      if (s >= ns || !(rn.meta[s] & RS_AVAIL)) continue;
      const int32_t ps = (int32_t)((rn.meta[s] >> 4) & 3);
      if ((pol == KG_RSV_POLICY_DEFAULT || ps == KG_RSV_POLICY_DEFAULT) && pol != ps) return o;
    }
  }
  int64_t t = 0;
  if (!eval_node(r, p, P, t)) return o;  // NodeResourcesFit + LoadAware on the restored NodeInfo
  // fitsRequest over ephemeral-storage and the scalar resources the pod requests (reservation/plugin.go:469-479)
  if (aux_req && P.fit_filter && !aux_fits(T, i, aux_req)) return o;
  // satisfied(s): filterWithReservations([s]) (plugin.go:384-428) with fitsNode (:433-482), preemptible = 0
  const bool kc = (p.flags & P_CPU_KEY) != 0, km = (p.flags & P_MEM_KEY) != 0;
  uint32_t sat = 0;
  if (has_state) {
    const bool pods_ok = !(r.num_pods - nm + 1 > r.alloc_pods);
    const bool zero = p.req_cpu == 0 && p.req_mem == 0;  // fitsNode: a zero request fits
#pragma unroll
    for (int s = 0; s < kRsvSlots; ++s) {
      if (!(mm >> s & 1)) continue;
      const bool hc = rn.alloc_cpu[s] > 0, hm = rn.alloc_mem[s] > 0;
      if (!((kc && hc) || (km && hm))) continue;  // Intersection(rInfo.ResourceNames, pod request names) empty
      const int64_t rc = rsv_nn(rn.alloc_cpu[s], rn.allocd_cpu[s]), rm = rsv_nn(rn.alloc_mem[s], rn.allocd_mem[s]);
      bool fits = pods_ok && (zero || (!(p.req_cpu > r.alloc_cpu - (pr_c - rc - ra_c)) &&
                                       !(p.req_mem > r.alloc_mem - (pr_m - rm - ra_m))));
      if (((rn.meta[s] >> 4) & 3) == KG_RSV_POLICY_RESTRICTED)  // LessThanOrEqual(podRequests, rRemained)
        fits = fits && (!hc || !kc || p.req_cpu <= rc) && (!hm || !km || p.req_mem <= rm);
      if (fits) sat |= 1u << s;
    }
  }
  // plugin.go:361-364, 423-426 (a reserve pod skips this part of the Filter, :357)
  if (RP.filter && (rp.flags & RP_AFFINITY) && !(kExt && (rp.flags & RP_RESERVE)) && sat == 0) return o;
  int64_t dsraw = 0;
  // (ABI 13) DeviceShare with the node's GPU-holding reservations (reservation.go, plugin.go:280-330): dsr = the
  // plugin keeps a restore state here; dsok = the GPU-holding matched slots it can allocate from (FilterReservation)
  bool dsr = false;
  uint32_t dsok = 0;
  DsrCtx dc{nullptr, 0u, 0u};
  DsInst din{0, 0, 0, 0, 0};
  if (kDs && X.ds && dp && !dp->skip) {
    const DsNode& d = X.ds[i];
    uint32_t gslots = 0;
    if (kExt && X.rgpu && has_state)  // the batched exact rounds never see GPU reservations (host routing)
#pragma unroll
      for (int s = 0; s < kRsvSlots; ++s) gslots |= (s < ns && (rn.meta[s] & RS_GPU)) ? (1u << s) : 0u;
    dsr = (gslots & (mm | um)) != 0 && !dp->error && d.has_device;
    if (!dsr) {  // the node-level Filter + raw Score
      if (!ds_eval(d, *dp, X.DP, dsraw)) return o;
    } else {
      din = ds_instance(d, *dp);
      if (!din.ok) return o;
      dc = DsrCtx{X.rgpu + (size_t)i * kRsvSlots, um & gslots, mm & gslots};
#pragma unroll
      for (int s = 0; s < kRsvSlots; ++s)
        if (((dc.mt >> s) & 1u) &&
            dsr_slot_ok(d, din, dc, s, ((rn.meta[s] >> 4) & 3) == KG_RSV_POLICY_RESTRICTED))
          dsok |= 1u << s;
      // Filter: a matched GPU reservation that fits, else (unless the pod requires a reservation) the node with every
      // matched reservation's allocatable returned
      bool pass = dsok != 0;
      if (!pass && !(dc.mt != 0 && (rp.flags & RP_AFFINITY))) {
        const DsrView v = dsr_view(d, din, dc, -1, false, 0u);
        pass = v.any && v.nfit >= din.count;
      }
      if (X.DP.filter && !pass) return o;
    }
    // FilterReservation: a pod with device requests can use only a GPU-holding reservation DeviceShare can allocate
    // from (plugin.go:333-380: "no relevant Reservation information" for the others)
    sat &= dsok;
    // (ABI 17) the RDMA / FPGA types of the request (the host routes such queues here and refuses them next to
    // GPU-holding reservations): Allocate needs every requested type, Score sums them
    if constexpr (kExt && kXF) {
      if (X.dsx && (dp->xq[0] | dp->xq[1])) {
        int64_t xraw = 0;
        if (!ds_eval_x(X.dsx[i], d.has_device != 0, *dp, X.DP, xraw)) return o;
        dsraw += xraw;
      }
    }
  }
  int64_t nsc = 0;        // NodeNUMAResource's Score without preferred cpus
  NumaHint naff{0, 1, 0, 0};
  if (kNuma && X.ns && np) {  // NodeNUMAResource Filter + Score on the restored NodeInfo; Reserve reuses the stored affinity
    const NumaView nv = make_view(X.ns + i, X.nm + i, X.NP);
    if (!numa_eval(nv, *np, X.NP, r.req_cpu, r.req_mem, r.alloc_cpu, r.alloc_mem, nsc, naff)) return o;
    if (X.NP.score) t += nsc * X.NP.weight;
    if (X.aff) X.aff[i] = naff.nil ? 0x100u : naff.mask;
  }
  if (df) {  // BalancedAllocation on the restored NodeInfo; the two normalised raw Scores
    if (X.DF.bal) t += X.DF.w_bal * balanced_score(r.alloc_cpu, r.alloc_mem, r.req_cpu, r.req_mem, p.req_cpu, p.req_mem, X.DF);
    if (X.DF.img) t += X.DF.w_img * image_score(npd, *df);
    o.tcnt = X.DF.taint_score ? taint_raw(npd, *df) : 0;
    o.asum = X.DF.aff_score ? affinity_raw(npd, *df) : 0;
  }
  o.feas = true;
  o.base = t;
  o.dsraw = X.DP.score ? (int32_t)dsraw : 0;
  if (has_state) {
    // PreScore node order over matched (scoring.go:66, 162-181); nomination over FilterReservation-passing slots
    int32_t best_all = 0x7fffffff, best_sat = 0x7fffffff;
    int pick = -1;
#pragma unroll
    for (int s = 0; s < kRsvSlots; ++s) {
      if (!(mm >> s & 1)) continue;
      const int32_t od = rn.order[s];
      if (od != 0 && best_all > od) best_all = od;
      if ((sat >> s & 1) && od != 0 && best_sat > od) {
        best_sat = od;
        pick = s;
      }
    }
    o.order = best_all;
    // every satisfied slot's score once (the nominated slot's is its raw Reservation Score)
    int32_t ssc[kRsvSlots];
#pragma unroll
    for (int s = 0; s < kRsvSlots; ++s) ssc[s] = (sat >> s & 1) ? rsv_score_slot(rn, s, p) : 0;
    if (pick < 0) {
      // (ABI 13) prioritizeReservations sums every reservation score plugin: DeviceShare's ScoreReservation
      // (scoreWithNominatedReservation) normalized by DefaultReservationNormalizeScore over the candidates
      int32_t dnorm[kRsvSlots] = {0, 0, 0, 0};
      if (dsr && sat) {
        int64_t dsc[kRsvSlots] = {0, 0, 0, 0}, dmax = 0;
#pragma unroll
        for (int s = 0; s < kRsvSlots; ++s)
          if (sat >> s & 1) {
            dsc[s] = dsr_slot_score(X.ds[i], din, dc, s, ((rn.meta[s] >> 4) & 3) == KG_RSV_POLICY_RESTRICTED, X.DP);
            dmax = dsc[s] > dmax ? dsc[s] : dmax;
          }
        if (dmax > 0)
#pragma unroll
          for (int s = 0; s < kRsvSlots; ++s) dnorm[s] = (sat >> s & 1) ? (int32_t)div_small(100 * dsc[s], dmax) : 0;
      }
      int32_t best = -1;
#pragma unroll
      for (int s = 0; s < kRsvSlots; ++s)
        if (sat >> s & 1) {
          if (ssc[s] + dnorm[s] > best) {  // prioritizeReservations + sort (unstable; pinned: lowest slot on ties)
            best = ssc[s] + dnorm[s];
            pick = s;
          }
        }
    }
    o.nom = pick;
    int32_t raw = 0;
#pragma unroll
    for (int s = 0; s < kRsvSlots; ++s)
      if (s == pick) raw = ssc[s];
    o.raw = raw;
    // (ABI 15) NodeNUMAResource Score runs after the PreScore nomination: a cpuset-capable pod nominated into a
    // reservation holding cpus gets its reserved cpus as preferredCPUs (getReservationReservedCPUs, plugin.go:513-535)
    if (kExt && kXF && kNuma && X.rcpu && X.ns && np && X.NP.score && np->allow && pick >= 0 && (rn.meta[pick] & RS_CPUS)) {
      const CpuSet P = rsv_reserved_cpus(X.rcpu[(size_t)i * kRsvSlots + pick]);
      if (cs_count(P) > 0) {
        const NumaView nv = make_view(X.ns + i, X.nm + i, X.NP);
        const int64_t psc = numa_score_pref(X.ns[i], X.nm[i], nv, *np, X.NP, naff, P, r.req_cpu, r.req_mem,
                                            r.alloc_cpu, r.alloc_mem);
        o.base += (psc - nsc) * X.NP.weight;
      }
    }
  }
  if (kDs && dsr && X.DP.score) {  // Score (scoring.go:34-89): the nominated reservation's, else the node view's
    const DsNode& d = X.ds[i];
    if (o.nom >= 0 && ((dc.mt >> o.nom) & 1u))
      dsraw = dsr_slot_score(d, din, dc, o.nom, ((rn.meta[o.nom] >> 4) & 3) == KG_RSV_POLICY_RESTRICTED, X.DP);
    else
      dsraw = dsr_score(dsr_view(d, din, dc, -1, false, 0u), din, X.DP);
    o.dsraw = (int32_t)dsraw;
  }
  return o;
}

// pass-1 value of a feasible node: base << 32 | dsraw << 16 | raw << 8 | feasible << 7 | (nom + 1)
__device__ __forceinline__ uint64_t rsv_pack(const RsvOut& o) {
  return ((uint64_t)(uint32_t)o.base << 32) | ((uint64_t)(uint32_t)o.dsraw << 16) | ((uint64_t)(uint32_t)o.raw << 8) |
         (1ull << 7) | (uint64_t)(o.nom + 1);
}
// PreScore preferred-node key of a feasible node with an order label: max = smallest order, then lowest index
__device__ __forceinline__ uint64_t rsv_pref_key(const RsvOut& o, uint32_t i) {
  return o.order != 0x7fffffff ? ~(((uint64_t)(uint32_t)o.order << 32) | (uint64_t)i) : 0ull;
}

constexpr int kRsvThreads = 256;  // 4 waves per block: fewer block partials to reduce per pass

// Block max of a u64 over its waves (DPP wave max, then LDS); result valid in thread 0.
__device__ __forceinline__ uint64_t rsv_block_max(uint64_t v, uint64_t* s_red) {
  v = wave_max_u64_dpp(v);
  const int w = threadIdx.x / kWave;
  if ((threadIdx.x & (kWave - 1)) == 0) s_red[w] = v;
  __syncthreads();
  if (threadIdx.x == 0)
    for (int k = 1; k < kRsvThreads / kWave; ++k) v = s_red[k] > v ? s_red[k] : v;
  return v;
}

// Max over `nb` per-block partials, computed by one wave (every lane returns it).
__device__ __forceinline__ uint64_t rsv_partials_max(const uint64_t* __restrict__ part, int nb) {
  uint64_t v = 0;
  for (int k = threadIdx.x & (kWave - 1); k < nb; k += kWave) v = part[k] > v ? part[k] : v;
  return wave_max_u64_dpp(v);
}
// Block sum (thread 0 holds it) and the sum of `nb` partials (every lane)
__device__ __forceinline__ uint64_t rsv_block_sum(uint32_t v, uint64_t* s_red) {
  v = wave_sum_u32(v);
  const int w = threadIdx.x / kWave;
  if ((threadIdx.x & (kWave - 1)) == 0) s_red[w] = v;
  __syncthreads();
  uint64_t t = 0;
  if (threadIdx.x == 0)
    for (int k = 0; k < kRsvThreads / kWave; ++k) t += s_red[k];
  return t;
}
__device__ __forceinline__ uint64_t rsv_partials_sum(const uint64_t* __restrict__ part, int nb) {
  uint32_t v = 0;
  for (int k = threadIdx.x & (kWave - 1); k < nb; k += kWave) v += (uint32_t)part[k];
  return wave_sum_u32(v);
}

// DeviceShare Reserve on one node (one thread): the first `count` fitting minors in (score desc, minor asc) order
// (defaultAllocateDevices device_allocator.go:384-454 + sortDeviceResourcesByMinor device_resources.go:187-208),
// then nodeDevice.updateCacheUsed (device_cache.go:124-135).  Returns the minor mask, -1 if no allocation.
__device__ __forceinline__ int32_t rsv_ds_reserve(DsNode& dn, const DsPod& dp, const DsParams& DP) {
  if (dp.skip || !dn.has_device) return 0;
  if (dp.error) return -1;
  if (dp.nogpu) return 0;  // (ABI 17) only RDMA / FPGA requests: no GPU minor
  const DsInst in = ds_instance(dn, dp);
  if (!in.ok) return -1;
  int64_t sc[kMinors];
  uint32_t fit = 0;
  bool any = false;
#pragma unroll
  for (int m = 0; m < kMinors; ++m) {
    bool f = false, nz = false;
    sc[m] = ds_minor(dn, m, in, DP, f, nz);
    any |= nz;
    fit |= f ? (1u << m) : 0u;
  }
  if (!any || __popc(fit) < in.count) return -1;
  uint32_t taken = 0;
  for (int k = 0; k < in.count; ++k) {
    int best = -1;
#pragma unroll
    for (int m = 0; m < kMinors; ++m)
      if (((fit & ~taken) >> m) & 1u)
        if (best < 0 || sc[m] > sc[best]) best = m;
    taken |= 1u << best;
  }
#pragma unroll
  for (int m = 0; m < kMinors; ++m)
    if ((taken >> m) & 1u) {
      dn.ucore[m] += (int32_t)in.core;
      dn.uratio[m] += (int32_t)in.ratio;
      dn.umem[m] += in.mem;
    }
  return (int32_t)taken;
}

// (ABI 13) Allocate over a view (device_allocator.go:89-129, 384-454 + sortDeviceResourcesByMinor): the first `count`
// fitting minors in (preferred first, scoreDevice desc, minor asc) order, within `req` when set.  -1 = Insufficient.
__device__ __forceinline__ int32_t dsr_allocate(const DsNode& d, const DsInst& in, const DsrCtx& c, int slot, bool rr,
                                                uint32_t req, uint32_t pref, const DsParams& P) {
  const uint32_t minors = rr ? c.g[slot].minors & (uint32_t)d.present : (uint32_t)d.present;
  int64_t sc[kMinors];
  uint32_t fit = 0;
  bool any = false;
  const bool most = P.most != 0;
  for (int m = 0; m < kMinors; ++m) {
    sc[m] = 0;
    if (!((minors >> m) & 1u)) continue;
    int64_t f[3];
    dsr_free(d, c, m, slot, rr, f);
    const bool nz = (f[0] | f[1] | f[2]) != 0;
    any |= nz;
    if (nz && (!req || ((req >> m) & 1u)) && in.core <= f[0] && in.mem <= f[1] && in.ratio <= f[2]) fit |= 1u << m;
    int64_t num = 0, ws = 0;  // scoreDevice (scoring.go:183-203)
    ds_term(P.w_core, ds_tot(d, m, 0), f[0], in.core, num, ws, most);
    ds_term(P.w_mem, ds_tot(d, m, 1), f[1], in.mem, num, ws, most);
    ds_term(P.w_ratio, ds_tot(d, m, 2), f[2], in.ratio, num, ws, most);
    sc[m] = ws ? div_small(num, ws) : 0;
  }
  if (!any || __popc(fit) < in.count) return -1;
  uint32_t taken = 0;
  for (int k = 0; k < in.count; ++k) {
    int best = -1;
    for (int m = 0; m < kMinors; ++m) {
      if (!(((fit & ~taken) >> m) & 1u)) continue;
      if (best < 0) {
        best = m;
        continue;
      }
      const int pm = (pref >> m) & 1, pb = (pref >> best) & 1;
      if (pm > pb || (pm == pb && sc[m] > sc[best])) best = m;
    }
    taken |= 1u << best;
  }
  return (int32_t)taken;
}

// (ABI 13) DeviceShare Reserve with the node's GPU-holding reservations (plugin.go:388-437): the nominated reservation
// alone (allocateWithNominatedReservation → tryAllocateFromReservation, not required; none for a reserve pod), else the
// node view; updateCacheUsed adds the per-instance request to the allocated minors.  -1 = no allocation.
__device__ __forceinline__ int32_t rsv_ds_reserve_gpu(DsNode& dn, const DsPod& dp, const DsParams& DP, const DsrCtx& c,
                                                      int nominated, bool restricted, bool reserve_pod) {
  if (dp.skip || !dn.has_device) return 0;
  if (dp.error) return -1;
  if (dp.nogpu) return 0;  // (ABI 17) only RDMA / FPGA requests: no GPU minor
  const DsInst in = ds_instance(dn, dp);
  if (!in.ok) return -1;
  int32_t mask = -1;
  if (nominated >= 0 && ((c.mt >> nominated) & 1u) && !reserve_pod) {
    const uint32_t pref = c.g[nominated].minors;
    if (restricted) {
      const DsrView v1 = dsr_view(dn, in, c, nominated, false, pref);
      if (v1.any && v1.nfit >= in.count) mask = dsr_allocate(dn, in, c, nominated, true, pref, pref, DP);
    } else {
      mask = dsr_allocate(dn, in, c, nominated, false, 0u, pref, DP);
    }
  }
  if (mask < 0) mask = dsr_allocate(dn, in, c, -1, false, 0u, 0u, DP);
  if (mask <= 0) return mask;
#pragma unroll
  for (int m = 0; m < kMinors; ++m)
    if ((mask >> m) & 1) {
      dn.ucore[m] += (int32_t)in.core;
      dn.uratio[m] += (int32_t)in.ratio;
      dn.umem[m] += in.mem;
    }
  return mask;
}

// the pod's allocation on reservation slot s's minors (appendAllocatedByHints): sign +1 when assumed into it, −1 when
// it leaves (SubtractWithNonNegativeResult)
__device__ __forceinline__ void rsv_gpu_assign(RsvGpu& g, const DsInst& in, int32_t mask, int sign) {
  const uint32_t mm = (uint32_t)mask & g.minors;
  for (int m = 0; m < kMinors; ++m) {
    if (!((mm >> m) & 1u)) continue;
    const int64_t c = (int64_t)g.dcore[m] + sign * in.core, r = (int64_t)g.dratio[m] + sign * in.ratio,
                  b = g.dmem[m] + sign * in.mem;
    g.dcore[m] = (int32_t)(c > 0 ? c : 0);
    g.dratio[m] = (int32_t)(r > 0 ? r : 0);
    g.dmem[m] = b > 0 ? b : 0;
  }
}

__device__ __forceinline__ void rsv_quota_charge(const RsvExt& X, const DevPod& p, int64_t j) {
  if (X.nq == 0 || p.quota < 0) return;
  quota_row_charge(X.quotas[p.quota], quota_req(p, X.qdev + (size_t)j * kQuotaRes), (p.flags & P_NONPREEMPT) != 0);
}

// Reserve of pod j on its winner row w: DeviceShare first (a failure un-assumes the pod: nothing is placed), then
// NodeInfo + LoadAware assign cache and reservationCache.assumePod on the slot nominated there
// (reservation_info.go:317-326).  Called by the one thread that owns row w.  Returns false when not placed.
template <bool NUMA = true, bool DS = true, bool kXF = true>  // compile-time: the profile's plugins (see rsv_eval_node)
__device__ __forceinline__ bool rsv_reserve(const DevTable& T, RsvNode* __restrict__ RN, int64_t w, uint64_t v,
                                            const DevPod& p, const RsvExt& X, int64_t j, int32_t& slot_out,
                                            int diag_j = -1) {
  (void)diag_j;  // KG_STAMPS builds: the round-local pod index of the lane stamps
  slot_out = -1;
  KG_LANE_SUB(diag_j, 0);
  // NodeNUMAResource Reserve first (the profile's Reserve order), computed on copies: nothing is committed unless
  // every Reserve succeeds
  NumaMut nmw;
  CpuSet cpus = cs_zero();
  NumaAlloc rec;
  rec.res = 0;
  const int32_t nom_slot = (int32_t)(v & 7) - 1;  // the slot PreScore nominated on the winner (-1: none)
  if (NUMA && X.ns) {
    const NumaStatic nsw = X.ns[w];
    nmw = X.nm[w];
    const NumaView nv = make_view(&nsw, &nmw, X.NP);
    const uint32_t a = X.aff[w];
    const NumaHint aff{a & 0xFFu, (int)((a >> 8) & 1u), 0, 0};
    // (ABI 15) the nominated reservation's reserved cpus are Reserve's preferredCPUs too (getResourceOptions)
    CpuSet P = cs_zero();
    if (kXF && X.rcpu && nom_slot >= 0 && X.npods[j].allow && (RN[w].meta[nom_slot] & RS_CPUS))
      P = rsv_reserved_cpus(X.rcpu[(size_t)w * kRsvSlots + nom_slot]);
    const bool ok = cs_count(P) > 0 ? numa_reserve_pref(nsw, nmw, nv, X.npods[j], aff, P, cpus, rec)
                                    : numa_reserve(nsw, nmw, nv, X.npods[j], aff, cpus, rec);
    if (!ok) {
      if (X.out_minors) X.out_minors[j] = 0;
      return false;
    }
  }
  KG_LANE_SUB(diag_j, 1);
  int32_t gpu_minors = 0;  // (ABI 13) the DeviceShare allocation, for the reservation's allocated GPUs below
  if (DS && X.ds) {
    DsNode dn = X.ds[w];
    int32_t minors = 0;
    bool done = false;
    // (ABI 13) the winner's DeviceShare restore again (reservation.go:118-171) when it holds GPU reservations
    if (X.rgpu && X.rsv_n && X.rpods && !X.dpods[j].skip) {
      const int ns = X.rsv_n[w];
      uint32_t gslots = 0;
      for (int s = 0; s < kRsvSlots; ++s) gslots |= (s < ns && (RN[w].meta[s] & RS_GPU)) ? (1u << s) : 0u;
      if (gslots) {
        const RsvNode rn = RN[w];
        const RsvPod rp = X.rpods[j];
        Row rr = load_row(T, w);
        uint32_t mm = 0, um = 0;
        int nm = 0;
        int64_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
        bool hs = false;
        rsv_restore<true>(rn, ns, rp, X.rsv_pred ? X.rsv_pred + (size_t)w * kRsvSlots : nullptr,
                          (rp.flags & RP_SEL) && X.rsv_sel ? X.rsv_sel + rp.aux : nullptr, rr, mm, nm, a0, a1, a2, a3,
                          hs, &um);
        if (hs && (gslots & (mm | um))) {
          const DsrCtx c{X.rgpu + (size_t)w * kRsvSlots, um & gslots, mm & gslots};
          const int nom = (int)(v & 7) - 1;
          minors = rsv_ds_reserve_gpu(dn, X.dpods[j], X.DP, c, nom,
                                      nom >= 0 && ((rn.meta[nom] >> 4) & 3) == KG_RSV_POLICY_RESTRICTED,
                                      (rp.flags & RP_RESERVE) != 0);
          done = true;
        }
      }
    }
    if (!done) minors = rsv_ds_reserve(dn, X.dpods[j], X.DP);
    KG_LANE_SUB(diag_j, 2);
    // (ABI 17) the RDMA / FPGA types, on a copy: every requested type is allocated or none is
    int32_t xminors = 0;
    DsXNode xn;
    const bool xreq = kXF && X.dsx && (X.dpods[j].xq[0] | X.dpods[j].xq[1]);
    if (xreq && minors >= 0) {
      xn = X.dsx[w];
      xminors = ds_reserve_x(xn, dn.has_device != 0, X.dpods[j], X.DP);
    }
    if (minors < 0 || xminors < 0) {
      X.out_minors[j] = 0;
      return false;
    }
    if (minors) const_cast<DsNode*>(X.ds)[w] = dn;
    if (xminors) X.dsx[w] = xn;
    X.out_minors[j] = minors | xminors;
    gpu_minors = minors;
  }
  if (NUMA && X.ns) {
    X.nm[w] = nmw;
#pragma unroll
    for (int q = 0; q < kCpuWords; ++q) X.out_cpus[(size_t)j * kCpuWords + q] = cpus.w[q];
    int64_t* r = X.out_nrec + (size_t)j * kNumaRecWords;
    r[0] = rec.res;
#pragma unroll
    for (int k = 0; k < kNumaMax; ++k) {
      r[1 + k] = ((rec.res >> k) & 1u) ? rec.cpu[k] : 0;
      r[1 + kNumaMax + k] = ((rec.res >> k) & 1u) ? rec.mem[k] : 0;
    }
  }
  KG_LANE_SUB(diag_j, 3);
  Row r = load_row(T, w);
  const int64_t prod = (p.flags & P_PROD) ? 1 : 0;
  if (X.paux && (p.flags & P_AUX))  // NodeInfo.Requested of ephemeral-storage / the scalar resources
#pragma unroll
    for (int q = 0; q < kAux; ++q) T.aux[(size_t)(kAux + q) * T.cap + w] += X.paux[(size_t)j * kAux + q];
  r.req_cpu += p.req_cpu;
  r.req_mem += p.req_mem;
  r.nz_cpu += p.nz_cpu;
  r.nz_mem += p.nz_mem;
  r.la_used_cpu += p.est_cpu;
  r.la_used_mem += p.est_mem;
  r.la_pused_cpu += prod * p.est_cpu;
  r.la_pused_mem += prod * p.est_mem;
  r.num_pods += 1;
  store_mutable(T, w, r);
  if (X.gpods) group_apply(X.G, w, X.gpods[j], +1, X.GP.hard_w);  // the node's pod-group counters
  KG_LANE_SUB(diag_j, 4);
  const int32_t slot = (int32_t)(v & 7) - 1;
  if (slot >= 0) {  // Allocated += quotav1.Mask(requests, ResourceNames): only the reservation's keys (0 = absent)
    if (RN[w].alloc_cpu[slot] > 0) RN[w].allocd_cpu[slot] += p.req_cpu;
    if (RN[w].alloc_mem[slot] > 0) RN[w].allocd_mem[slot] += p.req_mem;
    RN[w].assigned[slot] += 1;
    // (ABI 13) the reservation's allocated GPUs: the pod's allocation on its minors
    if (DS && X.rgpu && gpu_minors > 0 && (RN[w].meta[slot] & RS_GPU))
      rsv_gpu_assign(X.rgpu[(size_t)w * kRsvSlots + slot], ds_instance(X.ds[w], X.dpods[j]), gpu_minors, +1);
    // (ABI 15) an assigned pod's cpus leave the reservation's reserved cpus at the next RestoreReservation
    if (kXF && NUMA && X.rcpu && X.ns && (RN[w].meta[slot] & RS_CPUS)) {
      RsvCpu& rc = X.rcpu[(size_t)w * kRsvSlots + slot];
#pragma unroll
      for (int q = 0; q < kCpuWords; ++q) rc.u[q] |= cpus.w[q];
    }
  }
  slot_out = slot;
  KG_LANE_SUB(diag_j, 5);
  return true;
}

// Pass 1 for pod j = cursor + g: first the Reserve of pod j - 1 (g > 0; its winner is the max of the previous
// rsv_select's block keys — the thread owning that row applies it, so no separate launch), then per-node Filter +
// Fit/LoadAware total + nominated slot and raw Scores.  val[i] = base << 32 | dsraw << 16 | raw << 8 | feasible << 7 |
// (nom + 1), 0 = filtered.  Per-block partials (no same-address atomics): part[b] = max ~(order << 32 | node) over
// feasible nodes with an order label (PreScore preferred node, 0 = none), part[nb + b] = max raw Reservation Score,
// part[3 nb + b] = max raw DeviceShare Score.
// ElasticQuota: pod j's PreFilter must see the Reserve of every earlier pod.  The quota rows hold the charges of
// pods < j - 1 (pod j - 2 was charged by rsv_select(j - 1)); pod j - 1's charge is added here explicitly when it was
// placed (g > 0; a group's last pod is charged by rsv_apply itself), and written into the rows by rsv_select(j), when
// no pass reads them (ws[0] = j tags it).
// F = RSV_F_* bits, compile-time: kernels without the plugins the profile lacks need fewer registers
constexpr int RSV_F_XF = 1, RSV_F_NUMA = 2, RSV_F_DS = 4;  // XF: X.dsx or X.rcpu set (see rsv_eval_node)
template <int F>
__global__ __launch_bounds__(kRsvThreads) void rsv_eval(DevTable T, RsvNode* __restrict__ RN,
                                                        const int32_t* __restrict__ rsv_n,
                                                        const DevPod* __restrict__ pods,
                                                        const RsvPod* __restrict__ rpods, int64_t end, int64_t n,
                                                        int g, EvalParams P, RsvParams RP, RsvExt X,
                                                        uint64_t* __restrict__ val, uint64_t* __restrict__ part,
                                                        uint64_t* __restrict__ out_keys, int32_t* __restrict__ out_slot,
                                                        unsigned long long* __restrict__ ws) {
  __shared__ uint64_t s_red[kRsvThreads / kWave];
  __shared__ int s_admit;
  if (end < 0) end = (int64_t)ws[4];  // graph launches: the call's end lives in the workspace
  const int64_t j = (int64_t)ws[3] + g;
  if (j - 1 >= end || (g == 0 && j >= end)) return;  // uniform across the grid
  const int nb = gridDim.x;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool prev_placed = false;
  if (g > 0) {  // Reserve of pod j - 1 (group profiles: group_pre ran it before this pass)
    const uint64_t k = rsv_partials_max(part + 2 * nb, nb);
    const int64_t w = k ? (int64_t)key_node(k) : -1;
    if (!X.gpods && (i == w || (w < 0 && i == 0))) {
      int32_t slot = -1;
      bool placed = false;
      if (w >= 0) placed = rsv_reserve<(F & RSV_F_NUMA) != 0, (F & RSV_F_DS) != 0, (F & RSV_F_XF) != 0>(T, RN, w, val[w],
                                                                                              pods[j - 1], X, j - 1,
                                                                                              slot);
      out_keys[j - 1] = placed ? k : 0;
      out_slot[j - 1] = slot;
      if (placed && X.nq > 0 && pods[j - 1].quota >= 0) {
        if (j >= end) rsv_quota_charge(X, pods[j - 1], j - 1);  // no later pass charges it
        else ws[0] = (unsigned long long)j;                     // rsv_select(j) charges it
      }
    }
    if (j >= end) return;
    prev_placed = k != 0;  // (a DeviceShare Reserve failure leaves it unplaced: only the ds dims could disagree)
  }
  const DevPod p = pods[j];
  if (threadIdx.x == 0) {  // ElasticQuota PreFilter of pod j (the same verdict in every block)
    int ok = 1;
    if (X.nq > 0 && p.quota >= 0) {
      const QuotaReq rq = quota_req(p, X.qdev + (size_t)j * kQuotaRes);
      int64_t au[kQuotaRes] = {}, an[kQuotaRes] = {};
      if (prev_placed) {
        const DevPod pp = pods[j - 1];
        if (pp.quota == p.quota) {
          const QuotaReq pr = quota_req(pp, X.qdev + (size_t)(j - 1) * kQuotaRes);
          const bool npp = (pp.flags & P_NONPREEMPT) != 0;
#pragma unroll
          for (int d = 0; d < kQuotaRes; ++d) au[d] = pr.r[d], an[d] = npp ? pr.r[d] : 0;
        }
      }
      ok = quota_row_admit(X.quotas[p.quota], rq, (p.flags & P_NONPREEMPT) != 0, au, an) ? 1 : 0;
    }
    s_admit = ok;
  }
  uint64_t pk = 0, rawv = 0, dsv = 0, tv = 0, av = 0;
  uint64_t v = 0;
  int32_t iraw = 0;      // InterPodAffinity raw Score of a feasible node
  bool ign = false;      // PodTopologySpread IgnoredNodes: a feasible node lacking a ScheduleAnyway key
  int32_t zone = 0;
  int64_t total = 0;
  GroupPod gp{};
  ZoneSums Z{};
  uint64_t pres = 0;
  __shared__ int64_t s_min[kSpread];
  if (X.gpods) {  // group_pre's reductions over the snapshot after pod j - 1's Reserve
    gp = X.gpods[j];
    Z = zone_sums(X, j);
    pres = *Z.pres;
    const uint64_t e = rsv_partials_max(part + 6 * nb, nb);
    total = (int64_t)rsv_partials_sum(part + 7 * nb, nb);
    if (threadIdx.x < kWave) {  // minMatchNum per DoNotSchedule constraint (MaxInt32 without pairs)
      for (int c = 0; c < gp.nsp; ++c) {
        if (!(gp.sp_flags[c] & KG_SPREAD_HARD)) continue;
        int64_t m = 0x7fffffff;
        if (gp.sp_flags[c] & KG_SPREAD_ZONE) {
          const uint64_t v = ((pres >> threadIdx.x) & 1ull) ? enc_min_i32(Z.zf[c * kZones + threadIdx.x]) : 0;
          const uint64_t mv = wave_max_u64_dpp(v);
          const uint64_t mm = readlane_u64(mv, kWave - 1);
          if (mm) m = dec_min_i32(mm);
        } else if (e) {
          m = dec_min_i32(e);
        }
        if (threadIdx.x == 0) s_min[c] = m;
      }
    }
    __syncthreads();
  }
  if (i < n) {
    const RsvPod rp = rpods[j];
    const DsPod* dp = X.ds ? &X.dpods[j] : nullptr;
    const NumaPod* np = X.ns ? &X.npods[j] : nullptr;
    const int64_t* aux = (X.paux && (p.flags & P_AUX)) ? X.paux + (size_t)j * kAux : nullptr;
    const DefPod* df = X.defp ? &X.defp[j] : nullptr;
    RsvOut o = rsv_eval_node<true, true, (F & RSV_F_XF) != 0, (F & RSV_F_NUMA) != 0, (F & RSV_F_DS) != 0>(
        T, RN, rsv_n, i, p, rp, P, RP, X, dp, np, nullptr, aux, df);
    if (o.feas && X.gpods) {
      zone = X.pred[i].zone;
      o.feas = groups_filter(X.G, i, gp, X.GP, node_affinity_match(X.pred, df, i), zone, s_min, Z, pres, total);
      if (o.feas) {
        ign = !spread_sysdef(gp) && !spread_has_keys(gp, 1, zone);
        iraw = interpod_raw(X.G, i, gp, zone, Z);
      }
    }
    if (o.feas) {
      v = rsv_pack(o);
      pk = rsv_pref_key(o, (uint32_t)i);
      rawv = (uint64_t)(uint32_t)o.raw;
      dsv = (uint64_t)(uint32_t)o.dsraw;
      tv = (uint64_t)(uint32_t)o.tcnt;
      av = (uint64_t)(uint32_t)o.asum;
    }
  }
  __syncthreads();
  if (!s_admit) v = 0, pk = 0, rawv = 0, dsv = 0, tv = 0, av = 0;  // PreFilter Unschedulable: no node is feasible
  if (i < n) val[i] = v;
  const bool dscore = X.val2 != nullptr;  // TaintToleration / NodeAffinity Score in the profile
  if (dscore && i < n) X.val2[i] = (uint32_t)(tv << 24 | av);
  if (X.gpods) {  // the PreScore / NormalizeScore inputs of both plugins over the filtered nodes
    const bool f = (v >> 7) & 1u;
    if (i < n) X.gval[i] = ((uint64_t)(uint32_t)iraw << 32) | (uint32_t)(zone << 1 | (ign ? 1 : 0));
    const uint64_t fc = rsv_block_sum(f ? 1u : 0u, s_red);
    __syncthreads();
    // ignored nodes; for a system-defaulted pod (none ignored), the filtered nodes without a zone label (the empty
    // zone value's domain)
    const uint64_t ic = rsv_block_sum(f && (spread_sysdef(gp) ? zone <= 0 : ign) ? 1u : 0u, s_red);
    __syncthreads();
    const uint64_t ix = rsv_block_max(f ? enc_max_i32(iraw) : 0, s_red);
    __syncthreads();
    const uint64_t in = rsv_block_max(f ? enc_min_i32(iraw) : 0, s_red);
    __syncthreads();
    // the zones of the filtered, not ignored nodes (a zone constraint's topology size)
    uint64_t zm = (f && !ign && zone > 0) ? 1ull << (zone - 1) : 0;
    for (int d = 1; d < kWave; d <<= 1) {
      const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)zm, d), hi = (uint32_t)__shfl_xor((int)(uint32_t)(zm >> 32), d);
      zm |= ((uint64_t)hi << 32) | lo;
    }
    if ((threadIdx.x & (kWave - 1)) == 0) s_red[threadIdx.x / kWave] = zm;
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int w = 1; w < kRsvThreads / kWave; ++w) zm |= s_red[w];
      part[8 * nb + blockIdx.x] = fc;
      part[9 * nb + blockIdx.x] = ix;
      part[10 * nb + blockIdx.x] = in;
      part[11 * nb + blockIdx.x] = ic;
      part[12 * nb + blockIdx.x] = zm;
    }
    __syncthreads();
  }
  pk = rsv_block_max(pk, s_red);
  __syncthreads();
  rawv = rsv_block_max(rawv, s_red);
  __syncthreads();
  dsv = rsv_block_max(dsv, s_red);
  if (dscore) {
    __syncthreads();
    tv = rsv_block_max(tv, s_red);
    __syncthreads();
    av = rsv_block_max(av, s_red);
  }
  if (threadIdx.x == 0) {
    part[blockIdx.x] = pk;
    part[nb + blockIdx.x] = rawv;
    part[3 * nb + blockIdx.x] = dsv;
    if (dscore) part[4 * nb + blockIdx.x] = tv, part[5 * nb + blockIdx.x] = av;
  }
}

// The weighted total of one feasible node from its pass-1 value: PreScore preferred node (1000), DefaultNormalizeScore
// of the Reservation / DeviceShare / TaintToleration / NodeAffinity raw Scores against the feasible nodes' maxima
// (mx already max(raw, 1000) when a preferred node exists), × weights.  Shared by rsv_select and the batched rounds.
__device__ __forceinline__ int64_t rsv_total(uint64_t v, uint32_t v2, bool is_pref, int64_t mx, int64_t mds,
                                             int64_t mt, int64_t ma, const RsvParams& RP, const RsvExt& X) {
  const int64_t raw = is_pref ? 1000 : (int64_t)((v >> 8) & 0xff);  // mostPreferredScore
  int64_t t = (int64_t)(v >> 32);
  if (RP.score && mx > 0) t += (int64_t)RP.weight * div_small(100 * raw, mx);
  if (X.DP.score && mds > 0) t += (int64_t)X.DP.weight * div_small(100 * (int64_t)((v >> 16) & 0xff), mds);
  if (X.DF.taint_score) t += (int64_t)X.DF.w_taint * normalize_default(v2 >> 24, mt, true);
  if (X.DF.aff_score) t += (int64_t)X.DF.w_aff * normalize_default(v2 & 0xFFFFFFu, ma, false);
  return t;
}

// Pass 2: PreScore preferred node (1000), DefaultNormalizeScore of both plugins over the feasible nodes, × weights,
// packed key; part[2 nb + b] = the block's max key.  Block 0 also charges pod j - 1's quota (tagged ws[0] = j).
// (ABI 12) Group profiles: this pass computes PodTopologySpread's raw Score per node (its weights need the filtered
// count and zones) with its extremes — part[13 nb + b] / part[14 nb + b] — and rsv_select2 makes the keys.
__device__ __forceinline__ uint64_t select_key(const uint64_t* __restrict__ val, int64_t i, int64_t n, int nb,
                                               const RsvParams& RP, const RsvExt& X,
                                               const uint64_t* __restrict__ part) {
  const uint64_t pk = rsv_partials_max(part, nb);
  const uint64_t mraw = rsv_partials_max(part + nb, nb);
  const uint64_t mds = X.ds ? rsv_partials_max(part + 3 * nb, nb) : 0;
  const int64_t mt = X.val2 ? (int64_t)rsv_partials_max(part + 4 * nb, nb) : 0;
  const int64_t ma = X.val2 ? (int64_t)rsv_partials_max(part + 5 * nb, nb) : 0;
  const int64_t pref = pk ? (int64_t)(uint32_t)(~pk) : -1;
  const int64_t mx = pk ? (mraw > 1000 ? (int64_t)mraw : 1000) : (int64_t)mraw;
  int64_t smin = 0, smax = 0, imin = 0, imax = 0;
  if (X.gpods) {
    const uint64_t sx = rsv_partials_max(part + 13 * nb, nb), sn = rsv_partials_max(part + 14 * nb, nb);
    const uint64_t ix = rsv_partials_max(part + 9 * nb, nb), in = rsv_partials_max(part + 10 * nb, nb);
    smax = sx ? dec_max_i32(sx) : 0;
    smin = sn ? dec_min_i32(sn) : 0;
    imax = ix ? dec_max_i32(ix) : 0;
    imin = in ? dec_min_i32(in) : 0;
  }
  uint64_t key = 0;
  if (i < n) {
    const uint64_t v = val[i];
    if (v & (1ull << 7)) {
      const uint32_t v2 = X.val2 ? X.val2[i] : 0u;
      int64_t t = rsv_total(v, v2, i == pref, mx, (int64_t)mds, mt, ma, RP, X);
      if (X.gpods) {
        const uint64_t gv = X.gval[i];
        const uint32_t sr = (uint32_t)gv;  // the spread raw + 2^31, 0 = ignored (NormalizeScore gives it 0)
        if (X.GP.spread_score && sr != 0)
          t += (int64_t)X.GP.w_spread * spread_normalize((int64_t)sr - 0x80000000ll, smin, smax);
        if (X.GP.ipa_score) t += (int64_t)X.GP.w_ipa * interpod_normalize((int32_t)(gv >> 32), imin, imax);
      }
      key = make_key(t, (uint32_t)i);
    }
  }
  return key;
}

__global__ __launch_bounds__(kRsvThreads) void rsv_select(const uint64_t* __restrict__ val, const DevPod* __restrict__ pods,
                                                          int64_t end, int64_t n, int g, RsvParams RP, RsvExt X,
                                                          uint64_t* __restrict__ part,
                                                          unsigned long long* __restrict__ ws) {
  __shared__ uint64_t s_red[kRsvThreads / kWave];
  if (end < 0) end = (int64_t)ws[4];
  const int64_t j = (int64_t)ws[3] + g;
  if (j >= end) return;
  const int nb = gridDim.x;
  if (blockIdx.x == 0 && threadIdx.x == 0 && X.nq > 0 && g > 0 && ws[0] == (unsigned long long)j)
    rsv_quota_charge(X, pods[j - 1], j - 1);
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (!X.gpods) {
    const uint64_t key = rsv_block_max(select_key(val, i, n, nb, RP, X, part), s_red);
    if (threadIdx.x == 0) part[2 * nb + blockIdx.x] = key;
    return;
  }
  // PodTopologySpread PreScore + Score: weights log(F − ignored + 2) (hostname) and log(#zones + 2) (zone)
  const GroupPod gp = X.gpods[j];
  const ZoneSums Z = zone_sums(X, j);
  const int64_t F = (int64_t)rsv_partials_sum(part + 8 * nb, nb), ig = (int64_t)rsv_partials_sum(part + 11 * nb, nb);
  uint64_t zm = 0;
  for (int k = threadIdx.x & (kWave - 1); k < nb; k += kWave) zm |= part[12 * nb + k];
  for (int d = 1; d < kWave; d <<= 1) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)zm, d), hi = (uint32_t)__shfl_xor((int)(uint32_t)(zm >> 32), d);
    zm |= ((uint64_t)hi << 32) | lo;
  }
  const bool sd = spread_sysdef(gp);  // (ABI 13) part[11] counts the filtered nodes without a zone label instead
  const int64_t hs = sd ? F : F - ig;
  const double w_host = X.logw[hs < 0 ? 0 : (hs < n ? hs : n)], w_zone = X.logw[__popcll(zm) + (sd && ig > 0 ? 1 : 0)];
  int32_t raw = 0;
  bool on = false;
  if (i < n && ((val[i] >> 7) & 1u)) {
    const uint64_t gv = X.gval[i];
    on = (gv & 1u) == 0;  // not ignored
    if (on) {
      raw = (int32_t)spread_raw(X.G, i, gp, (int32_t)((uint32_t)gv >> 1), Z.zs, w_host, w_zone);
      X.gval[i] = (gv & 0xFFFFFFFF00000000ull) | (uint32_t)((int64_t)raw + 0x80000000ll);
    } else {
      X.gval[i] = gv & 0xFFFFFFFF00000000ull;
    }
  }
  const uint64_t sx = rsv_block_max(on ? enc_max_i32(raw) : 0, s_red);
  __syncthreads();
  const uint64_t sn = rsv_block_max(on ? enc_min_i32(raw) : 0, s_red);
  if (threadIdx.x == 0) {
    part[13 * nb + blockIdx.x] = sx;
    part[14 * nb + blockIdx.x] = sn;
  }
  // pod j + 1's zone sums start from zero (pod j - 1 was their last reader)
  if (blockIdx.x == 0) {
    const ZoneSums Zn = zone_sums(X, j + 1);
    for (int k = threadIdx.x; k < kZoneSumWords; k += kRsvThreads) Zn.zf[k] = 0;
    if (threadIdx.x == 0) *Zn.pres = 0;
  }
}

// (ABI 12) Pass 3 of group profiles: the keys (the same weighted total as rsv_select, with both plugins' NormalizeScore)
__global__ __launch_bounds__(kRsvThreads) void rsv_select2(const uint64_t* __restrict__ val, int64_t end, int64_t n,
                                                           int g, RsvParams RP, RsvExt X, uint64_t* __restrict__ part,
                                                           const unsigned long long* __restrict__ ws) {
  __shared__ uint64_t s_red[kRsvThreads / kWave];
  if (end < 0) end = (int64_t)ws[4];
  const int64_t j = (int64_t)ws[3] + g;
  if (j >= end) return;
  const int nb = gridDim.x;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t key = rsv_block_max(select_key(val, i, n, nb, RP, X, part), s_red);
  if (threadIdx.x == 0) part[2 * nb + blockIdx.x] = key;
}

// (ABI 12) Pass 0 of group profiles for pod j = cursor + g: the Reserve of pod j - 1 (as rsv_eval does without
// groups: the thread owning the winner row), then the reductions pod j's Filters need over the snapshot after it:
// part[6 nb + b] = min over the block's valid nodes passing the pod's nodeSelector / required node affinity of the
// DoNotSchedule constraint's count (enc_min_i32; 0 = none: MaxInt32), part[7 nb + b] = Σ over valid nodes of pods
// matching the required pod-affinity group (only those carrying a zone label when every required term is zone-keyed:
// affinityCounts then has no hostname pairs); the zone sums (ZoneSums) with one atomic per block and nonzero word.
template <int F>  // RSV_F_* (as rsv_eval): the Reserve compiled for the profile's plugins only
__global__ __launch_bounds__(kRsvThreads) void group_pre(DevTable T, RsvNode* __restrict__ RN,
                                                         const DevPod* __restrict__ pods, int64_t end, int64_t n,
                                                         int g, RsvExt X, const uint64_t* __restrict__ val,
                                                         uint64_t* __restrict__ part, uint64_t* __restrict__ out_keys,
                                                         int32_t* __restrict__ out_slot,
                                                         unsigned long long* __restrict__ ws) {
  __shared__ uint64_t s_red[kRsvThreads / kWave];
  if (end < 0) end = (int64_t)ws[4];
  const int64_t j = (int64_t)ws[3] + g;
  if (j - 1 >= end || (g == 0 && j >= end)) return;  // uniform across the grid
  const int nb = gridDim.x;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g > 0) {
    const uint64_t k = rsv_partials_max(part + 2 * nb, nb);
    const int64_t w = k ? (int64_t)key_node(k) : -1;
    if (i == w || (w < 0 && i == 0)) {
      int32_t slot = -1;
      bool placed = false;
      if (w >= 0)
        placed = rsv_reserve<(F & RSV_F_NUMA) != 0, (F & RSV_F_DS) != 0, (F & RSV_F_XF) != 0>(T, RN, w, val[w],
                                                                                              pods[j - 1], X, j - 1,
                                                                                              slot);
      out_keys[j - 1] = placed ? k : 0;
      out_slot[j - 1] = slot;
      if (placed && X.nq > 0 && pods[j - 1].quota >= 0) {
        if (j >= end) rsv_quota_charge(X, pods[j - 1], j - 1);
        else ws[0] = (unsigned long long)j;
      }
    }
    if (j >= end) return;
  }
  const GroupPod gp = X.gpods[j];
  const ZoneSums Z = zone_sums(X, j);
  __shared__ int32_t s_zs[kZoneSumWords];  // the block's zone sums, flushed with one atomic each
  __shared__ unsigned long long s_pres;
  const bool zoned = gp.zone_keys != 0 || X.GP.ipa_zone;
  if (zoned) {
    for (int k = threadIdx.x; k < kZoneSumWords; k += kRsvThreads) s_zs[k] = 0;
    if (threadIdx.x == 0) s_pres = 0;
    __syncthreads();
  }
  uint64_t mn = 0;
  uint32_t sm = 0;
  if (i < n && (T.flags[i] & F_VALID)) {
    if (gp.nsp > 0) {
      const bool aff = node_affinity_match(X.pred, X.defp ? &X.defp[j] : nullptr, i);
      const int32_t zone = X.pred[i].zone;
      const bool ef = aff && spread_has_keys(gp, 0, zone), es = aff && spread_has_keys(gp, 1, zone);
      for (int c = 0; c < gp.nsp; ++c) {
        const bool hard = (gp.sp_flags[c] & KG_SPREAD_HARD) != 0, z = (gp.sp_flags[c] & KG_SPREAD_ZONE) != 0;
        if (!(hard ? ef : es)) continue;
        const int32_t v = X.G.cnt(gp.sp_g[c], i);
        if (z) {
          if (v) atomicAdd(&s_zs[((hard ? 0 : kSpread) + c) * kZones + zone - 1], v);
          if (hard) atomicOr(&s_pres, 1ull << (zone - 1));
        } else if (hard) {
          mn = enc_min_i32(v);
        }
      }
    }
    const int32_t zone = X.pred[i].zone;
    if (X.GP.ipa_filter && gp.req >= 0 && (gp.aff_terms || zone > 0)) sm = (uint32_t)X.G.cnt(gp.req, i);
    if (X.GP.ipa_zone && zone > 0) {
      int32_t c[kIpaZoneCh];
      ipa_zone_terms(X.G, i, gp, c);
#pragma unroll
      for (int h = 0; h < kIpaZoneCh; ++h)
        if (c[h]) atomicAdd(&s_zs[(2 * kSpread + h) * kZones + zone - 1], c[h]);
    }
  }
  mn = rsv_block_max(mn, s_red);
  __syncthreads();
  const uint64_t st = rsv_block_sum(sm, s_red);
  if (threadIdx.x == 0) {
    part[6 * nb + blockIdx.x] = mn;
    part[7 * nb + blockIdx.x] = st;
  }
  if (zoned) {
    __syncthreads();
    for (int k = threadIdx.x; k < kZoneSumWords; k += kRsvThreads) {
      const int32_t v = s_zs[k];
      if (v) atomicAdd(&Z.zf[k], v);  // zf, zs and zi are contiguous
    }
    if (threadIdx.x == 0 && s_pres) atomicOr((unsigned long long*)Z.pres, s_pres);
  }
}

// End of a group of kRsvGroup pods (one wave): Reserve of the group's last pod (cursor + g_last) with its quota
// charge, and the cursor advance.  Pods past `end` are skipped.
template <int F>  // RSV_F_* (as rsv_eval)
__global__ __launch_bounds__(kWave) void rsv_apply(DevTable T, RsvNode* __restrict__ RN,
                                                   const uint64_t* __restrict__ val, const DevPod* __restrict__ pods,
                                                   int64_t end, int nb, int g_last, RsvExt X,
                                                   const uint64_t* __restrict__ part,
                                                   uint64_t* __restrict__ out_keys, int32_t* __restrict__ out_slot,
                                                   unsigned long long* __restrict__ ws) {
  if (end < 0) end = (int64_t)ws[4];
  const int64_t base = (int64_t)ws[3];
  const int64_t j = base + g_last;
  if (base >= end) return;
  const uint64_t k = j < end ? rsv_partials_max(part + 2 * nb, nb) : 0;
  if (threadIdx.x != 0) return;
  if (j < end) {
    int32_t slot = -1;
    bool placed = false;
    if (k) {
      const int64_t w = (int64_t)key_node(k);
      placed = rsv_reserve<(F & RSV_F_NUMA) != 0, (F & RSV_F_DS) != 0, (F & RSV_F_XF) != 0>(T, RN, w, val[w], pods[j],
                                                                                            X, j, slot);
    }
    out_keys[j] = placed ? k : 0;
    out_slot[j] = slot;
    if (placed) rsv_quota_charge(X, pods[j], j);
  }
  ws[3] = (unsigned long long)(base + g_last + 1);
}

__global__ void scatter_rsv(RsvNode* __restrict__ RN, int32_t* __restrict__ rsv_n, uint64_t* __restrict__ pred,
                            const RsvNode* __restrict__ s, const int32_t* __restrict__ ns,
                            const uint64_t* __restrict__ sp, const int32_t* __restrict__ idx, int64_t n) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  RN[idx[k]] = s[k];
  rsv_n[idx[k]] = ns[k];
#pragma unroll
  for (int q = 0; q < kRsvSlots; ++q) pred[(size_t)idx[k] * kRsvSlots + q] = sp[(size_t)k * kRsvSlots + q];
}

}  // namespace kg
