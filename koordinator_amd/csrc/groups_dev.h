// (ABI 12) PodTopologySpread and InterPodAffinity with topologyKey kubernetes.io/hostname on the exact per-pod pass
// (SURVEY §8f-2).  The reference runs both from k8s.io/kubernetes v1.24.15 (not vendored), restated as published:
//   podtopologyspread/common.go, filtering.go  PreFilter counts, per topology pair, the pods matching a DoNotSchedule
//                                              constraint's selector in the pod's namespace over the nodes passing the
//                                              pod's nodeSelector / required node affinity; Filter: matchNum +
//                                              selfMatch − minMatchNum ≤ maxSkew (a node outside that set has no pair:
//                                              matchNum 0).
//   podtopologyspread/scoring.go               ScheduleAnyway: per node int64(cnt · log(size + 2) + maxSkew − 1), size
//                                              = the filtered nodes (hostname); NormalizeScore MaxNodeScore · (max +
//                                              min − s) / max, MaxNodeScore when max == 0 (also with no constraint).
//   interpodaffinity/filtering.go              required affinity (count of pods matching all terms > 0, or no pod in
//                                              the cluster matches them and the pod matches its own), required
//                                              anti-affinity, existing pods' required anti-affinity.
//   interpodaffinity/scoring.go                processExistingPod summed per node; NormalizeScore min–max in float64.
// With the hostname key every node is its own topology domain, so the per-pair maps become per-node counters over the
// caller's match groups (a label selector + namespaces, decided by the caller once per pod): an assume changes its
// winner's counters only.  The globals a pod's Filter needs (the minimum match count over the eligible nodes, the
// cluster-wide count of pods matching its required affinity) come from a reduction pass (group_pre) that runs after
// the previous pod's Reserve; the Score normalisations reuse the exact pass's second kernel.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/koordgpu.h"
#include "defaults_dev.h"
#include "kernels.h"

namespace kg {

constexpr int kGroups = KG_MAX_MATCH_GROUPS;
constexpr int kPodPref = KG_MAX_POD_PREFERRED;
constexpr int kSpread = KG_MAX_SPREAD;
constexpr int kZones = KG_MAX_ZONES;
constexpr int kGroupArrays = 5;
constexpr int kIpaZoneCh = 4;  // InterPodAffinity zone channels (ZoneSums::zi)

// per-node counters, structure of arrays [kGroupArrays][kGroups][cap] int32: pods matching group k, required
// anti-affinity terms of group k on the node, Σ symmetric weights of the node's pods' terms of group k; the last two
// again for the node's pods' zone-keyed terms
struct GroupTable {
  int32_t* __restrict__ g;
  int64_t cap;
  __device__ __forceinline__ int32_t& cnt(int k, int64_t i) const { return g[(size_t)k * cap + i]; }
  __device__ __forceinline__ int32_t& anti(int k, int64_t i) const { return g[(size_t)(kGroups + k) * cap + i]; }
  __device__ __forceinline__ int32_t& symw(int k, int64_t i) const { return g[(size_t)(2 * kGroups + k) * cap + i]; }
  __device__ __forceinline__ int32_t& anti_z(int k, int64_t i) const { return g[(size_t)(3 * kGroups + k) * cap + i]; }
  __device__ __forceinline__ int32_t& symw_z(int k, int64_t i) const { return g[(size_t)(4 * kGroups + k) * cap + i]; }
};

struct GroupPod {  // 112 B per staged pod
  uint32_t match, aff_terms, anti, anti_z;  // hostname-keyed required terms; anti_z: zone-keyed anti-affinity terms
  uint32_t aff_terms_z, pref_zone;          // zone-keyed required affinity terms; bit t: preferred term t zone-keyed
  int32_t req;              // conjunction group of the required pod-affinity terms (-1 none)
  int32_t npref;
  int32_t pref_g[kPodPref], pref_w[kPodPref];
  int32_t nsp;              // topology spread constraints, in the pod's order
  uint32_t zone_keys;       // bit 0: a DoNotSchedule constraint is zone-keyed, bit 1: a ScheduleAnyway one,
                            // bit 2 (kSpreadSysDefault): the constraints are the plugin's system defaults
  int32_t sp_g[kSpread], sp_skew[kSpread];
  uint32_t sp_flags[kSpread];  // KG_SPREAD_HARD | KG_SPREAD_ZONE
};
// the nodes a spread constraint set counts on: the pod's nodeSelector / required node affinity hold and the node
// carries every key of the set (kind 0: DoNotSchedule, 1: ScheduleAnyway)
__device__ __forceinline__ bool spread_has_keys(const GroupPod& gp, int kind, int32_t zone) {
  return !((gp.zone_keys >> kind) & 1u) || zone > 0;
}
// (ABI 13) requireAllTopologies = len(pod.Spec.TopologySpreadConstraints) > 0 || !systemDefaulted (podtopologyspread
// PreScore): a system-defaulted pod ignores no node; a filtered node without the zone label skips that constraint's
// Score term and adds the empty zone value to the constraint's topology size
constexpr uint32_t kSpreadSysDefault = 1u << 2;
__device__ __forceinline__ bool spread_sysdef(const GroupPod& gp) { return (gp.zone_keys & kSpreadSysDefault) != 0; }

struct GroupParams {
  int32_t spread_filter, spread_score, w_spread;
  int32_t ipa_filter, ipa_score, w_ipa;
  int32_t hard_w;
  int32_t ipa_zone;  // some pod carries zone-keyed InterPodAffinity terms: group_pre builds the zone channels
};

// NodeInfo.AddPod / RemovePod (sign ±1) of a pod's group contributions on node i (atomics: the delta pass applies
// several pods to one node at once; Reserve is one thread)
__device__ __forceinline__ void group_apply(const GroupTable& G, int64_t i, const GroupPod& gp, int sign, int hard_w) {
#pragma unroll
  for (int k = 0; k < kGroups; ++k) {
    if ((gp.match >> k) & 1u) atomicAdd(&G.cnt(k, i), sign);
    if ((gp.anti >> k) & 1u) atomicAdd(&G.anti(k, i), sign);
    if ((gp.anti_z >> k) & 1u) atomicAdd(&G.anti_z(k, i), sign);
    if (hard_w > 0 && ((gp.aff_terms >> k) & 1u)) atomicAdd(&G.symw(k, i), sign * hard_w);
    if (hard_w > 0 && ((gp.aff_terms_z >> k) & 1u)) atomicAdd(&G.symw_z(k, i), sign * hard_w);
  }
  for (int t = 0; t < gp.npref; ++t)
    atomicAdd((gp.pref_zone >> t) & 1u ? &G.symw_z(gp.pref_g[t], i) : &G.symw(gp.pref_g[t], i), sign * gp.pref_w[t]);
}

// PodMatchesNodeSelectorAndAffinityTerms: the pod's nodeSelector and required node affinity (the NodeAffinity Filter
// without its profile switch); no predicate table = no node selector / affinity on the pod
__device__ __forceinline__ bool node_affinity_match(const NodePred* pred, const DefPod* d, int64_t i) {
  if (!pred || !d) return true;
  const NodePred n = pred[i];
  if ((n.pred & d->sel) != d->sel) return false;
  if (d->nreq == 0) return true;
  bool any = false;
#pragma unroll
  for (int k = 0; k < kAffTerms; ++k) any |= k < d->nreq && term_holds(n.pred, d->req[k]);
  return any;
}

// Zone sums of one pod (group_pre, double-buffered by the pod's parity): per constraint c, zf[c][z] = Σ over the nodes
// passing the pod's node affinity with every DoNotSchedule key of the pods matching c's group in zone z, zs[c][z] the
// same over the ScheduleAnyway node set; pres = the zones holding such a DoNotSchedule node.  zi: InterPodAffinity's
// topologyToMatchedTermCount maps for the zone key, summed over the valid nodes carrying a zone label:
//   zi[0][z] pods matching the required affinity conjunction (affinityCounts),
//   zi[1][z] pods matching one of the pod's zone-keyed anti-affinity groups (antiAffinityCounts, > 0 test only),
//   zi[2][z] zone-keyed required anti-affinity terms of existing pods the pod matches (existingAntiAffinityCounts),
//   zi[3][z] topologyScore: the pod's zone-keyed preferred terms × matching pods + existing pods' zone-keyed terms
//            the pod matches
constexpr int kZoneSumWords = (2 * kSpread + kIpaZoneCh) * kZones;
struct ZoneSums {
  int32_t* __restrict__ zf;  // [kSpread][kZones]
  int32_t* __restrict__ zs;  // [kSpread][kZones]
  int32_t* __restrict__ zi;  // [kIpaZoneCh][kZones]
  uint64_t* __restrict__ pres;
};

// node i's contribution to the zone channels (group_pre; the node is valid and carries a zone label)
__device__ __forceinline__ void ipa_zone_terms(const GroupTable& G, int64_t i, const GroupPod& gp, int32_t c[kIpaZoneCh]) {
  c[0] = gp.req >= 0 && gp.aff_terms_z ? G.cnt(gp.req, i) : 0;
  c[1] = c[2] = c[3] = 0;
  for (int t = 0; t < gp.npref; ++t)
    if ((gp.pref_zone >> t) & 1u) c[3] += gp.pref_w[t] * G.cnt(gp.pref_g[t], i);
  uint32_t a = gp.anti_z;
  while (a) {
    const int k = __builtin_ctz(a);
    a &= a - 1;
    c[1] += G.cnt(k, i);
  }
  uint32_t m = gp.match;
  while (m) {
    const int k = __builtin_ctz(m);
    m &= m - 1;
    c[2] += G.anti_z(k, i);
    c[3] += G.symw_z(k, i);
  }
}

// Filters of both plugins on node i (true = feasible).  min_match[c]: TpKeyToCriticalPaths' minimum per DoNotSchedule
// constraint (hostname: over the eligible nodes' counts; zone: over the present zones' sums); total: the cluster-wide
// count of pods matching the required pod-affinity group
__device__ __forceinline__ bool groups_filter(const GroupTable& G, int64_t i, const GroupPod& gp, const GroupParams& GP,
                                              bool nodeaff, int32_t zone, const int64_t* min_match, const ZoneSums& Z,
                                              uint64_t pres, int64_t total) {
  if (GP.spread_filter) {
    const bool elig = nodeaff && spread_has_keys(gp, 0, zone);
    for (int c = 0; c < gp.nsp; ++c) {
      if (!(gp.sp_flags[c] & KG_SPREAD_HARD)) continue;
      int64_t match;
      if (gp.sp_flags[c] & KG_SPREAD_ZONE) {
        if (zone <= 0) return false;  // the node lacks the constraint's key
        match = ((pres >> (zone - 1)) & 1ull) ? Z.zf[c * kZones + zone - 1] : 0;
      } else {
        match = elig ? G.cnt(gp.sp_g[c], i) : 0;
      }
      const int64_t self = (gp.match >> gp.sp_g[c]) & 1u;
      if (match + self - min_match[c] > gp.sp_skew[c]) return false;
    }
  }
  if (GP.ipa_filter) {
    if (gp.req >= 0) {  // satisfyPodAffinity: every term's key on the node, then its pair's count
      if (gp.aff_terms_z && zone <= 0) return false;
      const bool exist = (!gp.aff_terms || G.cnt(gp.req, i) > 0) && (!gp.aff_terms_z || Z.zi[zone - 1] > 0);
      if (!exist && !(total == 0 && ((gp.match >> gp.req) & 1u))) return false;
    }
    for (int k = 0; k < kGroups; ++k) {
      if (((gp.anti >> k) & 1u) && G.cnt(k, i) > 0) return false;
      if (((gp.match >> k) & 1u) && G.anti(k, i) > 0) return false;
    }
    if (GP.ipa_zone && zone > 0 && (Z.zi[kZones + zone - 1] > 0 || Z.zi[2 * kZones + zone - 1] > 0)) return false;
  }
  return true;
}

// InterPodAffinity raw Score on node i: the pod's preferred terms against the node's matching pods, plus the node's
// pods' terms the pod matches
__device__ __forceinline__ int32_t interpod_raw(const GroupTable& G, int64_t i, const GroupPod& gp, int32_t zone,
                                              const ZoneSums& Z) {
  int32_t s = zone > 0 ? Z.zi[3 * kZones + zone - 1] : 0;  // the zone key's topologyScore
  for (int t = 0; t < gp.npref; ++t)
    if (!((gp.pref_zone >> t) & 1u)) s += gp.pref_w[t] * G.cnt(gp.pref_g[t], i);
  uint32_t m = gp.match;
  while (m) {
    const int k = __builtin_ctz(m);
    m &= m - 1;
    s += G.symw(k, i);
  }
  return s;
}

// PodTopologySpread raw Score of node i (not ignored): Σ over the ScheduleAnyway constraints in the pod's order of
// float64(cnt)·w + float64(maxSkew − 1), from 0, then int64(); hostname: the node's count, weight log(F − ignored + 2);
// zone: its zone's sum, weight log(#zones + 2) — both from the host's table of Go's math.Log (r5); the products and
// sums round separately (-ffp-contract=off)
__device__ __forceinline__ int64_t spread_raw(const GroupTable& G, int64_t i, const GroupPod& gp, int32_t zone,
                                              const int32_t* __restrict__ zs, double w_host, double w_zone) {
  double s = 0;
  for (int c = 0; c < gp.nsp; ++c) {
    if (gp.sp_flags[c] & KG_SPREAD_HARD) continue;
    const bool z = (gp.sp_flags[c] & KG_SPREAD_ZONE) != 0;
    if (z && zone <= 0) continue;  // Score: no label, no term (reached only by a system-defaulted pod, ABI 13)
    const int64_t cnt = z ? zs[c * kZones + zone - 1] : G.cnt(gp.sp_g[c], i);
    s += (double)cnt * (z ? w_zone : w_host) + (double)(gp.sp_skew[c] - 1);
  }
  return (int64_t)s;
}

__device__ __forceinline__ int64_t spread_normalize(int64_t raw, int64_t mn, int64_t mx) {
  return mx == 0 ? 100 : 100 * (mx + mn - raw) / mx;
}

__device__ __forceinline__ int64_t interpod_normalize(int64_t raw, int64_t mn, int64_t mx) {
  const int64_t d = mx - mn;
  return d <= 0 ? 0 : (int64_t)(100.0 * ((double)(raw - mn) / (double)d));
}

// order-preserving encodings for max-reductions of signed / min values
__device__ __forceinline__ uint64_t enc_max_i32(int32_t v) { return (uint64_t)((int64_t)v + 0x80000000ll) + 1; }
__device__ __forceinline__ int32_t dec_max_i32(uint64_t e) { return (int32_t)((int64_t)(e - 1) - 0x80000000ll); }
__device__ __forceinline__ uint64_t enc_min_i32(int32_t v) { return 0x100000000ull - (uint64_t)((int64_t)v + 0x80000000ll); }
__device__ __forceinline__ int32_t dec_min_i32(uint64_t e) { return (int32_t)((int64_t)(0x100000000ull - e) - 0x80000000ll); }

__global__ void group_deltas(GroupTable G, const GroupPod* __restrict__ gp, const int32_t* __restrict__ node,
                             const int32_t* __restrict__ sign, int64_t n, int hard_w) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  group_apply(G, node[k], gp[k], sign[k], hard_w);
}

}  // namespace kg
