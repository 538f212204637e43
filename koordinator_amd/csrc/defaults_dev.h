// Upstream default plugins of a stock koord-scheduler profile on the exact per-pod pass:
// TaintToleration, NodeAffinity and NodeResourcesBalancedAllocation.  The reference runs them from
// k8s.io/kubernetes v1.24.15 (go.mod:57, replace go.mod:275; not vendored in the reference tree), restated here as
// published and pinned as DESIGN.md §3.13 says:
//   tainttoleration/taint_toleration.go   Filter: FindMatchingUntoleratedTaint over NoSchedule / NoExecute taints;
//                                         Score: countIntolerableTaintsPreferNoSchedule, NormalizeScore
//                                         = DefaultNormalizeScore(MaxNodeScore, reverse = true)
//   nodeaffinity/node_affinity.go         Filter: RequiredNodeAffinity.Match (nodeSelector AND any required term);
//                                         Score: Σ weights of matching preferred terms,
//                                         NormalizeScore = DefaultNormalizeScore(MaxNodeScore, reverse = false)
//   imagelocality/image_locality.go       Score: calculatePriority(sumImageScores(node, pod.Spec.Containers), #containers)
//                                         with minThreshold 23 MiB, maxThreshold 1000 MiB × #containers; no NormalizeScore.
//                                         scaledImageScore is node-independent: the caller passes it per container.
//   noderesources/balanced_allocation.go  Score (useRequested = true): fraction_r = float64(Requested_r + podRequest_r)
//   + resource_allocation.go              / float64(Allocatable_r) capped at 1 over the configured resources with a
//                                         non-zero Allocatable; std = |f_cpu − f_mem| / 2 for two of them, 0 for
//                                         fewer; score = int64((1 − std) · 100).  No NormalizeScore.
// Label / taint matching is string work the caller does once per node update (kg_node_predicates): the device sees
// bitmasks over the caller's predicate and taint tables, and combines them per pod.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/koordgpu.h"

namespace kg {

constexpr int kAffTerms = KG_MAX_AFF_TERMS;

struct NodePred {  // 40 B per node (the masks of kg_node_predicates; its ABI 11 table sizes stay on the host)
  uint64_t pred, hard, soft, images;
  int32_t zone;     // (ABI 12) 1 + topology.kubernetes.io/zone index, 0 = no zone label
  int32_t pad;
};

constexpr int kContainers = KG_MAX_CONTAINERS;
struct DefPod {  // 184 B per staged pod; the pass broadcasts one
  uint64_t tol, sel;
  uint64_t req[kAffTerms], pref[kAffTerms];
  int32_t w[kAffTerms];
  int32_t nreq, npref;
  // ImageLocality: the distinct image bits of the pod's containers with Σ scaledImageScore over the containers using
  // each (a container's image counts once per container, sumImageScores), and len(pod.Spec.Containers)
  int64_t img_w[kContainers];
  uint8_t img_bit[kContainers];
  int32_t nimg, ncont;
};

struct DefParams {
  int32_t taint_filter, taint_score, w_taint;
  int32_t aff_filter, aff_score, w_aff;
  int32_t bal, w_bal, bal_cpu, bal_mem;
  int32_t img, w_img;
};

// nodeSelectorTerm.match: every requirement of the term holds; a term without requirements matches no node
__device__ __forceinline__ bool term_holds(uint64_t pred, uint64_t term) { return term != 0 && (pred & term) == term; }

// Filter of both plugins on one node (true = feasible)
__device__ __forceinline__ bool defaults_filter(const NodePred& n, const DefPod& d, const DefParams& F) {
  if (F.taint_filter && (n.hard & ~d.tol) != 0) return false;  // an untolerated NoSchedule / NoExecute taint
  if (F.aff_filter) {
    if ((n.pred & d.sel) != d.sel) return false;  // pod.Spec.NodeSelector
    if (d.nreq > 0) {                             // RequiredDuringSchedulingIgnoredDuringExecution: any term
      bool any = false;
#pragma unroll
      for (int k = 0; k < kAffTerms; ++k) any |= k < d.nreq && term_holds(n.pred, d.req[k]);
      if (!any) return false;
    }
  }
  return true;
}

// TaintToleration raw Score: PreferNoSchedule taints the pod does not tolerate
__device__ __forceinline__ int32_t taint_raw(const NodePred& n, const DefPod& d) {
  return __popcll(n.soft & ~d.tol);
}

// NodeAffinity raw Score: Σ weights of the matching preferred terms (weight 0 terms are skipped upstream)
__device__ __forceinline__ int32_t affinity_raw(const NodePred& n, const DefPod& d) {
  int32_t s = 0;
#pragma unroll
  for (int k = 0; k < kAffTerms; ++k)
    if (k < d.npref && term_holds(n.pred, d.pref[k])) s += d.w[k];
  return s;
}

// NodeResourcesBalancedAllocation Score on the (restored) NodeInfo: Requested (not NonZeroRequested) + the pod's
// plain requests.  Float64 with correctly rounded division (no contraction is possible in these expressions).
__device__ __forceinline__ int64_t balanced_score(int64_t alloc_cpu, int64_t alloc_mem, int64_t req_cpu,
                                                  int64_t req_mem, int64_t pod_cpu, int64_t pod_mem,
                                                  const DefParams& F) {
  double f[2];
  int n = 0;
  if (F.bal_cpu && alloc_cpu != 0) {
    double x = (double)(req_cpu + pod_cpu) / (double)alloc_cpu;
    f[n++] = x > 1.0 ? 1.0 : x;
  }
  if (F.bal_mem && alloc_mem != 0) {
    double x = (double)(req_mem + pod_mem) / (double)alloc_mem;
    f[n++] = x > 1.0 ? 1.0 : x;
  }
  const double std = n == 2 ? fabs((f[0] - f[1]) / 2.0) : 0.0;
  return (int64_t)((1.0 - std) * 100.0);
}

// ImageLocality Score: calculatePriority(sumImageScores, numContainers) — Σ over the pod's containers whose image the
// node holds of scaledImageScore, clamped to [minThreshold, maxThreshold], MaxNodeScore · (sum − min) / (max − min)
// in int64 (Go truncation; both operands non-negative except with 0 containers, where the numerator is 0)
constexpr int64_t kImgMB = 1024 * 1024, kImgMin = 23 * kImgMB, kImgMaxPerContainer = 1000 * kImgMB;
__device__ __forceinline__ int64_t image_score(const NodePred& n, const DefPod& d) {
  int64_t sum = 0;
#pragma unroll
  for (int k = 0; k < kContainers; ++k)
    if (k < d.nimg && ((n.images >> d.img_bit[k]) & 1ull)) sum += d.img_w[k];
  const int64_t mx = kImgMaxPerContainer * d.ncont;
  sum = sum < kImgMin ? kImgMin : (sum > mx ? mx : sum);
  const int64_t num = 100 * (sum - kImgMin), den = mx - kImgMin;
  return num == 0 ? 0 : num / den;
}

// DefaultNormalizeScore (helper/normalize_score.go) of one node's raw score against the feasible nodes' maximum
__device__ __forceinline__ int64_t normalize_default(int64_t raw, int64_t mx, bool reverse) {
  if (mx == 0) return reverse ? 100 : raw;
  const int64_t s = div_small(100 * raw, mx);
  return reverse ? 100 - s : s;
}

}  // namespace kg
