// Reservation plugin on the device (SURVEY §8a A15–A18): per-node reservation slots in HBM and the per-pod
// pass that restores NodeInfo for matched / unmatched reservations (BeforePreFilter, transformer.go:49-346), runs
// NodeResourcesFit + LoadAware on the restored row, the Reservation Filter (plugin.go:357-428), the nomination
// (nominator.go:76-134) and Score (scoring.go:103-203) with the PreScore preferred node, DefaultNormalizeScore,
// then Reserve (plugin.go:521-559).
//
// One pod per pass, three kernels (HBM-bound wide pass, normalise + argmax pass, one-lane Reserve), captured in a
// hipGraph per group of pods; the pod index is read from a device cursor that the Reserve kernel advances.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/koordgpu.h"
#include "kernels.h"

namespace kg {

constexpr int kRsvSlots = KG_MAX_RSV_SLOTS;
constexpr uint32_t RS_AVAIL = 1u << 0, RS_ONCE = 1u << 1, RS_UNSCHED = 1u << 2;  // policy in bits 4..5
constexpr uint32_t RP_AFFINITY = 1u << 0;

struct RsvNode {  // 192 B: one node's slots, read only for nodes with slots (rsv_n[i] > 0)
  int64_t alloc_cpu[kRsvSlots], alloc_mem[kRsvSlots];
  int64_t allocd_cpu[kRsvSlots], allocd_mem[kRsvSlots];
  int32_t owner[kRsvSlots], assigned[kRsvSlots], order[kRsvSlots];
  uint32_t meta[kRsvSlots];
};
static_assert(sizeof(RsvNode) == 192, "RsvNode layout");

struct RsvPod {
  int32_t owner;
  uint32_t flags;
};

struct RsvParams {
  int32_t filter, score, weight, pad;
};

// ws words: [0] ~min(order << 32 | node) over feasible nodes with an order label (0 = none), [1] max raw Score,
// [2] max selection key, [3] pod cursor
struct RsvOut {
  bool feas;
  int64_t base;   // Fit + LoadAware weighted total
  int32_t raw;    // Reservation Score of the nominated slot (0 = none)
  int32_t nom;    // nominated slot, -1 = none
  int32_t order;  // findMostPreferredReservationByOrder over matched (INT32_MAX = none)
};

__device__ __forceinline__ int64_t rsv_nn(int64_t a, int64_t b) { return a - b > 0 ? a - b : 0; }

// scoreReservation (scoring.go:183-203): MostAllocated over the reservation's non-zero allocatable.
__device__ __forceinline__ int32_t rsv_score_slot(const RsvNode& rn, int s, const DevPod& p) {
  const int64_t rc = p.req_cpu + rn.allocd_cpu[s], rm = p.req_mem + rn.allocd_mem[s];
  int64_t w = 0, sc = 0;
  if (rn.alloc_cpu[s] != 0) {
    ++w;
    if (rc <= rn.alloc_cpu[s]) sc += 100 * rc / rn.alloc_cpu[s];
  }
  if (rn.alloc_mem[s] != 0) {
    ++w;
    if (rm <= rn.alloc_mem[s]) sc += 100 * rm / rn.alloc_mem[s];
  }
  return w ? (int32_t)(sc / w) : 0;
}

__device__ __forceinline__ RsvOut rsv_eval_node(const DevTable& T, const RsvNode* __restrict__ RN,
                                                const int32_t* __restrict__ rsv_n, int64_t i, const DevPod& p,
                                                const RsvPod& rp, const EvalParams& P, const RsvParams& RP) {
  Row r = load_row(T, i);
  const int ns = rsv_n[i];
  RsvOut o{false, 0, 0, -1, 0x7fffffff};
  uint32_t mm = 0;  // matched slots
  int nm = 0;
  int64_t pr_c = 0, pr_m = 0, ra_c = 0, ra_m = 0;
  bool has_state = false;
  RsvNode rn;
  if (ns > 0) {
    rn = RN[i];
    uint32_t um = 0;
    for (int s = 0; s < ns; ++s) {
      const uint32_t m = rn.meta[s];
      if (!(m & RS_AVAIL) || ((m & RS_ONCE) && rn.assigned[s] > 0)) continue;  // transformer.go:101-110
      if (rp.owner != 0 && rn.owner[s] == rp.owner && !(m & RS_UNSCHED)) mm |= 1u << s;
      else if (rn.assigned[s] > 0) um |= 1u << s;
    }
    has_state = (mm | um) != 0 && !((rp.flags & RP_AFFINITY) && mm == 0);  // transformer.go:127-136
    if (has_state) {
      for (int s = 0; s < ns; ++s)
        if (um >> s & 1) {  // restoreUnmatchedReservations (transformer.go:265-291)
          r.req_cpu -= rn.alloc_cpu[s];
          r.req_mem -= rn.alloc_mem[s];
          r.nz_cpu -= rn.alloc_cpu[s];
          r.nz_mem -= rn.alloc_mem[s];
          const int64_t rc = rsv_nn(rn.alloc_cpu[s], rn.allocd_cpu[s]), rm = rsv_nn(rn.alloc_mem[s], rn.allocd_mem[s]);
          if (rc != 0 || rm != 0) {
            r.req_cpu += rc;
            r.req_mem += rm;
            r.nz_cpu += rc;
            r.nz_mem += rm;
          }
        }
      pr_c = r.req_cpu;
      pr_m = r.req_mem;
      for (int s = 0; s < ns; ++s)
        if (mm >> s & 1) {  // restoreMatchedReservation: NodeInfo.RemovePod(reserve pod) (transformer.go:240-263)
          r.req_cpu -= rn.alloc_cpu[s];
          r.req_mem -= rn.alloc_mem[s];
          r.nz_cpu -= rn.alloc_cpu[s];
          r.nz_mem -= rn.alloc_mem[s];
          r.num_pods -= 1;
          ra_c += rn.allocd_cpu[s];
          ra_m += rn.allocd_mem[s];
          ++nm;
        }
    }
  }
  int64_t t = 0;
  if (!eval_node(r, p, P, t)) return o;  // NodeResourcesFit + LoadAware on the restored NodeInfo
  // satisfied(s): filterWithReservations([s]) (plugin.go:384-428) with fitsNode (:433-482), preemptible = 0
  const bool zero = p.req_cpu == 0 && p.req_mem == 0;
  uint32_t sat = 0;
  if (has_state && !zero) {
    const bool pods_ok = !(r.num_pods - nm + 1 > r.alloc_pods);
    for (int s = 0; s < ns; ++s) {
      if (!(mm >> s & 1)) continue;
      const int64_t rc = rsv_nn(rn.alloc_cpu[s], rn.allocd_cpu[s]), rm = rsv_nn(rn.alloc_mem[s], rn.allocd_mem[s]);
      bool fits = pods_ok && !(p.req_cpu > r.alloc_cpu - (pr_c - rc - ra_c)) &&
                  !(p.req_mem > r.alloc_mem - (pr_m - rm - ra_m));
      if (((rn.meta[s] >> 4) & 3) == KG_RSV_POLICY_RESTRICTED) fits = fits && p.req_cpu <= rc && p.req_mem <= rm;
      if (fits) sat |= 1u << s;
    }
  }
  if (RP.filter && (rp.flags & RP_AFFINITY) && sat == 0) return o;  // plugin.go:361-364, 423-426
  o.feas = true;
  o.base = t;
  if (has_state) {
    // PreScore node order over matched (scoring.go:66, 162-181); nomination over FilterReservation-passing slots
    int32_t best_all = 0x7fffffff, best_sat = 0x7fffffff;
    int pick = -1;
    for (int s = 0; s < ns; ++s) {
      if (!(mm >> s & 1)) continue;
      const int32_t od = rn.order[s];
      if (od != 0 && best_all > od) best_all = od;
      if ((sat >> s & 1) && od != 0 && best_sat > od) {
        best_sat = od;
        pick = s;
      }
    }
    o.order = best_all;
    if (pick < 0) {
      int32_t best = -1;
      for (int s = 0; s < ns; ++s)
        if (sat >> s & 1) {
          const int32_t sc = rsv_score_slot(rn, s, p);
          if (sc > best) {  // prioritizeReservations + sort (unstable; pinned: lowest slot on ties)
            best = sc;
            pick = s;
          }
        }
    }
    o.nom = pick;
    o.raw = pick >= 0 ? rsv_score_slot(rn, pick, p) : 0;
  }
  return o;
}

// Pass 1: per-node Filter + Fit/LoadAware total + nominated slot and raw Score; wave-reduced preferred-node key and
// max raw Score into ws[0], ws[1].  val[i] = (base << 32) | raw << 8 | feasible << 7 | (nom + 1), 0 = filtered.
__global__ __launch_bounds__(256) void rsv_eval(DevTable T, const RsvNode* __restrict__ RN,
                                                const int32_t* __restrict__ rsv_n, const DevPod* __restrict__ pods,
                                                const RsvPod* __restrict__ rpods, int64_t end, int64_t n,
                                                EvalParams P, RsvParams RP, uint64_t* __restrict__ val,
                                                unsigned long long* __restrict__ ws) {
  const int64_t j = (int64_t)ws[3];
  if (j >= end) return;  // uniform across the grid
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t pk = 0;
  uint32_t rawv = 0;
  if (i < n) {
    const DevPod p = pods[j];
    const RsvPod rp = rpods[j];
    const RsvOut o = rsv_eval_node(T, RN, rsv_n, i, p, rp, P, RP);
    uint64_t v = 0;
    if (o.feas) {
      v = ((uint64_t)(uint32_t)o.base << 32) | ((uint64_t)(uint32_t)o.raw << 8) | (1ull << 7) | (uint64_t)(o.nom + 1);
      if (o.order != 0x7fffffff) pk = ~(((uint64_t)(uint32_t)o.order << 32) | (uint64_t)(uint32_t)i);
      rawv = (uint32_t)o.raw;
    }
    val[i] = v;
  }
  pk = wave_max_u64_dpp(pk);
  rawv = wave_max_u32(rawv);
  if ((threadIdx.x & (kWave - 1)) == 0) {
    if (pk) atomicMax(&ws[0], (unsigned long long)pk);
    if (rawv) atomicMax(&ws[1], (unsigned long long)rawv);
  }
}

// Pass 2: PreScore preferred node (1000), DefaultNormalizeScore over the feasible nodes, × weight, packed argmax.
__global__ __launch_bounds__(256) void rsv_select(const uint64_t* __restrict__ val, int64_t end, int64_t n,
                                                  RsvParams RP, unsigned long long* __restrict__ ws) {
  if ((int64_t)ws[3] >= end) return;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t pk = ws[0];
  const int64_t pref = pk ? (int64_t)(uint32_t)(~pk) : -1;
  const int64_t mx = pk ? (ws[1] > 1000 ? (int64_t)ws[1] : 1000) : (int64_t)ws[1];
  uint64_t key = 0;
  if (i < n) {
    const uint64_t v = val[i];
    if (v & (1ull << 7)) {
      const int64_t raw = (i == pref) ? 1000 : (int64_t)((v >> 8) & 0xff);  // mostPreferredScore
      int64_t t = (int64_t)(v >> 32);
      if (RP.score && mx > 0) t += (int64_t)RP.weight * (100 * raw / mx);
      key = make_key(t, (uint32_t)i);
    }
  }
  key = wave_max_key(key);
  if ((threadIdx.x & (kWave - 1)) == 0 && key) atomicMax(&ws[2], (unsigned long long)key);
}

// Pass 3 (one lane): Reserve — assume on the winner row (NodeInfo + LoadAware assign cache) and
// reservationCache.assumePod on its nominated slot (reservation_info.go:317-326); advance the cursor.
__global__ void rsv_apply(DevTable T, RsvNode* __restrict__ RN, const uint64_t* __restrict__ val,
                          const DevPod* __restrict__ pods, int64_t end, uint64_t* __restrict__ out_keys,
                          int32_t* __restrict__ out_slot, unsigned long long* __restrict__ ws) {
  const int64_t j = (int64_t)ws[3];
  if (j >= end) return;
  const uint64_t k = ws[2];
  int32_t slot = -1;
  if (k) {
    const int64_t w = (int64_t)key_node(k);
    const DevPod p = pods[j];
    Row r = load_row(T, w);
    const int64_t prod = (p.flags & P_PROD) ? 1 : 0;
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
    slot = (int32_t)(val[w] & 7) - 1;
    if (slot >= 0) {
      RN[w].allocd_cpu[slot] += p.req_cpu;
      RN[w].allocd_mem[slot] += p.req_mem;
      RN[w].assigned[slot] += 1;
    }
  }
  out_keys[j] = k;
  out_slot[j] = slot;
  ws[0] = 0;
  ws[1] = 0;
  ws[2] = 0;
  ws[3] = (unsigned long long)(j + 1);
}

__global__ void scatter_rsv(RsvNode* __restrict__ RN, int32_t* __restrict__ rsv_n, const RsvNode* __restrict__ s,
                            const int32_t* __restrict__ ns, const int32_t* __restrict__ idx, int64_t n) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  RN[idx[k]] = s[k];
  rsv_n[idx[k]] = ns[k];
}

}  // namespace kg
