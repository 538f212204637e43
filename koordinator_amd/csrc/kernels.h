// kernels.h — device data layout and per-(pod,node) evaluation shared by every kernel of the engine.
//
// Node state lives in HBM as structure-of-arrays (one column per field, int64 like the reference's
// framework.Resource fields), replicated on every rank.  A pod is pre-decoded on the host into DevPod
// (requests, non-zero requests, LoadAware estimate, flags).  eval_node() is the fused body of
//   upstream NodeResourcesFit.Filter (fitsRequest)       — restated in-tree: reservation/plugin.go:433-482
//   LoadAwareScheduling.Filter                            — load_aware.go:123-171 (threshold bit precomputed)
//   upstream NodeResourcesFit.Score (LeastAllocated, NonZeroRequested) — nodenumaresource/scoring.go:191-230
//   LoadAwareScheduling.Score                             — load_aware.go:269-335, scorer :378-397
//   weighted sum over plugins                             — upstream RunScorePlugins (framework_extender.go:236-258)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kg {

constexpr int kWave = 64;

// node flags (device)
constexpr uint32_t F_VALID = 1u << 0;
constexpr uint32_t F_LA_SCORE = 1u << 1;      // NodeMetric present and not expired: LoadAware scores it
constexpr uint32_t F_LA_PASS = 1u << 2;       // LoadAware Filter verdict for a non-prod pod
constexpr uint32_t F_LA_PASS_PROD = 1u << 3;  // LoadAware Filter verdict for a prod pod

// pod flags (device)
constexpr uint32_t P_ZERO_REQ = 1u << 0;      // every request zero → fitsRequest skips resource checks
constexpr uint32_t P_DAEMONSET = 1u << 1;     // LoadAware Filter bypass (load_aware.go:129-131)
constexpr uint32_t P_PROD = 1u << 2;          // priority class koord-prod
constexpr uint32_t P_LA_PROD_SCORE = 1u << 3; // prod && ScoreAccordingProdUsage (load_aware.go:291)

struct DevTable {
  int64_t *alloc_cpu, *alloc_mem;        // NodeInfo.Allocatable
  int64_t *req_cpu, *req_mem;            // NodeInfo.Requested             (mutable)
  int64_t *nz_cpu, *nz_mem;              // NodeInfo.NonZeroRequested      (mutable)
  int64_t *la_alloc_cpu, *la_alloc_mem;  // EstimateNode allocatable
  int64_t *la_used_cpu, *la_used_mem;    // Σ EstimatePod(assigned) + NodeUsage   (mutable)
  int64_t *la_pused_cpu, *la_pused_mem;  // Σ EstimatePod(assigned prod pods)      (mutable)
  int32_t *alloc_pods, *num_pods;        // AllowedPodNumber, len(Pods)    (num_pods mutable)
  uint32_t *flags;
};

struct DevPod {
  int64_t req_cpu, req_mem;
  int64_t nz_cpu, nz_mem;
  int64_t est_cpu, est_mem;
  uint32_t flags;
  uint32_t pad;
};
static_assert(sizeof(DevPod) == 56, "DevPod layout");

struct EvalParams {
  int64_t fit_w_cpu, fit_w_mem;
  int64_t la_w_cpu, la_w_mem, la_wsum;
  int64_t weight_fit, weight_la;
  int32_t fit_filter, fit_score, la_filter, la_score;
  int32_t score_bits;  // bit width of the largest possible weighted total
  int32_t pad;
};

struct Row {
  int64_t alloc_cpu, alloc_mem, req_cpu, req_mem, nz_cpu, nz_mem;
  int64_t la_alloc_cpu, la_alloc_mem, la_used_cpu, la_used_mem, la_pused_cpu, la_pused_mem;
  int32_t alloc_pods, num_pods;
  uint32_t flags;
};

__device__ __forceinline__ Row load_row(const DevTable& T, int64_t i) {
  Row r;
  r.alloc_cpu = T.alloc_cpu[i];
  r.alloc_mem = T.alloc_mem[i];
  r.req_cpu = T.req_cpu[i];
  r.req_mem = T.req_mem[i];
  r.nz_cpu = T.nz_cpu[i];
  r.nz_mem = T.nz_mem[i];
  r.la_alloc_cpu = T.la_alloc_cpu[i];
  r.la_alloc_mem = T.la_alloc_mem[i];
  r.la_used_cpu = T.la_used_cpu[i];
  r.la_used_mem = T.la_used_mem[i];
  r.la_pused_cpu = T.la_pused_cpu[i];
  r.la_pused_mem = T.la_pused_mem[i];
  r.alloc_pods = T.alloc_pods[i];
  r.num_pods = T.num_pods[i];
  r.flags = T.flags[i];
  return r;
}

__device__ __forceinline__ void store_mutable(const DevTable& T, int64_t i, const Row& r) {
  T.req_cpu[i] = r.req_cpu;
  T.req_mem[i] = r.req_mem;
  T.nz_cpu[i] = r.nz_cpu;
  T.nz_mem[i] = r.nz_mem;
  T.la_used_cpu[i] = r.la_used_cpu;
  T.la_used_mem[i] = r.la_used_mem;
  T.la_pused_cpu[i] = r.la_pused_cpu;
  T.la_pused_mem[i] = r.la_pused_mem;
  T.num_pods[i] = r.num_pods;
}

// assume(pod) on a row: upstream NodeInfo.AddPod + LoadAware Reserve → podAssignCache.assign
// (load_aware.go:260-263; the estimate is EstimatePod, counted because PodsMetric has no entry for it).
__device__ __forceinline__ void apply_pod(Row& r, const DevPod& p) {
  r.req_cpu += p.req_cpu;
  r.req_mem += p.req_mem;
  r.nz_cpu += p.nz_cpu;
  r.nz_mem += p.nz_mem;
  r.num_pods += 1;
  r.la_used_cpu += p.est_cpu;
  r.la_used_mem += p.est_mem;
  if (p.flags & P_PROD) {
    r.la_pused_cpu += p.est_cpu;
    r.la_pused_mem += p.est_mem;
  }
}

// leastRequestedScore (load_aware.go:388-397; nodenumaresource/least_allocated.go:49-58):
//   capacity == 0 → 0; requested > capacity → 0; else ((capacity - requested) * 100) / capacity.
// The quotient lies in [0,100] whenever 0 <= requested <= capacity, so a float estimate is off by at most one
// and one exact int64 multiply-compare fixes it: no 64-bit integer division on the hot path.
__device__ __forceinline__ int64_t least_requested(int64_t requested, int64_t capacity) {
  if (capacity == 0 || requested > capacity) return 0;
  const int64_t x = capacity - requested;
  const int64_t num = x * 100;
  if (requested < 0) return num / capacity;  // outside the [0,100] range: exact slow path
  int q = (int)(((float)x * 100.0f) / (float)capacity);
  q = q < 0 ? 0 : (q > 100 ? 100 : q);
  const int64_t t = (int64_t)q * capacity;
  if (t > num) q -= 1;
  else if (t + capacity <= num) q += 1;
  return q;
}

// s / w for the per-plugin weight sums: 32-bit unsigned division whenever both fit (always, for validated
// weights ≤ 1e6), exact int64 truncating division otherwise (Go semantics).
__device__ __forceinline__ int64_t div_small(int64_t s, int64_t w) {
  if ((uint64_t)s < (1ull << 32) && (uint64_t)w < (1ull << 32)) return (int64_t)((uint32_t)s / (uint32_t)w);
  return s / w;
}

// Fused Filter + Score of one node for one pod. Returns false when any enabled Filter rejects the node;
// otherwise writes the weighted total Σ_p weight_p · score_p.
__device__ __forceinline__ bool eval_node(const Row& n, const DevPod& p, const EvalParams& P, int64_t& total,
                                          uint32_t* reject = nullptr, int64_t* fit_out = nullptr,
                                          int64_t* la_out = nullptr) {
  uint32_t rej = 0;
  if (!(n.flags & F_VALID)) rej |= 1u << 4;
  if (P.fit_filter) {
    if (n.num_pods + 1 > n.alloc_pods) rej |= 1u << 0;
    if (!(p.flags & P_ZERO_REQ)) {
      if (p.req_cpu > n.alloc_cpu - n.req_cpu) rej |= 1u << 1;
      if (p.req_mem > n.alloc_mem - n.req_mem) rej |= 1u << 2;
    }
  }
  if (P.la_filter && !(p.flags & P_DAEMONSET)) {
    const uint32_t pass = (p.flags & P_PROD) ? F_LA_PASS_PROD : F_LA_PASS;
    if (!(n.flags & pass)) rej |= 1u << 3;
  }
  if (reject) *reject = rej;
  if (rej && !fit_out && !la_out) return false;
  int64_t t = 0, fs = 0, ls = 0;
  if (P.fit_score || fit_out) {
    int64_t s = 0, ws = 0;
    if (P.fit_w_cpu && n.alloc_cpu != 0) {
      s += least_requested(n.nz_cpu + p.nz_cpu, n.alloc_cpu) * P.fit_w_cpu;
      ws += P.fit_w_cpu;
    }
    if (P.fit_w_mem && n.alloc_mem != 0) {
      s += least_requested(n.nz_mem + p.nz_mem, n.alloc_mem) * P.fit_w_mem;
      ws += P.fit_w_mem;
    }
    fs = ws ? div_small(s, ws) : 0;
    if (P.fit_score) t += fs * P.weight_fit;
  }
  if (P.la_score || la_out) {
    if (n.flags & F_LA_SCORE) {
      const bool prodv = (p.flags & P_LA_PROD_SCORE) != 0;
      const int64_t uc = (prodv ? n.la_pused_cpu : n.la_used_cpu) + p.est_cpu;
      const int64_t um = (prodv ? n.la_pused_mem : n.la_used_mem) + p.est_mem;
      int64_t s = 0;
      if (P.la_w_cpu) s += least_requested(uc, n.la_alloc_cpu) * P.la_w_cpu;
      if (P.la_w_mem) s += least_requested(um, n.la_alloc_mem) * P.la_w_mem;
      ls = div_small(s, P.la_wsum);
    }
    if (P.la_score) t += ls * P.weight_la;
  }
  if (fit_out) *fit_out = fs;
  if (la_out) *la_out = ls;
  total = t;
  return rej == 0;
}

// Packed selection key: higher total wins, then LOWER node index (BASELINE pin replacing selectHost's
// reservoir sampling). 0 = no feasible node.
__device__ __forceinline__ uint64_t make_key(int64_t total, uint32_t node) {
  return ((uint64_t)(uint32_t)total << 32) | (uint64_t)(0xFFFFFFFFu - node);
}
__device__ __forceinline__ uint32_t key_node(uint64_t k) { return 0xFFFFFFFFu - (uint32_t)k; }

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const uint64_t o = __shfl_xor(v, off, kWave);
    v = o > v ? o : v;
  }
  return v;
}

}  // namespace kg
