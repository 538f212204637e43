// kernels.h — device data layout and per-(pod,node) evaluation shared by every kernel of the engine.
//
// Node state lives in HBM as structure-of-arrays (one column per field, int64 like the reference's
// framework.Resource fields), replicated on every rank.  A pod is pre-decoded on the host into DevPod
// (requests, non-zero requests, LoadAware estimate, flags).  eval_node() is the fused, reference-shaped body of
//   upstream NodeResourcesFit.Filter (fitsRequest)       — restated in-tree: reservation/plugin.go:433-482
//   LoadAwareScheduling.Filter                            — load_aware.go:123-171 (threshold verdict precomputed)
//   upstream NodeResourcesFit.Score (LeastAllocated, NonZeroRequested) — nodenumaresource/scoring.go:191-230
//   LoadAwareScheduling.Score                             — load_aware.go:269-335, scorer :378-397
//   weighted sum over plugins                             — upstream RunScorePlugins (framework_extender.go:236-258)
// eval_fast<PF>() is the same function on hoisted per-node terms, specialised at compile time on the profile
// (PF bits) and branch-free in the pod flags; the two are checked equal on the device (kg_debug_eval_paths).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kg {

constexpr int kWave = 64;

// Diagnostic build only (-DKG_STAMPS): block 0 / lane 0 records (s_memtime, s_memrealtime) pairs at named
// points of each kernel into a device array read back by kg_debug_stamps.  No stamp executes in the product
// build (the macro expands to nothing).
#ifdef KG_STAMPS
__device__ unsigned long long g_stamps[4][32][2];
#define KG_STAMP(kern, point)                                                      \
  do {                                                                             \
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {                  \
      g_stamps[kern][point][0] = __builtin_amdgcn_s_memtime();                     \
      g_stamps[kern][point][1] = __builtin_amdgcn_s_memrealtime();                 \
    }                                                                              \
  } while (0)
// per-pod diagnostics of the last resolver launch: cycle stamp + path bits
__device__ unsigned long long g_pod_diag[64][6];
#define KG_POD_DIAG(j, bits)                                                       \
  do {                                                                             \
    if (threadIdx.x == 0 && (j) < 64) {                                            \
      g_pod_diag[j][0] = __builtin_amdgcn_s_memtime();                             \
      g_pod_diag[j][1] = (bits);                                                   \
    }                                                                              \
  } while (0)
// NUMA hint merges and the ones that needed the all-permutation fallback pass (diagnostic counters)
__device__ unsigned long long g_merge_count[2];
#define KG_COUNT(i)                                                                \
  do {                                                                             \
    atomicAdd(&g_merge_count[i], 1ull);                                            \
  } while (0)
// sub-phase stamp k (0..3) of pod j
#define KG_POD_SUB(j, k)                                                           \
  do {                                                                             \
    if (threadIdx.x == 0 && (j) < 64) g_pod_diag[j][2 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
// stamp k (0..7) of pod j taken by whichever lane executes it (e.g. the owner lane inside a Reserve)
__device__ unsigned long long g_lane_diag[64][8];
#define KG_LANE_SUB(j, k)                                                          \
  do {                                                                             \
    if ((j) >= 0 && (j) < 64) g_lane_diag[j][k] = __builtin_amdgcn_s_memtime();    \
  } while (0)
#else
#define KG_LANE_SUB(j, k) \
  do {                    \
  } while (0)
#define KG_COUNT(i) \
  do {              \
  } while (0)
#define KG_POD_DIAG(j, bits) \
  do {                       \
  } while (0)
#define KG_POD_SUB(j, k) \
  do {                   \
  } while (0)
#define KG_STAMP(kern, point) \
  do {                        \
  } while (0)
#endif

// profile bits (compile-time specialisation of the evaluation kernels)
constexpr int PF_FIT_FILTER = 1, PF_FIT_SCORE = 2, PF_LA_FILTER = 4, PF_LA_SCORE = 8;
constexpr int PF_LA_PROD = 16;  // LoadAware ScoreAccordingProdUsage: prod pods score on the prod-usage terms

// node flags (device)
constexpr uint32_t F_VALID = 1u << 0;
constexpr uint32_t F_LA_SCORE = 1u << 1;      // NodeMetric present and not expired: LoadAware scores it
constexpr uint32_t F_LA_PASS = 1u << 2;       // LoadAware Filter verdict for a non-prod pod
constexpr uint32_t F_LA_PASS_PROD = 1u << 3;  // LoadAware Filter verdict for a prod pod
constexpr uint32_t F_RARE = 1u << 4;          // EvalRow only: a score input lies outside eval_fast's exact domain
// ephemeral-storage Requested > Allocatable: fitsRequest compares EphemeralStorage for EVERY pod with a non-zero request
// (reservation/plugin.go:469-471: 0 > Allocatable - Requested rejects).  Scheduling never sets it (a placed request fits
// the free amount), so only host deltas (kg_pods_add / remove / unreserve, node upserts) move it: refresh_eph_flags.
constexpr uint32_t F_EPH_OVER = 1u << 6;
// EstimateNode == Allocatable for cpu and memory (no raw-allocatable annotation: default_estimator.go:110-129): the wide
// pass then takes LoadAware's capacity from the Fit columns instead of reading la_alloc_cpu / la_alloc_mem
constexpr uint32_t F_LA_ALLOC_EQ = 1u << 7;

// pod flags (device)
constexpr uint32_t P_ZERO_REQ = 1u << 0;      // every request zero → fitsRequest skips resource checks
constexpr uint32_t P_DAEMONSET = 1u << 1;     // LoadAware Filter bypass (load_aware.go:129-131)
constexpr uint32_t P_PROD = 1u << 2;          // priority class koord-prod
constexpr uint32_t P_LA_PROD_SCORE = 1u << 3; // prod && ScoreAccordingProdUsage (load_aware.go:291)
constexpr uint32_t P_NONPREEMPT = 1u << 4;    // extension.IsPodNonPreemptible (ElasticQuota min check)
constexpr uint32_t P_CPU_KEY = 1u << 5;       // cpu is a key of the pod's requests (PodRequestsAndLimits)
constexpr uint32_t P_MEM_KEY = 1u << 6;       // memory is a key of the pod's requests
constexpr uint32_t P_QDEV = 1u << 7;          // the pod requests device resources (quota dims 2.. are keys)
constexpr uint32_t P_AUX = 1u << 8;           // the pod requests ephemeral-storage or a scalar resource (kAux slots)

// NodeResourcesFit-only resources (kg_pod / kg_node slots KG_RES_EPHEMERAL .. KG_RES_MID_MEMORY): ephemeral-storage
// and the batch / mid cpu / memory extended resources.  Filter only (fitsRequest, reservation/plugin.go:469-479):
// per node an Allocatable and a Requested column each; a pod carries its requests in a side array (pod_aux).
constexpr int kAux = 5;
constexpr int kAuxFirst = 2;

struct DevTable {
  int64_t *alloc_cpu, *alloc_mem;        // NodeInfo.Allocatable
  int64_t *req_cpu, *req_mem;            // NodeInfo.Requested             (mutable)
  int64_t *nz_cpu, *nz_mem;              // NodeInfo.NonZeroRequested      (mutable)
  int64_t *la_alloc_cpu, *la_alloc_mem;  // EstimateNode allocatable
  int64_t *la_used_cpu, *la_used_mem;    // Σ EstimatePod(assigned) + NodeUsage   (mutable)
  int64_t *la_pused_cpu, *la_pused_mem;  // Σ EstimatePod(assigned prod pods)      (mutable)
  int32_t *alloc_pods, *num_pods;        // AllowedPodNumber, len(Pods)    (num_pods mutable)
  uint32_t *flags;
  float *inv_cpu;                        // [2][cap]: 100/alloc_cpu, 100/la_alloc_cpu        (f32 estimates)
  double *inv_mem;                       // [2][cap]: 100/alloc_mem, 100/la_alloc_mem        (f64 estimates)
  int64_t *aux;                          // [2 * kAux][cap]: Allocatable, then Requested, of the kAux resources
  int64_t cap;                           // column stride of the reciprocal columns
};

struct DevPod {
  int64_t req_cpu, req_mem;
  int64_t nz_cpu, nz_mem;
  int64_t est_cpu, est_mem;
  double nz_mem_d, est_mem_d;  // the same quantities as f64 (exact below 2^53) for the memory score terms
  double req_mem_d;            // min(req_mem, 2^53) for the f64 filter compare of the wide pass
  int32_t nz_cpu32, est_cpu32; // min(·, 2^30) for the 32-bit cpu score terms
  int32_t req_cpu32;           // min(req_cpu, 2^30 + 1) for the 32-bit filter compare of the wide pass
  uint32_t flags;
  int32_t quota;  // ElasticQuota table index, -1 = none
  int32_t pad;    // 96 B: a 16-B multiple for LDS-DMA
};
static_assert(sizeof(DevPod) == 96, "DevPod layout");
constexpr int kPodWords = (int)(sizeof(DevPod) / 8);

struct EvalParams {
  int64_t fit_w_cpu, fit_w_mem;
  int64_t la_w_cpu, la_w_mem, la_wsum;
  int64_t weight_fit, weight_la;
  int32_t fit_filter, fit_score, la_filter, la_score;
  int32_t score_bits;  // bit width of the largest possible weighted total
  int32_t monotone;    // every enabled plugin's key can only drop when a pod is assumed (Fit, LoadAware)
  float inv_la_wsum;
  float inv_fit_ws[4];  // 1 / Σ fit weights, indexed by (alloc_cpu != 0) | (alloc_mem != 0) << 1
  int32_t fit_wsum32;   // Σ fit weights (cpu + memory)
  int32_t la_prod_score;  // LoadAwareSchedulingArgs.ScoreAccordingProdUsage
  int32_t pad3;
};

struct Row {
  int64_t alloc_cpu, alloc_mem, req_cpu, req_mem, nz_cpu, nz_mem;
  int64_t la_alloc_cpu, la_alloc_mem, la_used_cpu, la_used_mem, la_pused_cpu, la_pused_mem;
  int32_t alloc_pods, num_pods;
  uint32_t flags;
  float inv_cpu, la_inv_cpu;
  double inv_mem, la_inv_mem;
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
  r.inv_cpu = T.inv_cpu[i];
  r.la_inv_cpu = T.inv_cpu[T.cap + i];
  r.inv_mem = T.inv_mem[i];
  r.la_inv_mem = T.inv_mem[T.cap + i];
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

// leastRequestedScore (load_aware.go:388-397; nodenumaresource/least_allocated.go:49-58):
//   capacity == 0 → 0; requested > capacity → 0; else ((capacity - requested) * 100) / capacity.
// Reference-shaped form (exact integer division when outside [0,100]).
__device__ __forceinline__ int64_t least_requested(int64_t requested, int64_t capacity) {
  if (capacity == 0 || requested > capacity) return 0;
  const int64_t x = capacity - requested;
  const int64_t num = x * 100;
  if (requested < 0) return num / capacity;
  // quotient estimate from v_rcp_f32 (relative error ≤ 2^-21 on a value ≤ 100: within ±1 of the exact quotient,
  // which the two int64 compares then restore — no IEEE division sequence)
  int q = (int)(((float)x * 100.0f) * __builtin_amdgcn_rcpf((float)capacity));
  q = q < 0 ? 0 : (q > 100 ? 100 : q);
  const int64_t t = (int64_t)q * capacity;
  if (t > num) q -= 1;
  else if (t + capacity <= num) q += 1;
  return q;
}

// mostRequestedScore (nodenumaresource/most_allocated.go:50-62, deviceshare/scoring.go:294-304): (min(requested, capacity) · 100) / capacity, division-free like
// least_requested (kernels.h): a float quotient estimate corrected by one exact int64 compare each way.
__device__ __forceinline__ int64_t most_requested64(int64_t requested, int64_t capacity) {
  if (capacity == 0) return 0;
  if (requested > capacity) requested = capacity;
  const int64_t num = requested * 100;
  if (requested < 0) return num / capacity;
  int q = (int)(((float)requested * 100.0f) * __builtin_amdgcn_rcpf((float)capacity));  // as least_requested
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

// Reference-shaped fused Filter + Score of one node for one pod (runtime profile).  Returns false when any
// enabled Filter rejects the node; otherwise writes the weighted total Σ_p weight_p · score_p.
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
      if (n.flags & F_EPH_OVER) rej |= 1u << 7;
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

// fitsRequest over the kAux resources for a pod requesting some of them (req: kAux values, 0 = not requested):
// `request > Allocatable - Requested` rejects (reservation/plugin.go:469-479)
__device__ __forceinline__ bool aux_fits(const DevTable& T, int64_t i, const int64_t* __restrict__ req) {
  bool ok = true;
#pragma unroll
  for (int r = 0; r < kAux; ++r)
    if (req[r] != 0) ok &= !(req[r] > T.aux[(size_t)r * T.cap + i] - T.aux[(size_t)(kAux + r) * T.cap + i]);
  return ok;
}

// Packed selection key: higher total wins, then LOWER node index (BASELINE pin replacing selectHost's
// reservoir sampling). 0 = no feasible node.
__device__ __forceinline__ uint64_t make_key(int64_t total, uint32_t node) {
  return ((uint64_t)(uint32_t)total << 32) | (uint64_t)(0xFFFFFFFFu - node);
}
__device__ __forceinline__ uint32_t key_node(uint64_t k) { return 0xFFFFFFFFu - (uint32_t)k; }

// ---------------------------------------------------------------------------------------------------
// wave primitives
// ---------------------------------------------------------------------------------------------------
// DPP max-reduction over the wave (gfx9 row_shr 1/2/4/8, row_bcast 15/31): result valid in lane 63,
// returned wave-uniform via readlane.  Lanes whose DPP source is out of row read the identity 0.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, CTRL, ROW_MASK, 0xf, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), CTRL, ROW_MASK, 0xf, false);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t wave_max_u64_dpp(uint64_t v) {
  uint64_t w;
  w = dpp_u64<0x111, 0xf>(v); v = w > v ? w : v;  // row_shr:1
  w = dpp_u64<0x112, 0xf>(v); v = w > v ? w : v;  // row_shr:2
  w = dpp_u64<0x114, 0xf>(v); v = w > v ? w : v;  // row_shr:4
  w = dpp_u64<0x118, 0xf>(v); v = w > v ? w : v;  // row_shr:8
  w = dpp_u64<0x142, 0xa>(v); v = w > v ? w : v;  // row_bcast:15
  w = dpp_u64<0x143, 0xc>(v); v = w > v ? w : v;  // row_bcast:31
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 63);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 63);
  return ((uint64_t)hi << 32) | lo;
}

// Inclusive prefix sum over the wave in lane order (DPP row_shr 1/2/4/8 + row_bcast 15/31).
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROW_MASK, 0xf, false);
}
__device__ __forceinline__ uint32_t wave_prefix_sum_u32(uint32_t v) {
  v += dpp_u32<0x111, 0xf>(v);
  v += dpp_u32<0x112, 0xf>(v);
  v += dpp_u32<0x114, 0xf>(v);
  v += dpp_u32<0x118, 0xf>(v);
  v += dpp_u32<0x142, 0xa>(v);
  v += dpp_u32<0x143, 0xc>(v);
  return v;
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readlane((int)wave_prefix_sum_u32(v), 63);
}

__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, int lane) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, lane);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), lane);
  return ((uint64_t)hi << 32) | lo;
}

// ---------------------------------------------------------------------------------------------------
// Wide-pass evaluation on hoisted per-node terms (no division: capacities' reciprocals are static columns).
// ---------------------------------------------------------------------------------------------------
// Domain of eval_fast's exact arithmetic (outside it the row carries F_RARE and the exact path runs):
//   cpu    : 0 < capacity < 2^24 millicores, -2^30 ≤ free ≤ capacity   → 32-bit terms, 24-bit multiplies
//   memory : 0 < capacity < 2^45 bytes,     -2^52 < free ≤ capacity   → f64 terms, every product < 2^53
constexpr int64_t kCpuCapMax = 1ll << 24, kCpuFreeMin = -(1ll << 30);
constexpr int64_t kMemCapMax = 1ll << 45, kMemFreeMin = -(1ll << 52);
constexpr int64_t kPodCpu32Max = 1ll << 30;

struct EvalRow {
  int64_t free_cpu, free_mem;                                     // Allocatable - Requested (fitsRequest)
  int64_t alloc_cpu, fnz_cpu, la_alloc_cpu, la_free_cpu, la_pfree_cpu;  // cpu terms (low dword on the fast path)
  double alloc_mem, fnz_mem, la_alloc_mem, la_free_mem, la_pfree_mem;   // memory terms, exact integers in f64
  double inv_mem, la_inv_mem;                                     // 100 / capacity (f64 estimate)
  float inv_cpu, la_inv_cpu;                                      // 100 / capacity (f32 estimate)
  float inv_fit_ws;                    // 1 / Σ fit weights of resources with non-zero allocatable
  int32_t fit_ws;
  int32_t pods_left;                   // AllowedPodNumber - len(Pods) - 1  (fits iff ≥ 0)
  int32_t alloc_pods;
  uint32_t flags;                      // node flags | F_RARE
  uint32_t pad;
};
static_assert(sizeof(EvalRow) == 144, "EvalRow layout");
constexpr int kEvalRowWords = 18;  // 144 B in uint64 words

__device__ __forceinline__ float i64_to_f32(int64_t x) {  // x ≥ 0; ~1 ulp, enough for a ±1 quotient estimate
  const uint64_t u = (uint64_t)x;
  return fmaf((float)(uint32_t)(u >> 32), 4294967296.0f, (float)(uint32_t)u);
}

__device__ __forceinline__ bool cpu_dom(int64_t cap, int64_t fr) {
  return cap > 0 && cap < kCpuCapMax && fr >= kCpuFreeMin && fr <= cap;
}
__device__ __forceinline__ bool mem_dom(int64_t cap, int64_t fr) {
  return cap > 0 && cap < kMemCapMax && fr > kMemFreeMin && fr <= cap;
}

// F_RARE for the free terms the profile scores (a pure function of the row; recomputed after each assume).
__device__ __forceinline__ uint32_t rare_bit(const EvalRow& e, const EvalParams& P) {
  bool ok = true;
  if (P.fit_score) {
    if (P.fit_w_cpu) ok &= cpu_dom(e.alloc_cpu, e.fnz_cpu);
    if (P.fit_w_mem) ok &= mem_dom((int64_t)e.alloc_mem, (int64_t)e.fnz_mem);
  }
  if (P.la_score && (e.flags & F_LA_SCORE)) {
    if (P.la_w_cpu) ok &= cpu_dom(e.la_alloc_cpu, e.la_free_cpu) && cpu_dom(e.la_alloc_cpu, e.la_pfree_cpu);
    if (P.la_w_mem)
      ok &= mem_dom((int64_t)e.la_alloc_mem, (int64_t)e.la_free_mem) &&
            mem_dom((int64_t)e.la_alloc_mem, (int64_t)e.la_pfree_mem);
  }
  return ok ? 0u : F_RARE;
}

__device__ __forceinline__ EvalRow make_eval_row(const Row& r, const EvalParams& P) {
  EvalRow e;
  e.free_cpu = r.alloc_cpu - r.req_cpu;
  e.free_mem = r.alloc_mem - r.req_mem;
  e.alloc_cpu = r.alloc_cpu;
  e.fnz_cpu = r.alloc_cpu - r.nz_cpu;
  e.la_alloc_cpu = r.la_alloc_cpu;
  e.la_free_cpu = r.la_alloc_cpu - r.la_used_cpu;
  e.la_pfree_cpu = r.la_alloc_cpu - r.la_pused_cpu;
  e.alloc_mem = (double)r.alloc_mem;
  e.fnz_mem = (double)(r.alloc_mem - r.nz_mem);
  e.la_alloc_mem = (double)r.la_alloc_mem;
  e.la_free_mem = (double)(r.la_alloc_mem - r.la_used_mem);
  e.la_pfree_mem = (double)(r.la_alloc_mem - r.la_pused_mem);
  e.inv_mem = r.inv_mem;
  e.la_inv_mem = r.la_inv_mem;
  e.inv_cpu = r.inv_cpu;
  e.la_inv_cpu = r.la_inv_cpu;
  const bool hc = P.fit_w_cpu && r.alloc_cpu != 0, hm = P.fit_w_mem && r.alloc_mem != 0;
  e.fit_ws = (hc ? (int32_t)P.fit_w_cpu : 0) + (hm ? (int32_t)P.fit_w_mem : 0);
  e.inv_fit_ws = hc ? (hm ? P.inv_fit_ws[3] : P.inv_fit_ws[1]) : (hm ? P.inv_fit_ws[2] : 0.0f);
  e.pods_left = r.alloc_pods - r.num_pods - 1;
  e.alloc_pods = r.alloc_pods;
  e.flags = r.flags;
  e.pad = 0;
  // the f64 memory terms are exact only inside the domain; outside it the exact path re-reads the table
  e.flags |= rare_bit(e, P);
  return e;
}

// assume(pod) on a hoisted row: upstream NodeInfo.AddPod + LoadAware Reserve → podAssignCache.assign
// (load_aware.go:260-263).  Capacities and reciprocals are unchanged; only the free terms move.
__device__ __forceinline__ void assume_on(EvalRow& e, const DevPod& p, const EvalParams& P) {
  const bool prod = (p.flags & P_PROD) != 0;
  e.free_cpu -= p.req_cpu;
  e.free_mem -= p.req_mem;
  e.fnz_cpu -= p.nz_cpu;
  e.fnz_mem -= p.nz_mem_d;
  e.la_free_cpu -= p.est_cpu;
  e.la_free_mem -= p.est_mem_d;
  e.la_pfree_cpu -= prod ? p.est_cpu : 0;
  e.la_pfree_mem -= prod ? p.est_mem_d : 0.0;
  e.pods_left -= 1;
  e.flags = (e.flags & ~F_RARE) | rare_bit(e, P);
}

// Mutable columns recovered from a hoisted row (inverse of make_eval_row; exact inside the domain).
__device__ __forceinline__ void store_eval_row(const DevTable& T, int64_t i, const EvalRow& e) {
  const int64_t am = (int64_t)e.alloc_mem, lam = (int64_t)e.la_alloc_mem;
  T.req_cpu[i] = e.alloc_cpu - e.free_cpu;
  T.req_mem[i] = am - e.free_mem;
  T.nz_cpu[i] = e.alloc_cpu - e.fnz_cpu;
  T.nz_mem[i] = am - (int64_t)e.fnz_mem;
  T.la_used_cpu[i] = e.la_alloc_cpu - e.la_free_cpu;
  T.la_used_mem[i] = lam - (int64_t)e.la_free_mem;
  T.la_pused_cpu[i] = e.la_alloc_cpu - e.la_pfree_cpu;
  T.la_pused_mem[i] = lam - (int64_t)e.la_pfree_mem;
  T.num_pods[i] = e.alloc_pods - e.pods_left - 1;
}

__device__ __forceinline__ Row row_of(const EvalRow& e) {  // the reference-shaped row behind a hoisted one
  Row r;
  const int64_t am = (int64_t)e.alloc_mem, lam = (int64_t)e.la_alloc_mem;
  r.alloc_cpu = e.alloc_cpu;
  r.alloc_mem = am;
  r.req_cpu = e.alloc_cpu - e.free_cpu;
  r.req_mem = am - e.free_mem;
  r.nz_cpu = e.alloc_cpu - e.fnz_cpu;
  r.nz_mem = am - (int64_t)e.fnz_mem;
  r.la_alloc_cpu = e.la_alloc_cpu;
  r.la_alloc_mem = lam;
  r.la_used_cpu = e.la_alloc_cpu - e.la_free_cpu;
  r.la_used_mem = lam - (int64_t)e.la_free_mem;
  r.la_pused_cpu = e.la_alloc_cpu - e.la_pfree_cpu;
  r.la_pused_mem = lam - (int64_t)e.la_pfree_mem;
  r.alloc_pods = e.alloc_pods;
  r.num_pods = e.alloc_pods - e.pods_left - 1;
  r.flags = e.flags & ~F_RARE;
  r.inv_cpu = e.inv_cpu;
  r.inv_mem = e.inv_mem;
  r.la_inv_cpu = e.la_inv_cpu;
  r.la_inv_mem = e.la_inv_mem;
  return r;
}

// leastRequestedScore ((x · 100) / capacity, x = capacity - requested; 0 when x < 0) on the fast path.
// cpu (32-bit): the f32 quotient is within ±1 (relative error ≤ 3·2^-24 on a value ≤ 100); one 24-bit
// multiply-compare each way corrects it — q·cap and 100·x stay below 2^31 inside the domain.
__device__ __forceinline__ int32_t lrs_cpu(int32_t x, int32_t cap, float inv) {
  const int32_t xc = x < 0 ? 0 : x;  // x < 0 scores 0, and so does xc = 0 (cap > 0 in the domain)
  int q = (int)((float)xc * inv);
  const int32_t t = (int32_t)__umul24((uint32_t)q, (uint32_t)cap);
  const int32_t num = (int32_t)__umul24((uint32_t)xc, 100u);
  q -= (int)(t > num);
  q += (int)(t + cap <= num);
  return q;
}
// memory (f64): any reciprocal estimate with relative error ≪ 2^-40 puts x·inv within ±1 of the quotient (a value
// ≤ 100); one exact f64 compare each way corrects it — q·cap, (q+1)·cap and 100·x are integers below 2^52.  The wide
// pass feeds it inv100_f64 (v_rcp_f64 + one Newton step, no column read); the exact paths the correctly rounded
// column value.
__device__ __forceinline__ int32_t lrs_mem(double x, double cap, double inv) {
  const double xc = __builtin_fmax(x, 0.0);  // as lrs_cpu: x < 0 → 0
  int q = (int)(xc * inv);
  const double num = xc * 100.0, t = (double)q * cap;
  q -= (int)(t > num);
  q += (int)(t + cap <= num);
  return q;
}

// s / w for 0 ≤ s ≤ 100·w, w ≤ 2·10⁶ (validate_config): f32 estimate + one correction step, 24-bit multiplies.
__device__ __forceinline__ int32_t div_est(int32_t s, int32_t w, float inv_w) {
  int q = (int)((float)s * inv_w);
  const int32_t t = (int32_t)__umul24((uint32_t)q, (uint32_t)w);
  q -= (int)(t > s);
  q += (int)(t + w <= s);
  return q;
}

// Value selects the optimiser cannot turn into a select of field ADDRESSES: that rewrite (select of two loads
// → load of a selected address) would keep a whole EvalRow array in scratch memory instead of registers.
__device__ __forceinline__ int64_t pick(bool c, int64_t a, int64_t b) {
  asm("" : "+v"(a), "+v"(b));
  return c ? b : a;
}
__device__ __forceinline__ int32_t pick(bool c, int32_t a, int32_t b) {
  asm("" : "+v"(a), "+v"(b));
  return c ? b : a;
}
__device__ __forceinline__ double pick(bool c, double a, double b) {
  asm("" : "+v"(a), "+v"(b));
  return c ? b : a;
}

// Branch-free fused Filter + Score on hoisted terms, specialised on the profile PF.  Returns feasibility;
// sets `rare` when the row lies outside the fast path's exact domain (F_RARE) — the caller then re-evaluates
// with eval_node.
template <int PF>
__device__ __forceinline__ bool eval_fast(const EvalRow& n, const DevPod& p, const EvalParams& P, uint32_t& total,
                                          bool& rare) {
  const uint32_t pf = p.flags;
  bool ok = (n.flags & F_VALID) != 0;
  if constexpr ((PF & PF_FIT_FILTER) != 0) {
    const bool fits = (p.req_cpu <= n.free_cpu) & (p.req_mem <= n.free_mem) & !(n.flags & F_EPH_OVER);
    ok = ok & (n.pods_left >= 0) & (((pf & P_ZERO_REQ) != 0) | fits);
  }
  if constexpr ((PF & PF_LA_FILTER) != 0) {
    const uint32_t passbit = (pf & P_PROD) ? F_LA_PASS_PROD : F_LA_PASS;
    ok = ok & (((pf & P_DAEMONSET) != 0) | ((n.flags & passbit) != 0));
  }
  uint32_t t = 0;
  if constexpr ((PF & (PF_FIT_SCORE | PF_LA_SCORE)) != 0) rare |= (n.flags & F_RARE) != 0;
  if constexpr ((PF & PF_FIT_SCORE) != 0) {
    const int32_t qc = lrs_cpu((int32_t)n.fnz_cpu - p.nz_cpu32, (int32_t)n.alloc_cpu, n.inv_cpu);
    const int32_t qm = lrs_mem(n.fnz_mem - p.nz_mem_d, n.alloc_mem, n.inv_mem);
    const int32_t s = (int32_t)(__umul24((uint32_t)qc, (uint32_t)P.fit_w_cpu) +
                                __umul24((uint32_t)qm, (uint32_t)P.fit_w_mem));
    const int32_t f = div_est(s, n.fit_ws, n.inv_fit_ws);
    t += __umul24((uint32_t)(n.fit_ws ? f : 0), (uint32_t)P.weight_fit);
  }
  if constexpr ((PF & PF_LA_SCORE) != 0) {
    const bool prodv = (pf & P_LA_PROD_SCORE) != 0;
    const int32_t fc = (int32_t)pick(prodv, n.la_free_cpu, n.la_pfree_cpu);
    const double fm = pick(prodv, n.la_free_mem, n.la_pfree_mem);
    const int32_t qc = lrs_cpu(fc - p.est_cpu32, (int32_t)n.la_alloc_cpu, n.la_inv_cpu);
    const int32_t qm = lrs_mem(fm - p.est_mem_d, n.la_alloc_mem, n.la_inv_mem);
    const int32_t s = (int32_t)(__umul24((uint32_t)qc, (uint32_t)P.la_w_cpu) +
                                __umul24((uint32_t)qm, (uint32_t)P.la_w_mem));
    const int32_t l = div_est(s, (int32_t)P.la_wsum, P.inv_la_wsum);
    t += __umul24((uint32_t)((n.flags & F_LA_SCORE) ? l : 0), (uint32_t)P.weight_la);
  }
  total = t;
  return ok;
}

// ---------------------------------------------------------------------------------------------------
// Wide-pass row (eval_round): the hoisted terms of one node in the narrowest exact types — cpu terms in
// 32-bit lanes, memory terms as exact f64 integers, pod-count fit folded into the flags.  ~23 VGPRs per node
// (EvalRow: 36) so a lane can hold 4 nodes at 4 waves/SIMD.  F_RARE marks a row outside the exact domain of
// eval_hot (a pure function of the node, so it is decided once per tile, not per pod).
// ---------------------------------------------------------------------------------------------------
constexpr uint32_t F_PODS_OK = 1u << 5;  // HotRow only: F_VALID && len(Pods) + 1 <= AllowedPodNumber
constexpr int64_t kFreeCpuAbs = 1ll << 30;  // |Allocatable - Requested| cpu bound of the 32-bit filter compare
constexpr int64_t kFreeMemAbs = 1ll << 52;  // |Allocatable - Requested| memory bound of the f64 filter compare

struct HotRow {
  int32_t free_cpu, fnz_cpu, alloc_cpu, la_free_cpu, la_pfree_cpu, la_alloc_cpu;
  float inv_cpu, la_inv_cpu;
  double free_mem, fnz_mem, alloc_mem, inv_mem, la_free_mem, la_pfree_mem, la_alloc_mem, la_inv_mem;
  uint32_t flags;
};

// 100 / capacity for the cpu terms from v_rcp_f32 (≤ 2 ulp), computed where a tile's rows are hoisted so that the
// wide pass does not read the f32 reciprocal columns: lrs_cpu needs only an estimate within ±1 of the quotient (its
// 24-bit multiply-compare corrects it both ways; relative error ≤ 2^-22 on a value ≤ 100), and inside the domain the
// capacity is < 2^24, so (float)c is exact.  (r3) The memory reciprocals likewise (inv100_f64): lrs_mem corrects both
// ways, so the f64 columns are read only by the exact paths.
__device__ __forceinline__ float inv100_f32(int64_t c) {
  return c > 0 ? 100.0f * __builtin_amdgcn_rcpf((float)c) : 0.0f;
}
// 100 / capacity for the memory terms: v_rcp_f64 refined by one Newton step (relative error far below 2^-40, which is
// all lrs_mem's two-way correction needs), so the wide pass does not read the f64 reciprocal columns either
__device__ __forceinline__ double inv100_f64(int64_t c) {
  if (c <= 0) return 0.0;
  const double d = (double)c;
  const double r0 = __builtin_amdgcn_rcp(d);
  return 100.0 * __builtin_fma(r0, __builtin_fma(-d, r0, 1.0), r0);
}

// The columns of one hot row, loaded without branches (every load unconditional, or from a selected column), so that
// a tile's rows are all in flight at once: the wide pass waits once for its rows instead of once per conditional load
// (r3: the branchy loads compiled to ~3 waits per row, ~half of a wave's life parked on vmcnt).
struct HotCols {
  uint32_t fl;
  int32_t np, ap;
  int64_t ac, am, rc, rm, nc, nm, luc, lum, lpc, lpm, lac, lam;
};
template <int PF>
__device__ __forceinline__ void load_hot_cols(const DevTable& T, int64_t i, HotCols& c) {
  constexpr bool kLa = (PF & PF_LA_SCORE) != 0, kProd = (PF & PF_LA_PROD) != 0;
  c.fl = T.flags[i];
  c.ac = T.alloc_cpu[i];
  c.am = T.alloc_mem[i];
  c.rc = T.req_cpu[i];
  c.rm = T.req_mem[i];
  c.nc = T.nz_cpu[i];
  c.nm = T.nz_mem[i];
  c.np = T.num_pods[i];
  c.ap = T.alloc_pods[i];
  c.luc = kLa ? T.la_used_cpu[i] : 0;
  c.lum = kLa ? T.la_used_mem[i] : 0;
  c.lpc = kProd ? T.la_pused_cpu[i] : 0;
  c.lpm = kProd ? T.la_pused_mem[i] : 0;
}
// EstimateNode capacity: the Fit column again (a cache hit) when F_LA_ALLOC_EQ, else the LoadAware column — one load
// from a selected column, after the flags
template <int PF>
__device__ __forceinline__ void load_hot_la_alloc(const DevTable& T, int64_t i, HotCols& c) {
  if constexpr ((PF & PF_LA_SCORE) != 0) {
    const bool eq = (c.fl & F_LA_ALLOC_EQ) != 0;
    const int64_t* cc = eq ? T.alloc_cpu : T.la_alloc_cpu;
    const int64_t* cm = eq ? T.alloc_mem : T.la_alloc_mem;
    c.lac = cc[i];
    c.lam = cm[i];
  } else {
    c.lac = c.lam = 0;
  }
}
template <int PF>
__device__ __forceinline__ HotRow hot_from_cols(const HotCols& c, const EvalParams& P) {
  HotRow h;
  const uint32_t fl = c.fl;
  const int64_t ac = c.ac, am = c.am;
  const int64_t fc = ac - c.rc, fm = am - c.rm;
  const int64_t fnc = ac - c.nc, fnm = am - c.nm;
  // LoadAware terms only for rows it scores
  constexpr bool kLa = (PF & PF_LA_SCORE) != 0;
  const bool la_row = kLa && (fl & F_LA_SCORE) != 0, la_eq = (fl & F_LA_ALLOC_EQ) != 0;
  const int64_t lac = la_row ? c.lac : 0, lam = la_row ? c.lam : 0;
  const int64_t lfc = la_row ? lac - c.luc : 0, lfm = la_row ? lam - c.lum : 0;
  constexpr bool kProd = (PF & PF_LA_PROD) != 0;
  const int64_t lpc = kProd && la_row ? lac - c.lpc : 0, lpm = kProd && la_row ? lam - c.lpm : 0;
  const bool pods_ok = c.np + 1 <= c.ap;
  bool ok = true;
  if constexpr ((PF & PF_FIT_FILTER) != 0) ok &= (fc >= -kFreeCpuAbs) & (fc <= kFreeCpuAbs) & (fm > -kFreeMemAbs) & (fm < kFreeMemAbs);
  if constexpr ((PF & PF_FIT_SCORE) != 0) {
    if (P.fit_w_cpu) ok &= cpu_dom(ac, fnc);
    if (P.fit_w_mem) ok &= mem_dom(am, fnm);
  }
  if constexpr ((PF & PF_LA_SCORE) != 0) {
    if (fl & F_LA_SCORE) {
      if (P.la_w_cpu) ok &= cpu_dom(lac, lfc) && (!kProd || cpu_dom(lac, lpc));
      if (P.la_w_mem) ok &= mem_dom(lam, lfm) && (!kProd || mem_dom(lam, lpm));
    }
  }
  h.free_cpu = (int32_t)fc;
  h.fnz_cpu = (int32_t)fnc;
  h.alloc_cpu = (int32_t)ac;
  h.la_free_cpu = (int32_t)lfc;
  h.la_pfree_cpu = (int32_t)lpc;
  h.la_alloc_cpu = (int32_t)lac;
  constexpr bool kFitS = (PF & PF_FIT_SCORE) != 0;
  h.inv_cpu = kFitS ? inv100_f32(ac) : 0.0f;
  h.la_inv_cpu = la_row ? inv100_f32(lac) : 0.0f;
  h.free_mem = (double)fm;
  h.fnz_mem = (double)fnm;
  h.alloc_mem = (double)am;
  h.inv_mem = kFitS ? inv100_f64(am) : 0.0;
  h.la_free_mem = (double)lfm;
  h.la_pfree_mem = (double)lpm;
  h.la_alloc_mem = (double)lam;
  h.la_inv_mem = !la_row ? 0.0 : (kFitS && la_eq) ? h.inv_mem : inv100_f64(lam);
  h.flags = (fl & ~(F_RARE | F_PODS_OK)) | ((fl & F_VALID) && pods_ok ? F_PODS_OK : 0u) | (ok ? 0u : F_RARE);
  return h;
}
template <int PF>
__device__ __forceinline__ HotRow load_hot(const DevTable& T, int64_t i, const EvalParams& P) {
  HotCols c;
  load_hot_cols<PF>(T, i, c);
  load_hot_la_alloc<PF>(T, i, c);
  return hot_from_cols<PF>(c, P);
}

// eval_hot<PF>: eval_fast on a HotRow (caller guarantees !(flags & F_RARE)).  The pod's request/estimate
// quantities come pre-narrowed in DevPod: req_cpu32 = min(req_cpu, 2^30 + 1) (any larger request fails the
// 32-bit compare exactly as the int64 one does, since |free_cpu| ≤ 2^30), req_mem_d = min(req_mem, 2^53).
template <int PF>
__device__ __forceinline__ bool eval_hot(const HotRow& n, const DevPod& p, const EvalParams& P, uint32_t& total) {
  const uint32_t pf = p.flags;
  bool ok = (n.flags & F_VALID) != 0;
  if constexpr ((PF & PF_FIT_FILTER) != 0) {
    const bool fits = (p.req_cpu32 <= n.free_cpu) & (p.req_mem_d <= n.free_mem) & !(n.flags & F_EPH_OVER);
    ok = ((n.flags & F_PODS_OK) != 0) & (((pf & P_ZERO_REQ) != 0) | fits);
  }
  if constexpr ((PF & PF_LA_FILTER) != 0) {
    const uint32_t passbit = (pf & P_PROD) ? F_LA_PASS_PROD : F_LA_PASS;
    ok = ok & (((pf & P_DAEMONSET) != 0) | ((n.flags & passbit) != 0));
  }
  uint32_t t = 0;
  if constexpr ((PF & PF_FIT_SCORE) != 0) {
    const int32_t qc = lrs_cpu(n.fnz_cpu - p.nz_cpu32, n.alloc_cpu, n.inv_cpu);
    const int32_t qm = lrs_mem(n.fnz_mem - p.nz_mem_d, n.alloc_mem, n.inv_mem);
    const int32_t s = (int32_t)(__umul24((uint32_t)qc, (uint32_t)P.fit_w_cpu) +
                                __umul24((uint32_t)qm, (uint32_t)P.fit_w_mem));
    // inside the domain every weighted resource has allocatable > 0: Σ weights is the profile constant
    const int32_t f = div_est(s, P.fit_wsum32, P.inv_fit_ws[3]);
    t += __umul24((uint32_t)(P.fit_wsum32 ? f : 0), (uint32_t)P.weight_fit);
  }
  if constexpr ((PF & PF_LA_SCORE) != 0) {
    int32_t fc = n.la_free_cpu;
    double fm = n.la_free_mem;
    if constexpr ((PF & PF_LA_PROD) != 0) {
      const bool prodv = (pf & P_LA_PROD_SCORE) != 0;
      fc = pick(prodv, n.la_free_cpu, n.la_pfree_cpu);
      fm = pick(prodv, n.la_free_mem, n.la_pfree_mem);
    }
    const int32_t qc = lrs_cpu(fc - p.est_cpu32, n.la_alloc_cpu, n.la_inv_cpu);
    const int32_t qm = lrs_mem(fm - p.est_mem_d, n.la_alloc_mem, n.la_inv_mem);
    const int32_t s = (int32_t)(__umul24((uint32_t)qc, (uint32_t)P.la_w_cpu) +
                                __umul24((uint32_t)qm, (uint32_t)P.la_w_mem));
    const int32_t l = div_est(s, (int32_t)P.la_wsum, P.inv_la_wsum);
    t += __umul24((uint32_t)((n.flags & F_LA_SCORE) ? l : 0), (uint32_t)P.weight_la);
  }
  total = t;
  return ok;
}

// Wave max of a packed 64-bit key in two 32-bit DPP max scans (high word, then the low word among the lanes
// holding the high maximum).  Returns the wave-uniform maximum.
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  v = max(v, dpp_u32<0x111, 0xf>(v));  // row_shr:1
  v = max(v, dpp_u32<0x112, 0xf>(v));  // row_shr:2
  v = max(v, dpp_u32<0x114, 0xf>(v));  // row_shr:4
  v = max(v, dpp_u32<0x118, 0xf>(v));  // row_shr:8
  v = max(v, dpp_u32<0x142, 0xa>(v));  // row_bcast:15
  v = max(v, dpp_u32<0x143, 0xc>(v));  // row_bcast:31
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
__device__ __forceinline__ uint64_t wave_max_key(uint64_t k) {
  const uint32_t hi = wave_max_u32((uint32_t)(k >> 32));
  const uint32_t lo = wave_max_u32((uint32_t)(k >> 32) == hi ? (uint32_t)k : 0u);
  return ((uint64_t)hi << 32) | lo;
}

// ---------------------------------------------------------------------------------------------------
// ElasticQuota admission inside the FIFO resolvers (elasticquota/plugin.go:211-256 PreFilter, :332-346 Reserve).
// The quota table in HBM holds KG_QUOTA_RES resources per quota (cpu, memory, then the 6 device resources of
// kg_pod.device_requests).  The lane-based resolvers (Fit + LoadAware, NodeNUMAResource) only see pods without
// device requests, so they keep quota q's cpu / memory part in lane q (DevQuota) and leave the device dims as they
// are; pod j+1's check reads it by readlane and a placed pod is charged by that lane, so pod j+1's check sees pod j's
// Reserve, as in the reference.  The DeviceShare / Reservation resolvers use the full rows (QuotaRow).
// ---------------------------------------------------------------------------------------------------
constexpr int kQuotaRes = 8;
struct QuotaRow {  // one kg_quota on the device (same field order, int64)
  int64_t used[kQuotaRes], np[kQuotaRes], lim[kQuotaRes], min[kQuotaRes];
};
static_assert(sizeof(QuotaRow) == 256, "QuotaRow layout");

struct DevQuota {
  int64_t used_c, used_m, np_c, np_m, lim_c, lim_m, min_c, min_m;
};

__device__ __forceinline__ DevQuota quota_load(const QuotaRow* __restrict__ q, int nq, int lane) {
  DevQuota r{0, 0, 0, 0, 0, 0, 0, 0};
  if (lane < nq) {
    const QuotaRow& x = q[lane];
    r = DevQuota{x.used[0], x.used[1], x.np[0], x.np[1], x.lim[0], x.lim[1], x.min[0], x.min[1]};
  }
  return r;
}
__device__ __forceinline__ void quota_store(QuotaRow* __restrict__ q, int nq, int lane, const DevQuota& r) {
  if (lane < nq) {
    QuotaRow& x = q[lane];
    x.used[0] = r.used_c, x.used[1] = r.used_m, x.np[0] = r.np_c, x.np[1] = r.np_m;
  }
}

// quotav1.LessThanOrEqual(Mask(Add(request, used), ResourceNames(request)), limit) over cpu / memory (wave-uniform):
// only the pod's request keys are compared, and only where the limit has the key (a limit < 0 is absent)
__device__ __forceinline__ bool quota_admit(const DevQuota& ql, const DevPod& p) {
  if (p.quota < 0) return true;
  const int q = p.quota;
  const bool kc = (p.flags & P_CPU_KEY) != 0, km = (p.flags & P_MEM_KEY) != 0;
  const int64_t uc = (int64_t)readlane_u64((uint64_t)ql.used_c, q), um = (int64_t)readlane_u64((uint64_t)ql.used_m, q);
  const int64_t lc = (int64_t)readlane_u64((uint64_t)ql.lim_c, q), lm = (int64_t)readlane_u64((uint64_t)ql.lim_m, q);
  bool ok = (!kc || lc < 0 || uc + p.req_cpu <= lc) && (!km || lm < 0 || um + p.req_mem <= lm);
  if (p.flags & P_NONPREEMPT) {
    const int64_t nc = (int64_t)readlane_u64((uint64_t)ql.np_c, q), nm = (int64_t)readlane_u64((uint64_t)ql.np_m, q);
    const int64_t mc = (int64_t)readlane_u64((uint64_t)ql.min_c, q), mm = (int64_t)readlane_u64((uint64_t)ql.min_m, q);
    ok = ok && (!kc || mc < 0 || nc + p.req_cpu <= mc) && (!km || mm < 0 || nm + p.req_mem <= mm);
  }
  return ok;
}

// GroupQuotaManager.ReservePod → updatePodUsedNoLock (core/group_quota_manager.go:613-648, 791-797)
__device__ __forceinline__ void quota_charge(DevQuota& ql, const DevPod& p, int lane) {
  if (p.quota != lane) return;
  ql.used_c += p.req_cpu;
  ql.used_m += p.req_mem;
  if (p.flags & P_NONPREEMPT) {
    ql.np_c += p.req_cpu;
    ql.np_m += p.req_mem;
  }
}

// Full-row forms (device requests included): the pod's request over the quota resources is (cpu, memory,
// dev[0..5]) with key flags; `add` (nullable) = earlier usage not yet in the row.
struct QuotaReq {
  int64_t r[kQuotaRes];
  uint32_t keys;  // bit d: resource d is a key of the pod's requests
};
__device__ __forceinline__ QuotaReq quota_req(const DevPod& p, const int64_t* __restrict__ dev6) {
  QuotaReq q;
  q.r[0] = p.req_cpu;
  q.r[1] = p.req_mem;
  q.keys = ((p.flags & P_CPU_KEY) ? 1u : 0u) | ((p.flags & P_MEM_KEY) ? 2u : 0u);
#pragma unroll
  for (int d = 0; d < kQuotaRes - 2; ++d) {
    q.r[2 + d] = (p.flags & P_QDEV) ? dev6[d] : 0;
    q.keys |= q.r[2 + d] != 0 ? (1u << (2 + d)) : 0u;
  }
  return q;
}
__device__ __forceinline__ bool quota_row_admit(const QuotaRow& Q, const QuotaReq& rq, bool nonpreempt,
                                                const int64_t* add_used = nullptr, const int64_t* add_np = nullptr) {
  // add_used / add_np (nullable): usage of earlier placements not yet charged into the row
  bool ok = true;
#pragma unroll
  for (int d = 0; d < kQuotaRes; ++d) {
    if (!((rq.keys >> d) & 1u)) continue;
    const int64_t au = add_used ? add_used[d] : 0, an = add_np ? add_np[d] : 0;
    if (Q.lim[d] >= 0 && Q.used[d] + au + rq.r[d] > Q.lim[d]) ok = false;
    if (nonpreempt && Q.min[d] >= 0 && Q.np[d] + an + rq.r[d] > Q.min[d]) ok = false;
  }
  return ok;
}
__device__ __forceinline__ void quota_row_charge(QuotaRow& Q, const QuotaReq& rq, bool nonpreempt) {
#pragma unroll
  for (int d = 0; d < kQuotaRes; ++d) {
    Q.used[d] += rq.r[d];
    if (nonpreempt) Q.np[d] += rq.r[d];
  }
}

}  // namespace kg
