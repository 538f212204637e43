// engine.hip — koordgpu: MI355X batch Filter/Score engine behind the C ABI of include/koordgpu.h.
//
// Device algorithm: scheduling is sequential per pod (each placement is assumed before the
// next pod is scored), but a placement changes exactly ONE node row.  The engine therefore works in rounds of
// B queued pods:
//   1. eval_round   — every (pod, node) pair of the round is scored against the round-start snapshot in one
//                     wide, coalesced pass; per (pod, 256-node tile) only the top-R packed keys survive
//                     (score-bit threshold select with wave ballots — no sort, no LDS).
//   2. [RCCL]       — n_ranks>1: ncclAllGather of the candidate lists (nodes are sharded, state replicated).
//   3. resolve_round — one wavefront replays the B pods in FIFO order: the best candidate not yet modified in
//                     this round, vs. the exact re-score of the ≤B rows modified in this round (held in
//                     registers).  If a tile's whole candidate list was modified and its unknown remainder could
//                     still win, the round stops early and the rest of the pods go to the next round.
// Result = exactly the sequential reference decision (proof sketch in DESIGN.md §3.3), ties → lowest index.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <mutex>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/koordgpu.h"
#include "kernels.h"
#include "numa_dev.h"
#include "ds_dev.h"
#include "rsv_dev.h"

using namespace kg;

namespace {

constexpr int kNPT = 4;               // nodes per lane in an eval tile
constexpr int kTile = kWave * kNPT;   // 256 nodes per tile
// (r4) eval_round's own geometry: kENPT nodes per lane, kEW tiles (waves) per block = 1,024-node tile groups.
// KG_EVAL_NPT=4 restores the round-3 shape (4 waves of 256-node tiles)
#ifndef KG_EVAL_NPT
#define KG_EVAL_NPT 2
#endif
#ifndef KG_EVAL_EW
#define KG_EVAL_EW (16 / KG_EVAL_NPT)
#endif
constexpr int kENPT = KG_EVAL_NPT;
constexpr int kETile = kWave * kENPT;
constexpr int kEW = KG_EVAL_EW;
constexpr int kR = 8;                 // candidates kept per (pod, tile)
#ifndef KG_GROUP_KEYS
#define KG_GROUP_KEYS 8
#endif
constexpr int kRG = KG_GROUP_KEYS;    // (r5) candidates kept per (pod, tile group of kEW tiles): the merge's input
static_assert(kRG % 2 == 0 && kRG <= kR, "group lists: an even count of at most kR keys");
constexpr int kEvalWaves = 4;         // waves (tiles) per eval block
constexpr int kMaxB = 64;             // modified rows are held one per lane of the resolver wave
constexpr int kC = 64;                // merged candidates per pod (> any modified-set size: kC > kMaxB - 1)
constexpr int kStaged = 3;            // hoisted rows of each pod's best candidates shipped with its record
constexpr int kRecRows = 72;          // record layout (uint64 words): [0,kC) keys, [kC] ub, [72, 72+3·17) rows
constexpr int kCandStride = 128;      // per-pod record: 1 KiB (a 16-B multiple, for LDS-DMA)
constexpr int kMergeThreads = 256;
constexpr int kMergeChunks = 4;       // chunks of 8 keys per merge thread: ≤ 1024 tile lists = 262144 nodes per rank
constexpr double kAlgoBytesPerNode = 76.0;  // SURVEY §8(d) b_node for C1-C3: Fit 56 B + LoadAware 20 B
constexpr int64_t kMaxBatchRounds = 256;
constexpr int64_t kSpinLimit = 1 << 25;  // resolver chain wait: ~2 s of s_sleep(2) before reporting an error  // rounds launched between two host synchronisations
constexpr int64_t kMaxNodes = 1 << 19;  // resolver LDS: N/8-byte bitmap (≤ 64 KiB) + the round's records (≤ 64 KiB)
static_assert(kRecRows + kStaged * kEvalRowWords <= kCandStride, "record layout");

thread_local std::string g_err;

// (r5) Go's math.Log (src/math/log.go; amd64 archLog evaluates the same expression, no FMA contraction), in plain IEEE
// double arithmetic (this file builds with -ffp-contract=off).  PodTopologySpread's topologyNormalizingWeight is
// math.Log(size + 2), truncated after a multiply-add, so the weight table is built with Go's algorithm, not libm's
// (the oracle's or_go_log is the same restatement; tests/test_go_log.py lists where glibc's log differs).
double go_log(double x) {
  const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10;
  const double L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01, L3 = 2.857142874366239149e-01,
               L4 = 2.222219843214978396e-01, L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01,
               L7 = 1.479819860511658591e-01;
  if (std::isnan(x) || (std::isinf(x) && x > 0)) return x;
  if (x < 0) return std::nan("");
  if (x == 0) return -HUGE_VAL;
  int ki = 0;
  double f1 = std::frexp(x, &ki);
  if (f1 < 0.70710678118654752440) {  // math.Sqrt2 / 2
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

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                                      \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    if (e_ != hipSuccess) return fail(KG_E_DEVICE, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

#define NCCL_TRY(expr)                                                                           \
  do {                                                                                           \
    ncclResult_t r_ = (expr);                                                                    \
    if (r_ != ncclSuccess) return fail(KG_E_COLLECTIVE, "%s: %s", #expr, ncclGetErrorString(r_)); \
  } while (0)

typedef __attribute__((address_space(3))) void* lds_void_ptr;
typedef const __attribute__((address_space(1))) void* global_cvoid_ptr;

// ------------------------------------------------------------------------------------------------
// Kernels
// ------------------------------------------------------------------------------------------------

// ---- round kernel 1: wide evaluation -------------------------------------------------------------
// One wave = one tile of kTile nodes (lane l holds nodes tile*kTile + j*64 + l, j < kNPT, as HotRows in
// registers) × pods_per_wave pods of the round [first, first + nb).  Writes lists[(pod, tile)][kR] = the
// tile's top-kR packed keys (ascending node order, zero-padded).  The table may be mid-update by the previous
// round's resolver (pipelining): every column load is a single aligned 8-/4-byte load, so a
// row reads as a mix of pre- and post-assume columns, whose key is ≥ the row's current key (monotone profile);
// the resolver re-scores those rows exactly.  `poison` ≠ 0: an earlier round of this batch stopped early, so
// this round's pods are not the next ones — nothing to do.
// Per (pod, tile): the tile's top-kR packed keys from v[j] = feasible ? total + 1 : 0 (one value per node, so a
// compare needs no feasibility mask).  τ = the largest v with count(v ≥ τ) ≥ kR, one ballot per value bit;
// ties at τ go to the lowest node index (register j, then lane).  Writes the list in ascending node order.
template <int NPT>
__device__ __forceinline__ void select_write(const uint32_t (&v)[NPT], const uint32_t (&gidx)[NPT], int vbits,
                                             uint64_t* __restrict__ out, int lane) {
  uint64_t fm[NPT], sel[NPT];
  int nfeas = 0;
#pragma unroll
  for (int j = 0; j < NPT; ++j) {
    fm[j] = __ballot(v[j] != 0);
    nfeas += __popcll(fm[j]);
  }
  if (nfeas <= kR) {
#pragma unroll
    for (int j = 0; j < NPT; ++j) sel[j] = fm[j];
  } else {
    // (r5) τ from the tile's maximum first: the kR best of 64·NPT values usually lie within kSelWin of it, where
    // log2(kSelWin) bisection steps suffice; otherwise the full vbits-step bisection (both give the same τ)
    constexpr uint32_t kSelWin = 16;
    uint32_t vm = 0;
#pragma unroll
    for (int j = 0; j < NPT; ++j) vm = v[j] > vm ? v[j] : vm;
    const uint32_t top = wave_max_u32(vm);
    const uint32_t lo = top > kSelWin ? top - (kSelWin - 1) : 1u;
    int cnt_lo = 0;
#pragma unroll
    for (int j = 0; j < NPT; ++j) cnt_lo += __popcll(__ballot(v[j] >= lo));
    uint32_t cur = 0;
    if (cnt_lo >= kR) {  // τ ∈ [lo, top]
      cur = lo;
#pragma unroll
      for (int b = 3; b >= 0; --b) {
        const uint32_t c = cur + (1u << b);
        int cnt = 0;
#pragma unroll
        for (int j = 0; j < NPT; ++j) cnt += __popcll(__ballot(v[j] >= c));
        if (c <= top && cnt >= kR) cur = c;
      }
    } else {
      for (int b = vbits - 1; b >= 0; --b) {
        const uint32_t c = cur | (1u << b);
        int cnt = 0;
#pragma unroll
        for (int j = 0; j < NPT; ++j) cnt += __popcll(__ballot(v[j] >= c));
        if (cnt >= kR) cur = c;
      }
    }
    int need = kR;
    uint64_t eq[NPT];
#pragma unroll
    for (int j = 0; j < NPT; ++j) {
      sel[j] = __ballot(v[j] > cur);
      eq[j] = __ballot(v[j] == cur);
      need -= __popcll(sel[j]);
    }
    // ties at τ in (register j, lane) order: a lane's rank among them is a masked bit count, no peeling loop
    const uint64_t lane_lt0 = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    int base = 0;
#pragma unroll
    for (int j = 0; j < NPT; ++j) {
      const int r = base + __popcll(eq[j] & lane_lt0);
      sel[j] |= __ballot(((eq[j] >> lane) & 1ull) && r < need);
      base += __popcll(eq[j]);
    }
  }
  const uint64_t lane_lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  int base = 0;
#pragma unroll
  for (int j = 0; j < NPT; ++j) {
    if ((sel[j] >> lane) & 1) out[base + __popcll(sel[j] & lane_lt)] = make_key(v[j] - 1, gidx[j]);
    base += __popcll(sel[j]);
  }
  if (lane >= base && lane < kR) out[lane] = 0;
}

// A tile holding a row outside eval_hot's exact domain: the reference-shaped int64 path for every pod (rare).
// The row index is laundered inside the loop so the compiler cannot hoist the 19 column addresses out of it
// (they would stay live across the wide loop and halve its occupancy).
template <int NPT>
__device__ __forceinline__ void eval_tile_exact(const DevTable& T, const DevPod* __restrict__ pods, int64_t first,
                                             int p0, int p1, int tile, int64_t node_base, int64_t n_local,
                                             const EvalParams& P, uint64_t* __restrict__ out, int64_t out_stride,
                                             int vbits, const int64_t* __restrict__ paux) {
  const int lane = threadIdx.x % kWave;
  uint32_t gidx[NPT];
#pragma unroll
  for (int j = 0; j < NPT; ++j) gidx[j] = (uint32_t)(node_base + (int64_t)tile * (kWave * NPT) + j * kWave + lane);
  for (int pi = p0; pi < p1; ++pi) {
    const DevPod p = pods[first + pi];
    uint32_t v[NPT];
#pragma unroll
    for (int j = 0; j < NPT; ++j) {
      int64_t local = (int64_t)tile * (kWave * NPT) + j * kWave + lane;
      asm volatile("" : "+v"(local));
      int64_t t = 0;
      v[j] = (local < n_local && eval_node(load_row(T, node_base + local), p, P, t)) ? (uint32_t)t + 1u : 0u;
      if (P.fit_filter && (p.flags & P_AUX) && v[j] && !aux_fits(T, node_base + local, paux + (size_t)(first + pi) * kAux))
        v[j] = 0;
    }
    select_write(v, gidx, vbits, out + (size_t)(pi - p0) * out_stride, lane);
  }
}

// one wave's tile for pods [p0, p1): its kR best packed keys per pod into out[(pi - p0) * kR ..]
template <int PF, int NPT, bool AUX>
__device__ __forceinline__ void eval_tile(const DevTable& T, const DevPod* __restrict__ pods, int64_t first, int p0,
                                          int p1, int tile, int64_t node_base, int64_t n_local, const EvalParams& P,
                                          uint64_t* __restrict__ out, int64_t out_stride, int vbits,
                                          const int64_t* __restrict__ paux, int lane) {

  HotRow rows[NPT];
  uint32_t gidx[NPT];
  bool rare = false;
  {  // every column load of the tile's rows issued before any is used (a row past the shard reads the shard's last
     // row — row 0 for an empty shard — and is masked invalid): one wait for the tile instead of a wait per
     // conditional load
    HotCols c[NPT];
    int64_t ii[NPT];
#pragma unroll
    for (int j = 0; j < NPT; ++j) {
      const int64_t local = (int64_t)tile * (kWave * NPT) + j * kWave + lane;
      gidx[j] = (uint32_t)(node_base + local);
      ii[j] = local < n_local ? node_base + local : (n_local > 0 ? node_base + n_local - 1 : 0);
      load_hot_cols<PF>(T, ii[j], c[j]);
    }
#pragma unroll
    for (int j = 0; j < NPT; ++j) load_hot_la_alloc<PF>(T, ii[j], c[j]);
#pragma unroll
    for (int j = 0; j < NPT; ++j) {
      const int64_t local = (int64_t)tile * (kWave * NPT) + j * kWave + lane;
      rows[j] = hot_from_cols<PF>(c[j], P);
      if (local >= n_local) rows[j].flags = 0;  // not F_VALID → never feasible
      rare |= (rows[j].flags & F_RARE) != 0;
    }
  }
  KG_STAMP(0, 1);
  // a row outside eval_hot's exact domain anywhere in the tile: the whole tile takes the exact path
  if (__ballot(rare)) {
    eval_tile_exact<NPT>(T, pods, first, p0, p1, tile, node_base, n_local, P, out, out_stride, vbits, paux);
    return;
  }
  for (int pi = p0; pi < p1; ++pi) {
    const DevPod p = pods[first + pi];
    uint32_t v[NPT];
#pragma unroll
    for (int j = 0; j < NPT; ++j) {
      uint32_t t = 0;
      v[j] = eval_hot<PF>(rows[j], p, P, t) ? t + 1u : 0u;
    }
    // ephemeral-storage / scalar requests: the Allocatable-Requested columns.  (r5) Compiled only into the AUX
    // instantiation (a staged queue holding such a pod): the check cost the common kernel 20 VGPRs
    if constexpr (AUX && (PF & PF_FIT_FILTER) != 0) {
      if (p.flags & P_AUX) {
        const int64_t* rq = paux + (size_t)(first + pi) * kAux;
#pragma unroll
        for (int j = 0; j < NPT; ++j)
          if (v[j] && !aux_fits(T, gidx[j], rq)) v[j] = 0;
      }
    }
    select_write(v, gidx, vbits, out + (size_t)(pi - p0) * out_stride, lane);
  }
}

template <int L, int LL>
__device__ __forceinline__ void merge_pod(const DevTable& T, const EvalParams& P, const uint64_t* __restrict__ base,
                                          int n_lists, uint64_t* sel, uint64_t* __restrict__ o, int lane);

// (r5) The merge fused into the wide pass's tail.  Every block of a pod group publishes its lists (its stores drained,
// the XCD L2 written back: the guide's release form) and takes a ticket; the block drawing the group's last ticket
// acquires and merges the group's pods into their records, one pod per wave (merge_pod, as the merge_wave kernel
// does), then resets the ticket for the slot's next round (stream order: that round's kernel starts after this one
// ends).  n_lists ≤ 2·kWave (the caller's condition).  A round poisoned mid-launch can leave a partial count: the
// batch is abandoned then, and every batch starts from zeroed tickets.
template <int LL>
__device__ __forceinline__ void merge_tail(const DevTable& T, const EvalParams& P, const uint64_t* __restrict__ lists,
                                           int n_lists, int p0, int p1, int ppw, int n_tg, uint32_t* __restrict__ tickets,
                                           uint64_t* __restrict__ records, uint64_t* s_lds) {
  __shared__ uint32_t s_last;
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t* t = tickets + p0 / ppw;
    const uint32_t old = __hip_atomic_fetch_add(t, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t last = old + 1 == (uint32_t)n_tg ? 1u : 0u;
    if (last) {
      __hip_atomic_store(t, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    s_last = last;
  }
  __syncthreads();
  if (!s_last) return;
  const int64_t pstride = (int64_t)n_lists * LL;
  uint64_t* sel = s_lds + (size_t)wave * kC;  // the block's list staging is free again: kEW·kC words (host-sized)
  for (int pl = wave; pl < p1 - p0; pl += kEW) {
    const uint64_t* base = lists + (size_t)(p0 + pl) * pstride;
    uint64_t* o = records + (size_t)(p0 + pl) * kCandStride;
    if (n_lists <= kWave) merge_pod<1, LL>(T, P, base, n_lists, sel, o, lane);
    else merge_pod<2, LL>(T, P, base, n_lists, sel, o, lane);
  }
}

// (r5) the fused merge tail (KG_FUSE=1 at run time) is compiled into eval_round only with -DKG_FUSE_TAIL=1: measured
// slower (fused_merge below), and its merge code raised the wide pass's scalar-register pressure
#ifndef KG_FUSE_TAIL
#define KG_FUSE_TAIL 0
#endif
// 4 waves per SIMD for the 2-node shape: all of the C3 grid (3,136 waves) resident at once (KG_EVAL_WPE=0: the
// compiler's choice, 130 VGPRs and 3 waves per SIMD)
#ifndef KG_EVAL_WPE
#define KG_EVAL_WPE (KG_EVAL_NPT == 2 ? 4 : 0)
#endif
#if KG_EVAL_WPE > 0
#define KG_EVAL_ATTR __attribute__((amdgpu_waves_per_eu(KG_EVAL_WPE)))
#else
#define KG_EVAL_ATTR
#endif
template <int PF, bool AUX>
__global__ __launch_bounds__(kWave* kEW) KG_EVAL_ATTR void eval_round(DevTable T, const DevPod* __restrict__ pods,
                                                                  int64_t first, int nb, int pods_per_wave,
                                                                  int64_t node_base, int64_t n_local, int nt_local,
                                                                  EvalParams P, uint64_t* __restrict__ lists,
                                                                  const int32_t* __restrict__ poison,
                                                                  const int64_t* __restrict__ paux, int combine,
                                                                  uint32_t* __restrict__ tickets,
                                                                  uint64_t* __restrict__ records) {
  KG_STAMP(0, 0);
  if (*poison) return;
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  // XCD-aware swizzle (bijective for any grid size): the blocks of one tile group — one per pod group — get
  // consecutive ids on the same XCD label, so the group's node rows come from HBM once and from that XCD's
  // L2 for the other pod groups (the straight grid spread them over all 8 L2s: ~12x the table per launch).
  const int n_pg = (nb + pods_per_wave - 1) / pods_per_wave;
  const uint32_t nwg = gridDim.x, bid = blockIdx.x, xcd = bid % 8u, q = nwg / 8u, r = nwg % 8u;
  const uint32_t wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8u;
  const int tile0 = (int)(wgid / (uint32_t)n_pg) * kEW, tile = tile0 + wave;
  const int p0 = (int)(wgid % (uint32_t)n_pg) * pods_per_wave;
  if (tile0 >= nt_local || p0 >= nb) return;  // block-uniform
  const int p1 = (p0 + pods_per_wave) < nb ? (p0 + pods_per_wave) : nb;
  const int vbits = P.score_bits + 1;  // v = total + 1 ≤ 2^score_bits
  // (r4) each wave's per-pod tile top-kR goes to LDS; the block then combines its kEW tiles into one
  // top-kR list per (pod, tile group) — a quarter of the candidate lists for the merge to read and rank
  // (a shard of fewer than kCombineTiles tiles keeps one list per tile: a pod's record needs kC candidates)
  extern __shared__ __attribute__((aligned(16))) uint64_t s_lists[];  // [kEW][pods_per_wave][kR]
  const int ng_local = (nt_local + kEW - 1) / kEW, grp = tile0 / kEW;
  if (!combine) {
    if (tile < nt_local)
      eval_tile<PF, kENPT, AUX>(T, pods, first, p0, p1, tile, node_base, n_local, P, lists + ((size_t)p0 * nt_local + tile) * kR,
                    (int64_t)nt_local * kR, vbits, paux, lane);
#if KG_FUSE_TAIL
    if (tickets) merge_tail<kR>(T, P, lists, nt_local, p0, p1, pods_per_wave, ng_local, tickets, records, s_lists);
#endif
    return;
  }
  uint64_t* my_l = s_lists + (size_t)wave * pods_per_wave * kR;
  if (tile < nt_local) eval_tile<PF, kENPT, AUX>(T, pods, first, p0, p1, tile, node_base, n_local, P, my_l, kR, vbits, paux, lane);
  else
    for (int q = lane; q < (p1 - p0) * kR; q += kWave) my_l[q] = 0;
  __syncthreads();
  // group list = the kR largest of the block's kEW·kR keys, in descending key order (within one score:
  // ascending node index, as the merge's tie rule reads lists); a full group list's minimum bounds every key the
  // block left out, as a full tile list's did (a full tile list's kR keys are all in the union)
  static_assert(kEW * kR <= kWave, "one key per lane");
  for (int pl = wave; pl < p1 - p0; pl += kEW) {
    const uint64_t key = lane < kEW * kR ? s_lists[((size_t)(lane / kR) * pods_per_wave + pl) * kR + lane % kR] : 0;
    int rank = 0;
#pragma unroll
    for (int w = 0; w < kEW; ++w) {
      const ulonglong2* l2 = reinterpret_cast<const ulonglong2*>(s_lists + ((size_t)w * pods_per_wave + pl) * kR);
#pragma unroll
      for (int q = 0; q < kR / 2; ++q) {
        const ulonglong2 x = l2[q];  // broadcast LDS reads
        rank += (x.x > key) + (x.y > key);
      }
    }
    const int nnz = __popcll(__ballot(key != 0));
    uint64_t* out = lists + ((size_t)(p0 + pl) * ng_local + grp) * kRG;  // the kRG best (a full list still bounds)
    if (key != 0 && rank < kRG) out[rank] = key;
    if (lane >= nnz && lane < kRG) out[lane] = 0;
  }
#if KG_FUSE_TAIL
  if (tickets) merge_tail<kRG>(T, P, lists, ng_local, p0, p1, pods_per_wave, ng_local, tickets, records, s_lists);
#endif
  KG_STAMP(0, 31);
}

// ---- round kernel 2: per-pod merge ------------------------------------------------------------------
// One block per pod of the round: the kC largest keys of the union of the pod's candidate lists, sorted
// descending (0-padded), plus a STRICT upper bound `ub` on every key left out (0 = nothing left out):
//   ub = max(max_l ub_l, largest key left out + 1), where a tile list's ub_l is its minimum when it is full
//   (its unseen nodes all score lower) and a rank list carries its own ub in slot kC.
// Selection: keys are unique (score << 32 | ~idx) and the lists, read in order, enumerate nodes in ascending
// index within each score (tile lists: ascending node order; rank lists: descending keys of contiguous shards).
// So the top kC = every key with score > τ plus the first `need` keys with score == τ in list order, where τ
// is the largest score with count(score ≥ τ) ≥ kC: one LDS histogram of the scores (score_bits ≤ kHistBits)
// and two block scans.  Wider score ranges use an 8-bit radix select over the whole key.
// The record also carries the hoisted rows of the kStaged best candidates, read from this rank's replica of
// the node table, so that the resolver never waits on HBM for a likely winner.
constexpr int kHistBits = 10;

__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* red, int lane, int wave, uint32_t& total) {
  const uint32_t incl = wave_prefix_sum_u32(v);
  if (lane == kWave - 1) red[wave] = incl;
  __syncthreads();
  uint32_t off = incl - v, tot = 0;
#pragma unroll
  for (int w = 0; w < kMergeThreads / kWave; ++w) {
    off += w < wave ? red[w] : 0u;
    tot += red[w];
  }
  __syncthreads();
  total = tot;
  return off;
}

template <bool RANK_LISTS>
__global__ __launch_bounds__(kMergeThreads) void merge_round(DevTable T, EvalParams P,
                                                             const uint64_t* __restrict__ in, int64_t pod_stride,
                                                             int64_t list_stride, int n_lists, int list_len,
                                                             int nb, const int32_t* __restrict__ poison,
                                                             uint64_t* __restrict__ out) {
  __shared__ uint32_t hist[1 << kHistBits];
  __shared__ __attribute__((aligned(16))) uint64_t sel[kC];
  __shared__ uint64_t red64[kMergeThreads / kWave];
  __shared__ uint32_t red32[kMergeThreads / kWave];
  __shared__ uint64_t sh_prefix;
  __shared__ uint32_t sh_target;
  KG_STAMP(1, 0);
  const int pod = blockIdx.x;
  const int tid = threadIdx.x, lane = tid % kWave, wave = tid / kWave;
  if (*poison || pod >= nb) return;
  const uint64_t* base = in + (size_t)pod * pod_stride;

  // Keys held in registers: thread t owns chunks c = t + kMergeThreads*i of 8 consecutive keys (chunk order
  // = list order = ascending node index within a score).
  const int chunks_per_list = list_len / 8;
  const int n_chunks = n_lists * chunks_per_list;
  uint64_t k[kMergeChunks][8];
  uint64_t ub_in = 0, kmax = 0;
  uint32_t nz = 0;
#pragma unroll
  for (int i = 0; i < kMergeChunks; ++i) {
    const int c = tid + kMergeThreads * i;
    if (c < n_chunks) {
      const int l = c / chunks_per_list, part = c - l * chunks_per_list;
      const uint64_t* src = base + (size_t)l * list_stride + part * 8;
#pragma unroll
      for (int r = 0; r < 8; r += 2) {
        const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(src + r);
        k[i][r] = v.x;
        k[i][r + 1] = v.y;
      }
      if (RANK_LISTS) {
        if (part == 0) {
          const uint64_t u = base[(size_t)l * list_stride + kC];
          ub_in = u > ub_in ? u : ub_in;
        }
      } else {
        uint64_t mn = ~0ull;
        int cnt = 0;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          cnt += k[i][r] != 0;
          mn = (k[i][r] && k[i][r] < mn) ? k[i][r] : mn;
        }
        if (cnt == 8) ub_in = mn > ub_in ? mn : ub_in;  // full tile list: unseen nodes < its minimum
      }
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        nz += k[i][r] != 0;
        kmax = k[i][r] > kmax ? k[i][r] : kmax;
      }
    } else {
#pragma unroll
      for (int r = 0; r < 8; ++r) k[i][r] = 0;
    }
  }
  const bool hist_path = P.score_bits <= kHistBits;
  if (hist_path)
    for (int b = tid; b < (1 << kHistBits); b += kMergeThreads) hist[b] = 0;
  KG_STAMP(1, 1);
  // block reductions: Σ nz, max ub_in, max kmax
  {
    const uint32_t s = wave_sum_u32(nz);
    const uint64_t u = wave_max_key(ub_in), m = wave_max_key(kmax);
    if (lane == 0) {
      red32[wave] = s;
      red64[wave] = u;
      sel[wave] = m;
    }
    __syncthreads();
    uint32_t tot = 0;
    uint64_t ubm = 0, km = 0;
    for (int w = 0; w < kMergeThreads / kWave; ++w) {
      tot += red32[w];
      ubm = red64[w] > ubm ? red64[w] : ubm;
      km = sel[w] > km ? sel[w] : km;
    }
    nz = tot;
    ub_in = ubm;
    kmax = km;
    __syncthreads();
  }
  KG_STAMP(1, 2);

  // selection predicate: key ≥ kth, and for the histogram path score > tau || (score == tau && tie rank < need)
  uint64_t kth = 1;  // select every non-zero key when there are at most kC of them
  uint32_t tau = 0, need = 0;
  bool use_tau = false;
  if (nz > (uint32_t)kC && hist_path) {
#pragma unroll
    for (int i = 0; i < kMergeChunks; ++i)
#pragma unroll
      for (int r = 0; r < 8; ++r)
        if (k[i][r]) atomicAdd(&hist[(uint32_t)(k[i][r] >> 32)], 1u);
    __syncthreads();
    if (wave == 0) {
      // lane l holds bins top-16l .. top-16l-15 (descending); τ = the bin where the count from the top reaches kC
      constexpr int kPer = (1 << kHistBits) / kWave;
      uint32_t b[kPer], s = 0;
#pragma unroll
      for (int q = 0; q < kPer; ++q) {
        b[q] = hist[(1 << kHistBits) - 1 - kPer * lane - q];
        s += b[q];
      }
      uint32_t above = wave_prefix_sum_u32(s) - s;
#pragma unroll
      for (int q = 0; q < kPer; ++q) {
        if (above < (uint32_t)kC && above + b[q] >= (uint32_t)kC) {
          sh_prefix = (uint64_t)((1 << kHistBits) - 1 - kPer * lane - q);
          sh_target = (uint32_t)kC - above;  // keys needed from the τ bin
        }
        above += b[q];
      }
    }
    __syncthreads();
    tau = (uint32_t)sh_prefix;
    need = sh_target;
    use_tau = true;
    KG_STAMP(1, 3);
  } else if (nz > (uint32_t)kC) {
    int top = 7;
    while (top > 0 && ((kmax >> (8 * top)) & 0xFF) == 0) --top;  // bytes above kmax's leading byte are 0
    uint64_t prefix = 0, pmask = 0;
    uint32_t target = kC;
    for (int byte = top; byte >= 0; --byte) {
      const int shift = 8 * byte;
      hist[tid] = 0;  // kMergeThreads == 256 bins
      __syncthreads();
#pragma unroll
      for (int i = 0; i < kMergeChunks; ++i)
#pragma unroll
        for (int r = 0; r < 8; ++r)
          if (k[i][r] && (k[i][r] & pmask) == prefix) atomicAdd(&hist[(k[i][r] >> shift) & 0xFF], 1u);
      __syncthreads();
      if (wave == 0) {
        // lane l holds digits 255-4l .. 252-4l (descending); keys with a higher digit sit in lanes < l
        uint32_t b[4], s = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          b[q] = hist[255 - 4 * lane - q];
          s += b[q];
        }
        uint32_t above = wave_prefix_sum_u32(s) - s;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (above < target && above + b[q] >= target) {
            sh_prefix = prefix | ((uint64_t)(255 - 4 * lane - q) << shift);
            sh_target = target - above;
          }
          above += b[q];
        }
      }
      __syncthreads();
      prefix = sh_prefix;
      target = sh_target;
      pmask |= 0xFFull << shift;
    }
    kth = prefix;
  }
  // tie ranks at τ in list order (chunk c = t + 256·i: i-major, then thread), 16-bit fields per chunk pair
  uint32_t tie_base[kMergeChunks] = {0, 0, 0, 0};
  if (use_tau) {
    uint32_t c01 = 0, c23 = 0;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      c01 += ((k[0][r] >> 32) == tau && k[0][r]) + (((k[1][r] >> 32) == tau && k[1][r]) << 16);
      c23 += ((k[2][r] >> 32) == tau && k[2][r]) + (((k[3][r] >> 32) == tau && k[3][r]) << 16);
    }
    uint32_t t01, t23;
    const uint32_t o01 = block_excl_scan(c01, red32, lane, wave, t01);
    const uint32_t o23 = block_excl_scan(c23, red32, lane, wave, t23);
    const uint32_t T0 = t01 & 0xFFFF, T1 = t01 >> 16, T2 = t23 & 0xFFFF;
    tie_base[0] = o01 & 0xFFFF;
    tie_base[1] = T0 + (o01 >> 16);
    tie_base[2] = T0 + T1 + (o23 & 0xFFFF);
    tie_base[3] = T0 + T1 + T2 + (o23 >> 16);
  }
  // selection + compaction + the best key left out
  uint32_t mycnt = 0;
  uint64_t next = 0;
  uint32_t selmask[kMergeChunks];
#pragma unroll
  for (int i = 0; i < kMergeChunks; ++i) {
    uint32_t m = 0, tr = tie_base[i];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const uint64_t v = k[i][r];
      bool s;
      if (use_tau) {
        const uint32_t sc = (uint32_t)(v >> 32);
        const bool tie = v && sc == tau;
        s = v && (sc > tau || (tie && tr < need));
        tr += tie;
      } else {
        s = v && v >= kth;
      }
      m |= (uint32_t)s << r;
      if (v && !s) next = v > next ? v : next;
    }
    selmask[i] = m;
    mycnt += __popc(m);
  }
  uint32_t n_sel;
  uint32_t off = block_excl_scan(mycnt, red32, lane, wave, n_sel);
  next = wave_max_key(next);
  if (lane == 0) red64[wave] = next;
  if (tid < kC) sel[tid] = 0;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kMergeChunks; ++i)
#pragma unroll
    for (int r = 0; r < 8; ++r)
      if ((selmask[i] >> r) & 1) sel[off++] = k[i][r];
  __syncthreads();
  KG_STAMP(1, 13);
  uint64_t* o = out + (size_t)pod * kCandStride;
  if (wave == 0) {
    uint64_t nx = 0;
    for (int w = 0; w < kMergeThreads / kWave; ++w) nx = red64[w] > nx ? red64[w] : nx;
    // rank sort of the ≤ kC selected keys (unique): position = number of larger keys
    const uint64_t v = sel[lane];
    int rank = 0;
    const ulonglong2* s2 = reinterpret_cast<const ulonglong2*>(sel);
#pragma unroll
    for (int q = 0; q < kC / 2; ++q) {
      const ulonglong2 x = s2[q];  // broadcast LDS reads, all issued back to back
      rank += (x.x > v) + (x.y > v);
    }
    if (lane < (int)n_sel) o[rank] = v;
    else o[lane] = 0;  // positions ≥ n_sel
    if (lane == 0) {
      const uint64_t ub_sel = nx ? nx + 1 : 0;
      o[kC] = ub_in > ub_sel ? ub_in : ub_sel;
    }
    // hoisted rows of the kStaged best candidates (the resolver's likely winners)
    // (DeviceShare rounds merge all B pod slots, the ones past the round's pods holding stale lists: a node index
    // outside the table is never dereferenced)
    if (lane < (int)n_sel && rank < kStaged && key_node(v) < (uint32_t)T.cap) {
      const EvalRow er = make_eval_row(load_row(T, key_node(v)), P);
      uint64_t words[kEvalRowWords];
      __builtin_memcpy(words, &er, sizeof(er));  // well-defined type punning (no strict-aliasing hazard)
      uint64_t* dst = o + kRecRows + rank * kEvalRowWords;
#pragma unroll
      for (int w = 0; w < kEvalRowWords; ++w) dst[w] = words[w];
    }
  }
  KG_STAMP(1, 14);
}

// ---- (r4) round kernel 2b: per-pod merge on one wavefront (eval_round's tile-group lists) ---------------------
// The same record as merge_round<false> (kC largest keys sorted, strict bound ub, the kStaged best rows), with no block
// barrier: lane l holds lists l, l + 64, … (L per lane, ≤ 64·L lists; tile lists or tile-group lists) in registers.
//  * ub_in = max over full lists of their minimum; every key below it is useless to the resolver, which stops once
//    its best candidate falls below ub ≥ ub_in, so those keys are dropped before the selection.
//  * τ = the largest score with count(score ≥ τ) ≥ kC (a ballot-sum binary search over the score bits), the first
//    `need` keys of score τ in list order (lists by index, then position: ascending node index, as for tile lists) —
//    i.e. the kC largest keys.
//  * compaction into LDS by a wave prefix sum, a rank sort of ≤ kC keys, then the staged rows.
__device__ __forceinline__ uint32_t wave_excl_prefix_u32(uint32_t v) { return wave_prefix_sum_u32(v) - v; }

// One pod's record from its n_lists candidate lists at base (list l at base + l·kR), by one wavefront; sel = kC words of
// this wave's LDS, o = the record.  Shared by merge_wave and (r5) eval_round's fused tail (opt-in).
// (r5) Per-step costs measured in-kernel at C3 size (KG_STAMPS, profiles/r05/stamps_merge*.txt) drove the layout: the
// staged rows of the 3 best keys are requested first (a knock-out wave max), so their HBM latency overlaps the
// selection instead of ending the kernel; the threshold τ is a bisection over the live score range with ballot
// popcounts (no DPP sums); the rank sort reads the zero-padded selection with all its broadcast loads in flight.
__device__ __forceinline__ uint32_t ballot_count(bool c) { return (uint32_t)__popcll(__ballot(c)); }

template <int L, int LL>
__device__ __forceinline__ void merge_pod(const DevTable& T, const EvalParams& P, const uint64_t* __restrict__ base,
                                          int n_lists, uint64_t* sel, uint64_t* __restrict__ o, int lane) {
  uint64_t k[L][LL];
  uint64_t ub_in = 0;
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const int l = lane + kWave * i;
    if (l < n_lists) {
      const ulonglong2* src = reinterpret_cast<const ulonglong2*>(base + (size_t)l * LL);
#pragma unroll
      for (int r = 0; r < LL / 2; ++r) {
        const ulonglong2 v = src[r];
        k[i][2 * r] = v.x;
        k[i][2 * r + 1] = v.y;
      }
    } else {
#pragma unroll
      for (int r = 0; r < LL; ++r) k[i][r] = 0;
    }
    // a full list (LL keys: a tile list in node order, or a sorted tile-group list) bounds its unseen nodes by its
    // minimum
    uint64_t mn = ~0ull;
    int cnt = 0;
#pragma unroll
    for (int r = 0; r < LL; ++r) {
      cnt += k[i][r] != 0;
      mn = k[i][r] != 0 && k[i][r] < mn ? k[i][r] : mn;
    }
    if (cnt == LL) ub_in = mn > ub_in ? mn : ub_in;
  }
  ub_in = wave_max_key(ub_in);
  KG_STAMP(1, 1);
  // keys below ub_in can never be listed (ub_in bounds them already); the 3 best keys' rows go out to HBM now
  uint64_t top[kStaged];
  {
    uint64_t bound = ~0ull;
#pragma unroll
    for (int q = 0; q < kStaged; ++q) {
      uint64_t m = 0;
#pragma unroll
      for (int i = 0; i < L; ++i)
#pragma unroll
        for (int r = 0; r < LL; ++r) {
          if (q == 0 && k[i][r] < ub_in) k[i][r] = 0;
          m = k[i][r] < bound && k[i][r] > m ? k[i][r] : m;
        }
      top[q] = wave_max_key(m);
      bound = top[q] ? top[q] : 1;  // 1: nothing below an empty maximum (every later top is 0)
    }
  }
  const uint64_t my_top = lane == 0 ? top[0] : lane == 1 ? top[1] : top[2];
  const bool stage = lane < kStaged && my_top != 0 && key_node(my_top) < (uint32_t)T.cap;
  Row srow;
  if (stage) srow = load_row(T, key_node(my_top));  // consumed at the end: its latency overlaps the selection
  uint32_t sc[L][LL];  // score + 1 of a live key, 0 for a dropped one
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < L; ++i)
#pragma unroll
    for (int r = 0; r < LL; ++r) {
      sc[i][r] = k[i][r] ? (uint32_t)(k[i][r] >> 32) + 1u : 0u;
      c += k[i][r] != 0;
    }
  const uint32_t total = wave_sum_u32(c);
  const bool all = total <= (uint32_t)kC;
  uint32_t tau = 0, need = kC;
  if (!all) {
    // τ = the largest t with count(sc ≥ t) ≥ kC, bisected over (lo, hi]: count(sc ≥ lo) = total ≥ kC holds at lo = 1,
    // and no key reaches the best key's score + 2
    uint32_t lo = 1, hi = (uint32_t)(top[0] >> 32) + 2;
    while (hi - lo > 1) {
      const uint32_t mid = lo + (hi - lo) / 2;
      uint32_t n = 0;
#pragma unroll
      for (int i = 0; i < L; ++i)
#pragma unroll
        for (int r = 0; r < LL; ++r) n += ballot_count(sc[i][r] >= mid);
      if (n >= (uint32_t)kC) lo = mid;
      else hi = mid;
    }
    tau = lo;
    uint32_t a = 0;
#pragma unroll
    for (int i = 0; i < L; ++i)
#pragma unroll
      for (int r = 0; r < LL; ++r) a += ballot_count(sc[i][r] > tau);
    need = (uint32_t)kC - a;
  }
  KG_STAMP(1, 2);
  // selection with tie ranks in list order (i-major, then lane, then position) and the best key left out
  uint32_t tie_base = 0, mycnt = 0;
  uint64_t next = 0;
  uint32_t selm[L];
#pragma unroll
  for (int i = 0; i < L; ++i) {
    uint32_t ties = 0;
    if (!all) {
#pragma unroll
      for (int r = 0; r < LL; ++r) ties += sc[i][r] == tau;
    }
    uint32_t tr = tie_base + wave_excl_prefix_u32(ties);
    tie_base += wave_sum_u32(ties);
    uint32_t m = 0;
#pragma unroll
    for (int r = 0; r < LL; ++r) {
      const uint64_t v = k[i][r];
      const bool tie = !all && sc[i][r] == tau;
      const bool sl = sc[i][r] != 0 && (all || sc[i][r] > tau || (tie && tr < need));
      tr += tie;
      m |= (uint32_t)sl << r;
      if (v != 0 && !sl) next = v > next ? v : next;
    }
    selm[i] = m;
    mycnt += __popc(m);
  }
  const uint32_t n_sel = wave_sum_u32(mycnt);
  uint32_t off = wave_excl_prefix_u32(mycnt);
  next = wave_max_key(next);
#pragma unroll
  for (int i = 0; i < L; ++i)
#pragma unroll
    for (int r = 0; r < LL; ++r)
      if ((selm[i] >> r) & 1u) sel[off++] = k[i][r];
  if (lane >= (int)n_sel) sel[lane] = 0;  // zero padding: the rank sort reads all kC slots
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  KG_STAMP(1, 13);
  // rank sort of the ≤ kC selected keys (unique, 0-padded): position = number of larger keys
  const uint64_t v = sel[lane];
  int rank = 0;
  const ulonglong2* s2 = reinterpret_cast<const ulonglong2*>(sel);
#pragma unroll
  for (int q = 0; q < kC / 2; ++q) {
    const ulonglong2 x = s2[q];  // broadcast LDS reads
    rank += (x.x > v) + (x.y > v);
  }
  o[lane < (int)n_sel ? rank : lane] = lane < (int)n_sel ? v : 0;
  if (lane == 0) {
    const uint64_t ub_sel = next ? next + 1 : 0;
    o[kC] = ub_in > ub_sel ? ub_in : ub_sel;
  }
  if (stage) {  // lane q holds the q-th best key's row: rank q of the record
    const EvalRow er = make_eval_row(srow, P);
    uint64_t words[kEvalRowWords];
    __builtin_memcpy(words, &er, sizeof(er));
    uint64_t* dst = o + kRecRows + lane * kEvalRowWords;
#pragma unroll
    for (int w = 0; w < kEvalRowWords; ++w) dst[w] = words[w];
  }
  KG_STAMP(1, 14);
}

template <int L, int LL>
__global__ __launch_bounds__(kWave * 4) void merge_wave(DevTable T, EvalParams P, const uint64_t* __restrict__ in,
                                                        int64_t pod_stride, int n_lists, int nb,
                                                        const int32_t* __restrict__ poison,
                                                        uint64_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint64_t s_sel[4][kC];
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int pod = blockIdx.x * 4 + wave;
  if (*poison || pod >= nb) return;  // no block barrier below: a wave may leave alone
  KG_STAMP(1, 0);
  merge_pod<L, LL>(T, P, in + (size_t)pod * pod_stride, n_lists, s_sel[wave], out + (size_t)pod * kCandStride, lane);
}

// ---- round kernel 3: FIFO resolve (one wavefront, modified rows in registers) ---------------------------
// One wavefront replays the round's pods [first, first + nb) in queue order against the merged candidates.
// The "modified set" of pod j = every node assumed by an earlier pod of this round or by the n_prev rounds before
// it that were still resolving when this round was evaluated (pipelining depth D: this round's eval read the table
// right after resolve(r - D), so rows of rounds r-D+1 .. r-1 may have been read mid-update).  Modified rows live
// in registers: slot s = bank·64 + lane holds node m[bank] as a hoisted EvalRow kept current by assume_on (two
// banks: ≤ 128 rows).  Per pod j, for a monotone profile (Fit, LoadAware: an assume only lowers a node's key; a
// row read as a mix of pre- and post-assume columns reads ≥ its current key):
//   e     = the best listed candidate not modified (its key is exact);
//   mbest = the exact re-score of every modified row — skipped when e is the pod's top candidate (every modified
//           node then reads ≤ its listed key < e);
//   best  = max(e, mbest) is the sequential answer when best ≥ ub (every unlisted node's key < ub).  Otherwise an
//           unseen node could still win: the round ends before pod j and sets `poison` (the rest of the batch,
//           evaluated for later pods, is skipped until the host restarts from the cursor).
// The next pod's candidate keys, pod record and modified-bitmap word are prefetched while pod j resolves (the
// prefetched word is patched with pod j's winner).  Rows of earlier rounds are loaded once, after the chain wait;
// a node listed by two earlier rounds keeps its first slot (LDS hash), the duplicate becomes an infeasible hole.
// Writes out_keys[first + j] (0 = unschedulable), the touched rows back to the table and into this round's
// modified-row list (modlists[slot]), and advances the cursor ctl[0].
constexpr int kMaxDepth = 4;          // pipelined rounds in flight (streams)
constexpr int kMaxMod = 2 * kWave;    // modified-row slots: two register banks
constexpr int kModHash = 512;         // node → slot hash for de-duplicating earlier rounds' lists
constexpr int kModListStride = 1 + kMaxB;  // [count, node ids...] per round slot

__device__ __forceinline__ uint32_t mod_hash(uint32_t node) { return (node * 2654435761u) >> (32 - 9); }
static_assert(kModHash == 512, "hash width");

// insert node → slot; returns the slot already holding node when present
__device__ __forceinline__ int mod_insert(uint32_t* h, uint32_t node, int slot) {
  const uint32_t v = ((node + 1u) << 8) | (uint32_t)slot;
  uint32_t i = mod_hash(node);
  for (int it = 0; it < kModHash; ++it) {
    const uint32_t prev = atomicCAS(&h[i], 0u, v);
    if (prev == 0u) return slot;
    if ((prev >> 8) == node + 1u) return (int)(prev & 0xFFu);
    i = (i + 1u) & (kModHash - 1);
  }
  return -1;
}

// End of a resolver: every store of this wave visible device-wide, then ctl[4] = seq (agent-scope release) for
// the next round's resolver, which may already be resident on another round stream.
// (r5) Release only (the guide's producer form): this wave's stores drained, the XCD L2 written back, the wait after
// the write-back kept by inline asm (the compiler may drop it), then a relaxed flag store.  The acq_rel
// __threadfence() it replaces also invalidated the L2 — a cost on the serial chain that nothing after it needs.
__device__ __forceinline__ void publish_round(int64_t* ctl, int64_t seq) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (threadIdx.x == 0) __hip_atomic_store(&ctl[4], seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// exact key of one modified row for pod p (0 = filtered out).  A row outside eval_fast's domain takes the
// reference-shaped eval_node with the EvalParams copy in LDS behind an opaque pointer: its runtime weight / flag
// tests then stay inside the (rare) branch instead of being hoisted as loop-invariant scalar masks that crowd the
// resolver's scalar registers.
constexpr int kParWords = (int)((sizeof(EvalParams) + 7) / 8);
template <int PF>
__device__ __forceinline__ uint64_t mod_key(const EvalRow& er, uint32_t node, const DevPod& p, const EvalParams& P,
                                            const uint64_t* s_par) {
  uint32_t t = 0;
  bool rare = false;
  bool ok = eval_fast<PF>(er, p, P, t, rare);
  if (rare) {
    const uint64_t* q = s_par;
    asm volatile("" : "+v"(q));
    EvalParams Pr;
    __builtin_memcpy(&Pr, q, sizeof(Pr));
    int64_t t64 = 0;
    ok = eval_node(row_of(er), p, Pr, t64);
    t = (uint32_t)t64;
  }
  return ok ? make_key(t, node) : 0;
}

__device__ __forceinline__ EvalRow lds_row(const uint64_t* src) {
  uint64_t w[kEvalRowWords];
#pragma unroll
  for (int q = 0; q < kEvalRowWords; ++q) w[q] = src[q];
  EvalRow er;
  __builtin_memcpy(&er, w, sizeof(er));
  return er;
}

// One modified row held by a lane: its node and hoisted terms, kept current by assume_mod on every placement (the
// owner lane only).  A node that wins while unmodified takes a new slot lazily: `pend` = (j << 8) | pos records the
// placing pod j and the winner's position in pod j's record, and the row is brought in (shipped record row, or HBM
// beyond the staged rows) and assumed only when a later pod has to re-score the modified rows — all pending lanes
// at once (mod_row_settle).  The table write-back happens once per round, per placed pod (epilogue atomics).
constexpr uint32_t kNoNode = 0xFFFFFFFFu;
struct ModRow {
  uint32_t node;
  int32_t pend;  // -1: er is current
  EvalRow er;
};
__device__ __forceinline__ void mod_row_init(ModRow& m) {
  m.node = kNoNode;
  m.pend = -1;
  m.er.flags = 0;
}
template <int PF>
__device__ __forceinline__ uint64_t mod_row_key(const ModRow& m, const DevPod& p, const EvalParams& P,
                                                const uint64_t* s_par) {
  return m.node == kNoNode ? 0 : mod_key<PF>(m.er, m.node, p, P, s_par);
}

// assume(pod) on a modified row (NodeInfo.AddPod + LoadAware Reserve → podAssignCache.assign): only the free terms
// move, and only downwards, so eval_fast's exact domain can be left only through the lower bounds of the free terms
// the profile scores (the same test as rare_bit's, without its capacity compares or f64 → int64 conversions).
template <int PF>
__device__ __forceinline__ void assume_mod(EvalRow& e, const DevPod& p, const EvalParams& P) {
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
  bool out = false;
  // (whatever the weights: F_RARE only sends the row to the exact path, so marking it for a zero-weight term is safe)
  if constexpr ((PF & PF_FIT_SCORE) != 0) out |= (e.fnz_cpu < kCpuFreeMin) | !(e.fnz_mem > (double)kMemFreeMin);
  if constexpr ((PF & PF_LA_SCORE) != 0) {
    if (e.flags & F_LA_SCORE)
      out |= (e.la_free_cpu < kCpuFreeMin) | (e.la_pfree_cpu < kCpuFreeMin) | !(e.la_free_mem > (double)kMemFreeMin) |
             !(e.la_pfree_mem > (double)kMemFreeMin);
  }
  if (out) e.flags |= F_RARE;
}

// wave max of packed keys: one 32-bit DPP max when (score, node) fit 13 + 19 bits, else the two-word form
__device__ __forceinline__ uint64_t wave_max_modkey(uint64_t k, bool narrow) {
  if (narrow) {
    const uint32_t k32 = k ? (uint32_t)((k >> 32) << 19) | (0x7FFFFu - key_node(k)) : 0u;
    const uint32_t m = wave_max_u32(k32);
    return m ? make_key((int64_t)(m >> 19), 0x7FFFFu - (m & 0x7FFFFu)) : 0;
  }
  return wave_max_key(k);
}

// Round write-back: lane j < consumed adds placed pod j's NodeInfo.AddPod + podAssignCache.assign terms onto its
// winner's columns (int64 atomics: several pods of the round may share a winner; no other writer — earlier rounds'
// resolvers are done, later ones wait for this one; concurrent wide passes read mixed columns).
__device__ __forceinline__ void writeback_pod(const DevTable& T, uint32_t node, const DevPod& p,
                                              const int64_t* __restrict__ rq) {
  const int64_t i = node;
  const int64_t prod = (p.flags & P_PROD) ? 1 : 0;
  auto add = [](int64_t* a, int64_t v) { atomicAdd(reinterpret_cast<unsigned long long*>(a), (unsigned long long)v); };
  add(&T.req_cpu[i], p.req_cpu);
  add(&T.req_mem[i], p.req_mem);
  add(&T.nz_cpu[i], p.nz_cpu);
  add(&T.nz_mem[i], p.nz_mem);
  add(&T.la_used_cpu[i], p.est_cpu);
  add(&T.la_used_mem[i], p.est_mem);
  if (prod) {
    add(&T.la_pused_cpu[i], p.est_cpu);
    add(&T.la_pused_mem[i], p.est_mem);
  }
  atomicAdd(&T.num_pods[i], 1);
  if (p.flags & P_AUX)
#pragma unroll
    for (int r = 0; r < kAux; ++r)
      if (rq[r]) add(&T.aux[(size_t)(kAux + r) * T.cap + i], rq[r]);
}

// fitsRequest over the kAux resources on a modified row: the round-start Requested (the table; this round's
// placements are written back only by the epilogue) plus every earlier placement of this round on that node
__device__ __forceinline__ bool mod_aux_fits(const DevTable& T, uint32_t node, const int64_t* __restrict__ rq, int j,
                                             uint64_t my_out, const DevPod* s_pods, const int64_t* __restrict__ prq) {
  int64_t add[kAux] = {0, 0, 0, 0, 0};
  for (int q = 0; q < j; ++q) {
    const uint64_t k = readlane_u64(my_out, q);
    if (k == 0 || !(s_pods[q].flags & P_AUX)) continue;
    if (key_node(k) == node)
#pragma unroll
      for (int r = 0; r < kAux; ++r) add[r] += prq[(size_t)q * kAux + r];
  }
  bool ok = true;
#pragma unroll
  for (int r = 0; r < kAux; ++r)
    if (rq[r] != 0)
      ok &= !(rq[r] > T.aux[(size_t)r * T.cap + node] - (T.aux[(size_t)(kAux + r) * T.cap + node] + add[r]));
  return ok;
}

// The node table's columns are carved from two allocations (kg_engine: cols64 = 12 int64 columns + inv_mem[2],
// cols32 = alloc_pods, num_pods, flags, inv_cpu[2]), so a DevTable is (c64, c32, cap).  The single-wave resolvers
// rebuild it where a column is touched: the bases pass through an opaque asm so the 19 derived column addresses are
// not kept live in scalar registers across the per-pod loop (they spilled, costing v_readlane on the serial chain).
__device__ __forceinline__ DevTable table_at(const DevTable& T0) {
  int64_t* c64 = T0.alloc_cpu;
  int32_t* c32 = T0.alloc_pods;
  int64_t cap = T0.cap;
  asm volatile("" : "+s"(c64), "+s"(c32), "+s"(cap));
  DevTable T;
  T.alloc_cpu = c64 + 0 * cap;
  T.alloc_mem = c64 + 1 * cap;
  T.req_cpu = c64 + 2 * cap;
  T.req_mem = c64 + 3 * cap;
  T.nz_cpu = c64 + 4 * cap;
  T.nz_mem = c64 + 5 * cap;
  T.la_alloc_cpu = c64 + 6 * cap;
  T.la_alloc_mem = c64 + 7 * cap;
  T.la_used_cpu = c64 + 8 * cap;
  T.la_used_mem = c64 + 9 * cap;
  T.la_pused_cpu = c64 + 10 * cap;
  T.la_pused_mem = c64 + 11 * cap;
  T.inv_mem = reinterpret_cast<double*>(c64 + 12 * cap);
  T.aux = c64 + 14 * cap;
  T.alloc_pods = c32 + 0 * cap;
  T.num_pods = c32 + 1 * cap;
  T.flags = reinterpret_cast<uint32_t*>(c32 + 2 * cap);
  T.inv_cpu = reinterpret_cast<float*>(c32 + 3 * cap);
  T.cap = cap;
  return T;
}

template <int PF>
__device__ __forceinline__ void mod_row_settle(ModRow& R, const uint64_t* s_cand, const DevPod* s_pods, const DevTable& T0,
                                               const EvalParams& P) {
  if (R.pend >= 0) {
    const int pj = R.pend >> 8, ppos = R.pend & 0xFF;
    if (ppos < kStaged) R.er = lds_row(s_cand + (size_t)pj * kCandStride + kRecRows + ppos * kEvalRowWords);
    else R.er = make_eval_row(load_row(table_at(T0), R.node), P);
    assume_mod<PF>(R.er, s_pods[pj], P);
    R.pend = -1;
  }
}

constexpr int kBank1Probe = 8;  // modified keys above e matched against bank 1 before re-scoring it

template <int PF, bool QUOTA>
__global__ __launch_bounds__(kWave) void resolve_round(DevTable T0, const DevPod* __restrict__ pods,
                                                        int64_t* __restrict__ ctl, int64_t first, int nb,
                                                        const uint64_t* __restrict__ cand, EvalParams P,
                                                        uint64_t* __restrict__ out_keys, int bitmap_words,
                                                        int32_t* __restrict__ modlists, int slot, int depth,
                                                        int n_prev, int32_t* __restrict__ poison, int64_t seq,
                                                        int wait, QuotaRow* __restrict__ quotas, int nq,
                                                        const int64_t* __restrict__ paux) {
  extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
  KG_STAMP(2, 0);
  const int lane = threadIdx.x;
  // the serial chain outranks the wide pass's waves when they share a SIMD
  __builtin_amdgcn_s_setprio(3);
  uint64_t* s_cand = smem;                                            // [nb][kCandStride]
  uint64_t* s_podw = s_cand + (size_t)nb * kCandStride;               // [nb] DevPod (kPodWords words)
  uint64_t* s_par = s_podw + (size_t)nb * kPodWords;                  // [kParWords] EvalParams (rare-path copy)
  uint32_t* s_hash = reinterpret_cast<uint32_t*>(s_par + kParWords);  // [kModHash]
  uint32_t* s_prevn = s_hash + kModHash;                              // [kMaxMod] earlier rounds' nodes
  uint32_t* bitmap = s_prevn + kMaxMod;                               // [bitmap_words]
  {
    uint64_t pw[kParWords] = {};
    __builtin_memcpy(pw, &P, sizeof(P));
#pragma unroll
    for (int q = 0; q < kParWords; ++q)
      if (lane == q) s_par[q] = pw[q];
  }
  {  // prologue, independent of the previous round: LDS-DMA of this round's records (merged on this stream)
     // + pods, bitmap / hash clears (16-B stores)
    const int n16 = nb * kCandStride / 2;
    for (int it = 0; it * kWave < n16; ++it) {
      const int idx = it * kWave + lane;
      if (idx < n16)
        __builtin_amdgcn_global_load_lds((global_cvoid_ptr)(cand + 2 * (size_t)idx),
                                         (lds_void_ptr)(s_cand + 2 * (size_t)it * kWave), 16, 0, 0);
    }
    const uint64_t* pw = reinterpret_cast<const uint64_t*>(pods + first);
    const int p16 = nb * kPodWords / 2;
    for (int it = 0; it * kWave < p16; ++it) {
      const int idx = it * kWave + lane;
      if (idx < p16)
        __builtin_amdgcn_global_load_lds((global_cvoid_ptr)(pw + 2 * (size_t)idx),
                                         (lds_void_ptr)(s_podw + 2 * (size_t)it * kWave), 16, 0, 0);
    }
    uint4* b4 = reinterpret_cast<uint4*>(bitmap);
    for (int w = lane; w < bitmap_words / 4; w += kWave) b4[w] = make_uint4(0, 0, 0, 0);
    for (int w = (bitmap_words / 4) * 4 + lane; w < bitmap_words; w += kWave) bitmap[w] = 0;
    uint4* h4 = reinterpret_cast<uint4*>(s_hash);
    for (int w = lane; w < kModHash / 4; w += kWave) h4[w] = make_uint4(0, 0, 0, 0);
  }
  // Chain on the previous round's resolver (another round stream): its rows, cursor, poison and modified-row
  // list are published with an agent-scope release of ctl[4] = its sequence number.  Bounded spin: a missing
  // predecessor reports an error instead of hanging the device.
  int timed_out = 0;
  if (wait) {
    if (lane == 0) {
      int64_t it = 0;
      while (__hip_atomic_load(&ctl[4], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < seq - 1) {
        __builtin_amdgcn_s_sleep(1);
        if (++it > kSpinLimit) {
          timed_out = 1;
          break;
        }
      }
    }
    timed_out = __builtin_amdgcn_readfirstlane(timed_out);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  KG_STAMP(2, 1);
  // the period decomposition's resolver time: from the predecessor's hand-off (modified-row loads included)
  const uint64_t t_active = __builtin_amdgcn_s_memrealtime();
  if (timed_out || *poison || ctl[0] != first) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the LDS-DMA lands before the wave retires
    if (lane == 0 && timed_out) ctl[5] = 1;
    publish_round(ctl, seq);
    return;
  }
  // rows the n_prev previous rounds modified: slots [0, nM) of the register banks (slot s: lane s % 64, bank s / 64)
  ModRow R0, R1;
  mod_row_init(R0);
  mod_row_init(R1);
  int nM = 0;
  for (int d = 1; d <= n_prev; ++d) {  // concatenate the lists in LDS, then slot s → lane s % 64, bank s / 64
    const int32_t* ml = modlists + (size_t)(((slot - d) % depth + depth) % depth) * kModListStride;
    const int c = ml[0];
    for (int t = lane; t < c; t += kWave) s_prevn[nM + t] = (uint32_t)ml[1 + t];
    nM += c;
  }
  __syncthreads();
  if (lane < nM) {
    const uint32_t node = s_prevn[lane];
    if (mod_insert(s_hash, node, lane) == lane) {
      R0.node = node;
      R0.er = make_eval_row(load_row(table_at(T0), node), P);
      atomicOr(&bitmap[node >> 5], 1u << (node & 31));
    }
  }
  if (kWave + lane < nM) {
    const uint32_t node = s_prevn[kWave + lane];
    if (mod_insert(s_hash, node, kWave + lane) == kWave + lane) {
      R1.node = node;
      R1.er = make_eval_row(load_row(table_at(T0), node), P);
      atomicOr(&bitmap[node >> 5], 1u << (node & 31));
    }
  }
  const bool narrow = P.score_bits <= 13;  // packed keys fit 32 bits (node < 2^19 = kMaxNodes)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // LDS-DMA of records and pods (+ the rows above)
  __syncthreads();
  // ElasticQuota table (QUOTA instantiation only), after the chain wait: the previous resolver's charges are visible
  DevQuota ql = QUOTA ? quota_load(quotas, nq, lane) : DevQuota{0, 0, 0, 0, 0, 0, 0, 0};
  KG_STAMP(2, 2);
  const DevPod* s_pods = reinterpret_cast<const DevPod*>(s_podw);
  uint64_t my_out = 0;
  int consumed = 0, n_slow = 0;
  uint32_t last_w = kNoNode;
  // software pipeline: pod j's key / ub / record and bitmap word are in registers when pod j starts; pod j+1's key
  // was loaded one pod earlier, so its bitmap word issues without waiting on LDS (it misses pod j's own winner,
  // which the next pod patches with last_w)
  uint64_t key = s_cand[lane];
  uint64_t ub = s_cand[kC];
  uint32_t word = bitmap[key ? key_node(key) >> 5 : 0u];
  uint64_t key_n = s_cand[(size_t)(nb > 1 ? 1 : 0) * kCandStride + lane];
  uint32_t diag = 0;
  (void)diag;  // read by the KG_STAMPS build only
  for (int j = 0; j < nb; ++j) {
    KG_POD_DIAG(j, diag);
    diag = 0;
    const int j1 = j + 1 < nb ? j + 1 : j, j2 = j + 2 < nb ? j + 2 : j1;
    const uint32_t word_n = bitmap[key_n ? key_node(key_n) >> 5 : 0u];
    const uint64_t ub_n = s_cand[(size_t)j1 * kCandStride + kC];
    const uint64_t key_nn = s_cand[(size_t)j2 * kCandStride + lane];
    // (r4) the pod from the LDS copy: a scalar load on the chain made every LDS wait wait for it.  (r5) Read only where
    // it is used — the slow path (and the assume that follows it) or the quota check: on the fast path (the listed
    // winner is unmodified) its 96-byte load and the wait for it sat in front of the ballot of every pod.
    DevPod p;
    if (QUOTA) p = s_pods[j];
    const uint32_t node = key_node(key);  // key 0 → node 0xFFFFFFFF: masked below
    const bool unmod = (key != 0) & !((word >> (node & 31)) & 1u) & (node != last_w);
    bool placed = false;
    uint32_t w = kNoNode;
    if (!QUOTA || quota_admit(ql, p)) {  // ElasticQuota PreFilter rejects: Unschedulable, no node search
      const uint64_t um = __ballot(unmod);
      const int pos = um ? (int)__builtin_ctzll(um) : kC;
      uint64_t best = um ? readlane_u64(key, pos) : 0;
      diag = (uint32_t)pos << 8;
      KG_POD_SUB(j, 0);
      bool from_mod = false;
      if (nM > 0 && pos > 0) {  // a modified node is listed above e: re-score the modified rows exactly
        if (!QUOTA) p = s_pods[j];
        ++n_slow;
        diag |= 1;
        const bool aux = (PF & PF_FIT_FILTER) && (p.flags & P_AUX);  // ephemeral-storage / scalar requests
        const int64_t* rq = paux + (size_t)(first + j) * kAux;
        mod_row_settle<PF>(R0, s_cand, s_pods, T0, P);
        if (lane == 0) KG_LANE_SUB(j, 0);
        uint64_t mk = mod_row_key<PF>(R0, p, P, s_par);
        if (lane == 0) KG_LANE_SUB(j, 1);
        if (aux && mk && !mod_aux_fits(table_at(T0), R0.node, rq, j, my_out, s_pods, paux + (size_t)first * kAux))
          mk = 0;
        // (r5) bank 1 only when one of its rows is listed above e: a modified row listed below e, or not listed, reads
        // at most its listed key / ub (monotone profile), so it cannot beat e (≥ ub).  The ≤ kBank1Probe modified
        // keys above e are matched against bank 1's nodes (past that, both banks as before).
        bool need1 = nM > kWave;
        if (need1 && pos <= kBank1Probe) {
          uint64_t hit = 0;
          for (int q = 0; q < pos; ++q) hit |= __ballot(R1.node == key_node(readlane_u64(key, q)));
          need1 = hit != 0;
        }
        if (need1) {
          mod_row_settle<PF>(R1, s_cand, s_pods, T0, P);
          uint64_t k1 = mod_row_key<PF>(R1, p, P, s_par);
          if (aux && k1 && !mod_aux_fits(table_at(T0), R1.node, rq, j, my_out, s_pods, paux + (size_t)first * kAux))
            k1 = 0;
          mk = k1 > mk ? k1 : mk;
        }
        if (lane == 0) KG_LANE_SUB(j, 2);
        const uint64_t mbest = wave_max_modkey(mk, narrow);
        if (lane == 0) KG_LANE_SUB(j, 3);
        from_mod = mbest > best;
        best = from_mod ? mbest : best;
      }
      if (best < ub) break;  // an unseen node could still win: leave this pod to the next round
      KG_POD_SUB(j, 1);
      my_out = lane == j ? best : my_out;
      if (best != 0) {  // 0: unschedulable (ub == 0: no feasible node anywhere)
        placed = true;
        w = key_node(best);
        // assume (NodeInfo.AddPod + LoadAware Reserve: podAssignCache.assign): onto the winner's settled row when it
        // is a modified node, else a new pending slot (e, at position pos of pod j's record)
        if (from_mod) {
          if (R0.node == w) assume_mod<PF>(R0.er, p, P);
          if (R1.node == w) assume_mod<PF>(R1.er, p, P);
        } else {
          diag |= 2;
          const int sl = nM++;
          const int pend = (j << 8) | pos;
          if (sl < kWave) {
            if (lane == sl) R0.node = w, R0.pend = pend;
          } else if (lane == sl - kWave) {
            R1.node = w, R1.pend = pend;
          }
          if (lane == (sl & (kWave - 1))) atomicOr(&bitmap[w >> 5], 1u << (w & 31));
        }
        KG_POD_SUB(j, 2);
      }
    } else {
      my_out = lane == j ? 0 : my_out;
    }
    if (QUOTA && placed) quota_charge(ql, p, lane);  // ElasticQuota Reserve
    ++consumed;
    last_w = w;
    key = key_n;
    key_n = key_nn;
    ub = ub_n;
    word = word_n;
  }
  KG_STAMP(2, 30);
  KG_POD_DIAG(consumed, diag);
  // write-back: each placed pod's terms onto its winner + this round's modified-row list (winners, duplicates
  // allowed: the next resolver's hash keeps one slot per node)
  const bool mine = lane < consumed && my_out != 0;
  const uint32_t my_node = mine ? key_node(my_out) : kNoNode;
  if (mine) writeback_pod(table_at(T0), my_node, s_pods[lane], paux + (size_t)(first + lane) * kAux);
  int32_t* my_mod = modlists + (size_t)slot * kModListStride;
  const uint64_t lane_lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const uint64_t bm = __ballot(mine);
  if (mine) my_mod[1 + __popcll(bm & lane_lt)] = (int32_t)my_node;
  if (lane < consumed) out_keys[first + lane] = my_out;
  if (QUOTA) quota_store(quotas, nq, lane, ql);
  if (lane == 0) {
    my_mod[0] = __popcll(bm);
    ctl[0] = first + consumed;
    ctl[1] += 1;
    ctl[2] += consumed;
    ctl[6] += n_slow;  // diagnostics: pods that re-scored modified rows
    if (consumed < nb) *poison = 1;
    ctl[8] += (int64_t)(__builtin_amdgcn_s_memrealtime() - t_active);
  }
  publish_round(ctl, seq);
  KG_STAMP(2, 31);
}

// ---- round kernel 3 (r4): FIFO resolve with look-ahead helper waves (monotone profiles) ----------------------
// One workgroup: the chain wave, a keeper wave and kHelpers helper waves.  resolve_round above did everything on one
// wave, so every pod's re-score of the modified rows (~190 VALU instructions at one instruction per 4 cycles) and its
// assume sat on the serial chain.  Here the chain only decides; the re-score moves to helpers that work kLag pods
// ahead, and the assume to the keeper:
//   helper(j), on the table after pods ≤ j − kLag (the winners the chain has published by then), scores pod j on
//   every modified row (lane = slot) and on its listed candidates, and hands the chain the kTop best keys T_j of
//   {listed candidates not modified by then} ∪ {modified rows}, each with where its row lives in LDS.
//   chain step j: S = the winners of pods j − kLag + 1 .. j − 1 (≤ kLag − 1 nodes, the only rows that can have
//   changed since helper(j)'s snapshot).  c* = the first entry of T_j not in S: every node outside S holds its
//   snapshot key, and T_j is the top of those, so c* is their maximum (|S| < kTop, so some entry lies outside S).
//   A node of S can only have lost score since the snapshot (monotone profile), so only the S nodes listed in T_j
//   above c* need an exact re-score — on the chain's current copy of their rows.  best = max(c*, those); best < ub
//   stops the round as before (ub bounds every node outside the pod's record, modified or not).
// The chain publishes, per pod, the winner and its slot; the keeper applies the pod's assume to the slot's row (its
// own register copy, lane = slot) and publishes the row's new state; each helper advances its own register copy of
// the rows to its lag from those states, and the chain reads them only to re-score a recent winner (rare: ~5 % of C3
// pods).
constexpr int kHelpers = 5;                        // helper waves
constexpr int kLag = kHelpers + 1;                 // helper(j) scores pod j on the table after pods ≤ j − kLag
constexpr int kTop = kLag;                         // candidates per pod handed to the chain (> |S| = kLag − 1)
constexpr int kMwThreads = kWave * (2 + kHelpers);  // the chain, the keeper, the helpers
constexpr uint32_t kTopMod = 0x80000000u;  // s_topx: a modified row (its slot in the low bits); otherwise the LDS
                                           // word offset of the candidate's round-start EvalRow
constexpr int64_t kMwSpin = 1 << 24;       // bounded in-workgroup waits (an error instead of a hang on a bug)

struct MwLayout {  // dynamic LDS carve; u64 arrays (word offsets), then u32 arrays (offsets from the u32 base)
  uint32_t cand, podw, par, prow, toprow, state, top, u64_end;
  uint32_t topx, win, wslot, nsl, ready, slot_node, slot_row, hash, prevn, sctl, u32_end;
};
__host__ __device__ inline MwLayout mw_layout(int nb) {
  MwLayout L;
  L.cand = 0;
  L.podw = L.cand + (uint32_t)nb * kCandStride;
  L.par = L.podw + (uint32_t)nb * kPodWords;
  L.prow = L.par + kParWords;                          // earlier rounds' rows (slots < nP)
  // slots of earlier rounds ≤ (depth − 1) · batch ≤ kMaxMod − nb (RoundGeom keeps depth · batch ≤ kMaxMod)
  L.toprow = L.prow + (uint32_t)(kMaxMod - nb) * kEvalRowWords;  // rows of listed candidates past the staged ones
  L.state = L.toprow + (uint32_t)nb * kTop * kEvalRowWords;  // the winner's row after pod j's assume
  L.top = L.state + (uint32_t)nb * kEvalRowWords;
  L.u64_end = L.top + (uint32_t)nb * kTop;
  L.topx = 0;
  L.win = L.topx + (uint32_t)nb * kTop;
  L.wslot = L.win + (uint32_t)nb;
  L.nsl = L.wslot + (uint32_t)nb;    // slots in use after pod j
  L.ready = L.nsl + (uint32_t)nb;    // helper(j) done
  L.slot_node = L.ready + (uint32_t)nb;
  L.slot_row = L.slot_node + kMaxMod;   // LDS word offset of the slot's round-start row
  L.hash = L.slot_row + kMaxMod;
  L.prevn = L.hash + kModHash;
  L.sctl = L.prevn + kMaxMod;  // [0] pods published, [1] chain ended, [2] abort, [3] nP, [4] error, [5] states kept
  L.u32_end = L.sctl + 8;
  return L;
}
inline size_t mw_lds_bytes(int nb) {
  const MwLayout L = mw_layout(nb);
  return (size_t)L.u64_end * 8 + (size_t)L.u32_end * 4;
}

// Hand-offs between the resolver's waves go through LDS only, and the LDS serves one wave's DS instructions in issue
// order: a flag written after the data it guards is seen by another wave only after that data, and that wave's data
// reads issued after it saw the flag are served after the writes.  So publishing needs no s_waitcnt (lds_rel: a
// compiler barrier, then the store) and observing needs none either (lds_acq: the load, then a compiler barrier) —
// the release / acquire fences would stall the chain on its own outstanding LDS traffic for nothing.
__device__ __forceinline__ uint32_t lds_ld(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ uint32_t lds_acq(const uint32_t* p) {
  const uint32_t v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  asm volatile("" ::: "memory");
  return v;
}
__device__ __forceinline__ void lds_rel(uint32_t* p, uint32_t v) {
  asm volatile("" ::: "memory");
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ int mod_lookup(const uint32_t* h, uint32_t node) {
  uint32_t i = mod_hash(node);
  for (int it = 0; it < kModHash; ++it) {
    const uint32_t v = lds_ld(&h[i]);
    if (v == 0u) return -1;
    if ((v >> 8) == node + 1u) return (int)(v & 0xFFu);
    i = (i + 1u) & (kModHash - 1);
  }
  return -1;
}
__device__ __forceinline__ void lds_put_row(uint64_t* dst, const EvalRow& er) {
  uint64_t w[kEvalRowWords];
  __builtin_memcpy(w, &er, sizeof(er));
#pragma unroll
  for (int q = 0; q < kEvalRowWords; ++q) dst[q] = w[q];
}
// fitsRequest over the kAux resources on a modified row whose state includes this round's pods ≤ upto (published
// winners in `win`)
__device__ __forceinline__ bool mw_aux_fits(const DevTable& T, uint32_t node, const int64_t* __restrict__ rq, int upto,
                                            const uint32_t* win, const DevPod* s_pods, const int64_t* __restrict__ prq) {
  int64_t add[kAux] = {0, 0, 0, 0, 0};
  for (int q = 0; q <= upto; ++q) {
    if (lds_ld(&win[q]) != node || !(s_pods[q].flags & P_AUX)) continue;
#pragma unroll
    for (int r = 0; r < kAux; ++r) add[r] += prq[(size_t)q * kAux + r];
  }
  bool ok = true;
#pragma unroll
  for (int r = 0; r < kAux; ++r)
    if (rq[r] != 0) ok &= !(rq[r] > T.aux[(size_t)r * T.cap + node] - (T.aux[(size_t)(kAux + r) * T.cap + node] + add[r]));
  return ok;
}

template <int PF, bool QUOTA>
__global__ __launch_bounds__(kMwThreads) void resolve_mw(DevTable T0, const DevPod* __restrict__ pods,
                                                         int64_t* __restrict__ ctl, int64_t first, int nb,
                                                         const uint64_t* __restrict__ cand, EvalParams P,
                                                         uint64_t* __restrict__ out_keys,
                                                         int32_t* __restrict__ modlists, int slot, int depth,
                                                         int n_prev, int32_t* __restrict__ poison, int64_t seq,
                                                         int wait, QuotaRow* __restrict__ quotas, int nq,
                                                         const int64_t* __restrict__ paux) {
  extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
  KG_STAMP(2, 0);
  const MwLayout L = mw_layout(nb);
  const int tid = threadIdx.x, lane = tid % kWave, wave = tid / kWave;
  if (wave == 0) __builtin_amdgcn_s_setprio(3);  // the chain first, then its helpers, then any wide-pass wave
  else __builtin_amdgcn_s_setprio(2);
  uint64_t* s_cand = smem + L.cand;
  uint64_t* s_par = smem + L.par;
  uint32_t* b32 = reinterpret_cast<uint32_t*>(smem + L.u64_end);
  uint32_t* s_topx = b32 + L.topx;
  uint32_t* s_win = b32 + L.win;
  uint32_t* s_wslot = b32 + L.wslot;
  uint32_t* s_nsl = b32 + L.nsl;
  uint32_t* s_ready = b32 + L.ready;
  uint32_t* s_slot_node = b32 + L.slot_node;
  uint32_t* s_slot_row = b32 + L.slot_row;
  uint32_t* s_hash = b32 + L.hash;
  uint32_t* s_prevn = b32 + L.prevn;
  uint32_t* s_ctl = b32 + L.sctl;
  const DevPod* s_pods = reinterpret_cast<const DevPod*>(smem + L.podw);
  if (tid < kParWords) {
    uint64_t pw[kParWords] = {};
    __builtin_memcpy(pw, &P, sizeof(P));
#pragma unroll
    for (int q = 0; q < kParWords; ++q)
      if (tid == q) s_par[q] = pw[q];
  }
  {  // prologue, independent of the previous round: LDS-DMA of the records and pods, flag / hash clears
    const int n16 = nb * kCandStride / 2;
    for (int it = 0; it * kMwThreads < n16; ++it) {
      const int idx = it * kMwThreads + tid;
      if (idx < n16)
        __builtin_amdgcn_global_load_lds((global_cvoid_ptr)(cand + 2 * (size_t)idx),
                                         (lds_void_ptr)(s_cand + 2 * ((size_t)it * kMwThreads + wave * kWave)), 16, 0, 0);
    }
    const uint64_t* pw = reinterpret_cast<const uint64_t*>(pods + first);
    const int p16 = nb * kPodWords / 2;
    for (int it = 0; it * kMwThreads < p16; ++it) {
      const int idx = it * kMwThreads + tid;
      if (idx < p16)
        __builtin_amdgcn_global_load_lds((global_cvoid_ptr)(pw + 2 * (size_t)idx),
                                         (lds_void_ptr)(smem + L.podw + 2 * ((size_t)it * kMwThreads + wave * kWave)), 16, 0, 0);
    }
    for (int w = tid; w < kModHash; w += kMwThreads) s_hash[w] = 0u;
    for (int w = tid; w < nb; w += kMwThreads) s_ready[w] = 0u;
    if (tid < 8) s_ctl[tid] = 0u;
  }
  // chain on the previous round's resolver (as resolve_round)
  if (wave == 0) {
    int timed_out = 0;
    if (wait) {
      if (lane == 0) {
        int64_t it = 0;
        while (__hip_atomic_load(&ctl[4], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < seq - 1) {
          __builtin_amdgcn_s_sleep(1);
          if (++it > kSpinLimit) {
            timed_out = 1;
            break;
          }
        }
      }
      timed_out = __builtin_amdgcn_readfirstlane(timed_out);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    KG_STAMP(2, 1);
    const int abort_ = timed_out || *poison || ctl[0] != first;
    if (abort_ && lane == 0 && timed_out) ctl[5] = 1;
    int nM = 0;
    if (!abort_) {  // rows the n_prev previous rounds modified: slots [0, nP), rows read after the chain wait
      for (int d = 1; d <= n_prev; ++d) {
        const int32_t* ml = modlists + (size_t)(((slot - d) % depth + depth) % depth) * kModListStride;
        const int c = ml[0];
        for (int t = lane; t < c; t += kWave) s_prevn[nM + t] = (uint32_t)ml[1 + t];
        nM += c;
      }
    }
    __builtin_amdgcn_wave_barrier();
    for (int s = lane; s < nM; s += kWave) {
      const uint32_t node = s_prevn[s];
      const bool mine = mod_insert(s_hash, node, s) == s;  // a node listed by two earlier rounds keeps its first slot
      s_slot_node[s] = mine ? node : kNoNode;
      s_slot_row[s] = L.prow + (uint32_t)s * kEvalRowWords;
      if (mine) lds_put_row(smem + L.prow + (size_t)s * kEvalRowWords, make_eval_row(load_row(table_at(T0), node), P));
    }
    if (lane == 0) {
      s_ctl[2] = (uint32_t)abort_;
      s_ctl[3] = (uint32_t)nM;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // LDS-DMA of records and pods (+ the rows above)
  __syncthreads();
  if (s_ctl[2]) {
    if (wave == 0) publish_round(ctl, seq);
    return;
  }
  KG_STAMP(2, 2);
  const uint64_t t_active = __builtin_amdgcn_s_memrealtime();  // the period decomposition's resolver time
  const int nP = (int)s_ctl[3];
  const bool narrow = P.score_bits <= 13;  // packed keys fit 32 bits (node < 2^19 = kMaxNodes)
  const int64_t* prq0 = paux + (size_t)first * kAux;

  if (wave >= 2) {
    // ---------------- helper waves: pods j ≡ wave − 2 (mod kHelpers) ----------------
    // The wave keeps its own copy of the modified rows at its snapshot (lane = slot, two banks), advanced by the
    // winners the chain publishes: a winner's row after its pod is read from s_state by its owner lane alone, so a
    // pod costs the LDS a few single-lane row reads instead of a 64-lane one (which saturated the CU's LDS pipe).
    int seen = nP;  // slots this wave has entered into the node → slot hash
    int applied = -1;  // pods whose placement this wave's rows include
    ModRow H0, H1;
    mod_row_init(H0);
    mod_row_init(H1);
    if (lane < nP && s_slot_node[lane] != kNoNode) {
      H0.node = s_slot_node[lane];
      H0.er = lds_row(smem + L.prow + (size_t)lane * kEvalRowWords);
    }
    if (kWave + lane < nP && s_slot_node[kWave + lane] != kNoNode) {
      H1.node = s_slot_node[kWave + lane];
      H1.er = lds_row(smem + L.prow + (size_t)(kWave + lane) * kEvalRowWords);
    }
    for (int j = wave - 2; j < nb; j += kHelpers) {
      const int lag = j - kLag;
      // the snapshot needs the keeper's states of pods ≤ lag (the chain has then published them too)
      uint32_t kept = lds_acq(&s_ctl[5]);
      bool gone = false;
      for (int64_t it = 0; (int)kept < lag + 1; ++it) {
        if (lds_acq(&s_ctl[1]) && (int)lds_acq(&s_ctl[0]) < lag + 1) {  // the chain ended before pod lag
          gone = true;
          break;
        }
        if (it > kMwSpin) {
          if (lane == 0) s_ctl[4] = 1u;  // waited too long: the round reports an error
          gone = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        kept = lds_acq(&s_ctl[5]);
      }
      if (gone) break;
      if (lane == 0) KG_LANE_SUB(j, 0);
      for (int k = applied + 1; k <= lag; ++k) {  // advance the snapshot to pods ≤ lag
        const uint32_t wk = s_win[k];
        if (wk == kNoNode) continue;
        const int sk = (int)s_wslot[k];
        if (sk < kWave) {
          if (lane == sk) H0.node = wk, H0.er = lds_row(smem + L.state + (size_t)k * kEvalRowWords);
        } else if (lane == sk - kWave) {
          H1.node = wk, H1.er = lds_row(smem + L.state + (size_t)k * kEvalRowWords);
        }
      }
      applied = lag > applied ? lag : applied;
      if (lane == 0) KG_LANE_SUB(j, 1);
      const int nSl = lag >= 0 ? (int)s_nsl[lag] : nP;
      for (int s = seen + lane; s < nSl; s += kWave) mod_insert(s_hash, s_slot_node[s], s);
      seen = nSl > seen ? nSl : seen;
      const DevPod p = s_pods[j];
      const bool aux = (PF & PF_FIT_FILTER) && (p.flags & P_AUX);
      const int64_t* rq = paux + (size_t)(first + j) * kAux;
      // the pod's listed candidates not modified at the snapshot (in key order: lane = record position)
      const uint64_t key = s_cand[(size_t)j * kCandStride + lane];
      bool modl = false;
      if (key) {
        const int sl = mod_lookup(s_hash, key_node(key));
        modl = sl >= 0 && sl < nSl;
      }
      const uint64_t um0 = __ballot(key != 0 && !modl);
      // lane i < kTop: the i-th of them; past the record's staged rows its round-start row comes from HBM, issued
      // now so that the load overlaps the modified rows' scoring below
      int my_lpos = -1;
      {
        uint64_t u = um0;
#pragma unroll
        for (int i = 0; i < kTop; ++i) {
          const int pos = u ? (int)__builtin_ctzll(u) : -1;
          u &= u - 1;
          if (lane == i) my_lpos = pos;
        }
      }
      const uint64_t my_lkey = __shfl(key, my_lpos >= 0 ? my_lpos : 0);  // every lane takes part in the permute
      const uint32_t my_lnode = key_node(my_lkey);
      const bool my_hbm = my_lpos >= kStaged;
      Row hr;
      if (my_hbm) hr = load_row(table_at(T0), my_lnode);
      // every modified row at the snapshot (after pods ≤ lag)
      uint64_t mk[2] = {0, 0};
      mk[0] = mod_row_key<PF>(H0, p, P, s_par);
      if (aux && mk[0] && !mw_aux_fits(table_at(T0), H0.node, rq, lag, s_win, s_pods, prq0)) mk[0] = 0;
      if (nSl > kWave) {
        mk[1] = mod_row_key<PF>(H1, p, P, s_par);
        if (aux && mk[1] && !mw_aux_fits(table_at(T0), H1.node, rq, lag, s_win, s_pods, prq0)) mk[1] = 0;
      }
      // T_j = the kTop best of the two descending sequences
      uint64_t um = um0;
      uint64_t tk_l = 0;
      uint32_t tx_l = 0;
      int n_listed = 0;  // listed entries taken so far (the n-th is lane n's my_lpos)
      uint64_t mrest = mk[0] > mk[1] ? mk[0] : mk[1];
      uint64_t mtop = wave_max_modkey(mrest, narrow);
#pragma unroll
      for (int i = 0; i < kTop; ++i) {
        const int lpos = um ? (int)__builtin_ctzll(um) : -1;
        const uint64_t lkey = lpos >= 0 ? readlane_u64(key, lpos) : 0;
        uint64_t tkey;
        uint32_t tx;
        if (lkey == 0 && mtop == 0) {
          tkey = 0;
          tx = 0;
        } else if (lkey > mtop) {
          tkey = lkey;
          um &= um - 1;
          tx = lpos < kStaged ? L.cand + (uint32_t)j * kCandStride + kRecRows + (uint32_t)lpos * kEvalRowWords
                              : L.toprow + (uint32_t)(j * kTop + n_listed) * kEvalRowWords;
          ++n_listed;
        } else {
          tkey = mtop;
          const uint64_t b0 = __ballot(mk[0] == mtop), b1 = __ballot(mk[1] == mtop);
          const int sl = b0 ? (int)__builtin_ctzll(b0) : kWave + (int)__builtin_ctzll(b1);
          tx = kTopMod | (uint32_t)sl;
          if (lane == (sl & (kWave - 1))) {
            if (sl < kWave) mk[0] = 0;
            else mk[1] = 0;
          }
          mrest = mk[0] > mk[1] ? mk[0] : mk[1];
          mtop = i + 1 < kTop ? wave_max_modkey(mrest, narrow) : 0;
        }
        if (lane == i) {
          tk_l = tkey;
          tx_l = tx;
        }
      }
      if (lane == 0) KG_LANE_SUB(j, 2);
      if (my_hbm && lane < n_listed)  // a listed entry of T_j past the staged rows: its row from the early load
        lds_put_row(smem + L.toprow + (size_t)(j * kTop + lane) * kEvalRowWords, make_eval_row(hr, P));
      if (lane < kTop) {
        smem[L.top + (size_t)j * kTop + lane] = tk_l;
        s_topx[j * kTop + lane] = tx_l;
      }
      if (lane == 0) lds_rel(&s_ready[j], 1u);
      if (lane == 0) KG_LANE_SUB(j, 3);
    }
    return;
  }

  if (wave == 1) {
    // ---------------- the keeper wave: the modified rows' states behind the chain ----------------
    // For each pod the chain has published, the winner's slot takes the pod's assume (NodeInfo.AddPod + LoadAware
    // Reserve → podAssignCache.assign) on its owner lane, and the row's new state goes to s_state[k]; helpers read
    // their snapshots from it, the chain only when it re-scores a recent winner.
    ModRow K0, K1;
    mod_row_init(K0);
    mod_row_init(K1);
    if (lane < nP && s_slot_node[lane] != kNoNode) {
      K0.node = s_slot_node[lane];
      K0.er = lds_row(smem + L.prow + (size_t)lane * kEvalRowWords);
    }
    if (kWave + lane < nP && s_slot_node[kWave + lane] != kNoNode) {
      K1.node = s_slot_node[kWave + lane];
      K1.er = lds_row(smem + L.prow + (size_t)(kWave + lane) * kEvalRowWords);
    }
    int known = nP;  // slots this wave holds (created in order by the chain)
    for (int k = 0; k < nb; ++k) {
      uint32_t done = lds_acq(&s_ctl[0]);
      for (int64_t it = 0; (int)done <= k; ++it) {
        if (lds_acq(&s_ctl[1]) || it > kMwSpin) break;
        __builtin_amdgcn_s_sleep(1);
        done = lds_acq(&s_ctl[0]);
      }
      if ((int)done <= k) {
        if (!lds_acq(&s_ctl[1]) && lane == 0) s_ctl[4] = 1u;
        break;
      }
      const uint32_t wk = s_win[k];
      if (wk != kNoNode) {
        const int sk = (int)s_wslot[k];
        const DevPod p = s_pods[k];
        if (sk >= known) {  // a new slot: its round-start row
          const uint32_t off = s_slot_row[sk];
          if (sk < kWave) {
            if (lane == sk) K0.node = wk, K0.er = lds_row(smem + off);
          } else if (lane == sk - kWave) {
            K1.node = wk, K1.er = lds_row(smem + off);
          }
          known = sk + 1;
        }
        if (sk < kWave) {
          if (lane == sk) {
            assume_mod<PF>(K0.er, p, P);
            lds_put_row(smem + L.state + (size_t)k * kEvalRowWords, K0.er);
          }
        } else if (lane == sk - kWave) {
          assume_mod<PF>(K1.er, p, P);
          lds_put_row(smem + L.state + (size_t)k * kEvalRowWords, K1.er);
        }
      }
      if (lane == 0) lds_rel(&s_ctl[5], (uint32_t)(k + 1));
    }
    return;
  }

  // ---------------- the chain wave ----------------
  DevQuota ql = QUOTA ? quota_load(quotas, nq, lane) : DevQuota{0, 0, 0, 0, 0, 0, 0, 0};
  uint32_t rw[kLag - 1];  // winners of the kLag − 1 previous pods (kNoNode: none), oldest first
  int rsl[kLag - 1];      // their slots
#pragma unroll
  for (int k = 0; k < kLag - 1; ++k) rw[k] = kNoNode, rsl[k] = -1;
  uint64_t my_out = 0;
  int consumed = 0, n_slow = 0, n_wait = 0, nS = nP, err = 0;
  // pod j's inputs are read during pod j − 1 (after its decision, before its publication): the helper's flag and T_j
  // in one LDS round trip — a wave's LDS reads are served in order, so T_j read after a set flag holds what the helper
  // wrote before it released the flag; a flag still clear is re-polled at pod j
  uint32_t rdy_n = lds_ld(&s_ready[0]);
  asm volatile("" ::: "memory");
  uint64_t tk_n = lane < kTop ? smem[L.top + lane] : 0;
  uint32_t tx_n = lane < kTop ? s_topx[lane] : 0u;
  uint64_t ub_n = s_cand[kC];
  DevPod p_n = s_pods[0];
  for (int j = 0; j < nb; ++j) {
    KG_POD_DIAG(j, (uint32_t)n_wait);
    const uint32_t rdy = rdy_n;
    uint64_t tk = tk_n;
    uint32_t tx = tx_n;
    const uint64_t ub = ub_n;
    const DevPod p = p_n;
    if (rdy == 0u) {
      ++n_wait;
      int64_t it = 0;
      while (lds_acq(&s_ready[j]) == 0u && ++it < kMwSpin) __builtin_amdgcn_s_sleep(0);
      if (it >= kMwSpin || lds_acq(&s_ctl[4])) {
        err = 1;
        break;
      }
      tk = lane < kTop ? smem[L.top + (size_t)j * kTop + lane] : 0;
      tx = lane < kTop ? s_topx[j * kTop + lane] : 0u;
    }
    bool placed = false;
    uint32_t w = kNoNode;
    int wsl = -1;
    if (!QUOTA || quota_admit(ql, p)) {  // ElasticQuota PreFilter rejects: Unschedulable, no node search
      const uint32_t tn = key_node(tk);
      bool inS = false;
#pragma unroll
      for (int k = 0; k < kLag - 1; ++k) inS |= tn == rw[k];
      inS &= tk != 0;
      const uint64_t okm = __ballot(tk != 0 && !inS);
      const int pos = okm ? (int)__builtin_ctzll(okm) : kTop;
      uint64_t best = okm ? readlane_u64(tk, pos) : 0;
      uint64_t above = __ballot(inS && lane < pos);
      KG_POD_SUB(j, 0);
      bool from_s = false;
      if (above) {  // recent winners listed above c*: re-score them exactly on their current rows (rare)
        ++n_slow;
        {  // the keeper has published the states of pods < j
          int64_t it = 0;
          while ((int)lds_acq(&s_ctl[5]) < j && ++it < kMwSpin) __builtin_amdgcn_s_sleep(0);
          if (it >= kMwSpin) {
            err = 1;
            break;
          }
        }
        // lane k < kLag − 1: window entry k (pod j − kLag + 1 + k); its state is the node's current row when no later
        // entry placed the same node
        uint32_t nd = kNoNode;
        bool last = true;
#pragma unroll
        for (int k = 0; k < kLag - 1; ++k) {
          if (lane == k) nd = rw[k];
          if (lane < k && nd == rw[k]) last = false;
        }
        bool want = false;
        while (above) {
          const int b = (int)__builtin_ctzll(above);
          above &= above - 1;
          want |= nd == (uint32_t)__builtin_amdgcn_readlane((int)tn, b);
        }
        want &= lane < kLag - 1 && nd != kNoNode && last;
        uint64_t mkv = 0;
        if (want) {
          const int step = j - (kLag - 1) + lane;
          const EvalRow er = lds_row(smem + L.state + (size_t)step * kEvalRowWords);
          mkv = mod_key<PF>(er, nd, p, P, s_par);
          const bool aux = (PF & PF_FIT_FILTER) && (p.flags & P_AUX);
          if (aux && mkv && !mod_aux_fits(table_at(T0), nd, paux + (size_t)(first + j) * kAux, j, my_out, s_pods, prq0))
            mkv = 0;
        }
        const uint64_t mbest = wave_max_modkey(mkv, narrow);
        from_s = mbest > best;
        best = from_s ? mbest : best;
      }
      if (best < ub) break;  // an unseen node could still win: leave this pod to the next round
      KG_POD_SUB(j, 1);
      my_out = lane == j ? best : my_out;
      if (best != 0) {  // 0: unschedulable (ub == 0: no feasible node anywhere)
        placed = true;
        w = key_node(best);
        if (from_s) {  // the slot of the last window entry that placed w
#pragma unroll
          for (int k = 0; k < kLag - 1; ++k) wsl = rw[k] == w ? rsl[k] : wsl;
        } else {
          const uint32_t cx = (uint32_t)__builtin_amdgcn_readlane((int)tx, pos);
          if (cx & kTopMod) {
            wsl = (int)(cx & 0xFFu);
          } else {  // a node first modified now: a new slot (the keeper loads its round-start row from LDS)
            wsl = nS++;
            if (lane == 0) {
              s_slot_node[wsl] = w;
              s_slot_row[wsl] = cx;
            }
          }
        }
      }
    } else {
      my_out = lane == j ? 0 : my_out;
    }
    KG_POD_SUB(j, 2);
    if (QUOTA && placed) quota_charge(ql, p, lane);  // ElasticQuota Reserve
    if (j + 1 < nb) {  // pod j + 1's inputs (see above)
      rdy_n = lds_ld(&s_ready[j + 1]);
      asm volatile("" ::: "memory");
      tk_n = lane < kTop ? smem[L.top + (size_t)(j + 1) * kTop + lane] : 0;
      tx_n = lane < kTop ? s_topx[(j + 1) * kTop + lane] : 0u;
      ub_n = s_cand[(size_t)(j + 1) * kCandStride + kC];
      p_n = s_pods[j + 1];
    }
    if (lane == 0) {
      s_win[j] = w;
      s_wslot[j] = (uint32_t)wsl;
      s_nsl[j] = (uint32_t)nS;
      lds_rel(&s_ctl[0], (uint32_t)(j + 1));
    }
    KG_POD_SUB(j, 3);
    ++consumed;
#pragma unroll
    for (int k = 0; k + 1 < kLag - 1; ++k) rw[k] = rw[k + 1], rsl[k] = rsl[k + 1];
    rw[kLag - 2] = w;
    rsl[kLag - 2] = wsl;
  }
  if (lane == 0) lds_rel(&s_ctl[1], 1u);  // the helpers stop waiting
  KG_STAMP(2, 30);
  // write-back (as resolve_round): each placed pod's terms onto its winner + this round's modified-row list
  const bool mine = !err && lane < consumed && my_out != 0;
  const uint32_t my_node = mine ? key_node(my_out) : kNoNode;
  if (mine) writeback_pod(table_at(T0), my_node, s_pods[lane], paux + (size_t)(first + lane) * kAux);
  int32_t* my_mod = modlists + (size_t)slot * kModListStride;
  const uint64_t lane_lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const uint64_t bm = __ballot(mine);
  if (mine) my_mod[1 + __popcll(bm & lane_lt)] = (int32_t)my_node;
  if (!err && lane < consumed) out_keys[first + lane] = my_out;
  if (QUOTA && !err) quota_store(quotas, nq, lane, ql);
  if (lane == 0) {
    my_mod[0] = __popcll(bm);
    if (err) {
      ctl[5] = 1;  // reported as a device error by the host
      *poison = 1;
    } else {
      ctl[0] = first + consumed;
      ctl[1] += 1;
      ctl[2] += consumed;
      ctl[6] += n_slow;  // diagnostics: pods that re-scored recent winners on the chain
      ctl[7] += n_wait;  // diagnostics: pods the chain waited for its helper
      if (consumed < nb) *poison = 1;
    }
    ctl[8] += (int64_t)(__builtin_amdgcn_s_memrealtime() - t_active);
  }
  publish_round(ctl, seq);
  KG_STAMP(2, 31);
}

// ---- NodeNUMAResource profiles (config C4) --------------------------------------------
// NUMA state per node: static TopologyOptions (NumaStatic, 128 B) + NodeAllocation (NumaMut, 96 B), AoS so
// one node's state is two contiguous lines.  The NUMA plugin is not monotone (Reserve moves cpus between
// NUMA nodes and the hint search can raise a score), so these profiles run unpipelined rounds and the
// resolver re-scores every modified row for every pod.
struct NumaTable {
  const NumaStatic* __restrict__ s;
  NumaMut* __restrict__ m;
};

// Reference-shaped Fit + LoadAware (eval_node) + NodeNUMAResource Filter/Score of one node for one pod.
// `aff` = the affinity NodeNUMAResource.Filter stores (valid when this returns true).
__device__ __forceinline__ bool eval_node_numa(const Row& r, const NumaView& nv, const DevPod& p, const NumaPod& np,
                                               const EvalParams& P, const NumaParams& NP, int64_t& total,
                                               NumaHint& aff) {
  int64_t t = 0;
  if (!eval_node(r, p, P, t)) return false;
  int64_t sc = 0;
  if (!numa_eval(nv, np, NP, r.req_cpu, r.req_mem, r.alloc_cpu, r.alloc_mem, sc, aff)) return false;
  total = t + (NP.score ? sc * NP.weight : 0);
  return true;
}

// Wide pass of a NUMA round.  One block per (256-node tile, pod group): wave w evaluates node row j = w of the tile
// (lane l → node tile·256 + w·64 + l) for the group's pods, Fit + LoadAware first, then NodeNUMAResource on the
// pods that survived, parking the values in LDS; after a barrier the waves split the group's pods for the
// per-pod top-kR selects of eval_round.  numa_eval is long and divergent, so one node per lane (4x the waves of
// a 4-nodes-per-lane tile) keeps the serial path of a wave short.  pods_per_wave ≤ kNumaPpw (host clamps).
constexpr int kNumaPpw = 8;

__global__ __launch_bounds__(kWave* kEvalWaves) void eval_round_numa(DevTable T, NumaTable NT,
                                                                       const DevPod* __restrict__ pods,
                                                                       const NumaPod* __restrict__ npods,
                                                                       int64_t first, int nb, int pods_per_wave,
                                                                       int64_t node_base, int64_t n_local,
                                                                       int nt_local, EvalParams P, NumaParams NP,
                                                                       uint64_t* __restrict__ lists,
                                                                       const int32_t* __restrict__ poison) {
  __shared__ uint32_t s_v[kNumaPpw][kNPT][kWave];
  if (*poison) return;
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int n_pg = (nb + pods_per_wave - 1) / pods_per_wave;
  const uint32_t nwg = gridDim.x, bid = blockIdx.x, xcd = bid % 8u, q = nwg / 8u, r = nwg % 8u;
  const uint32_t wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8u;
  const int tile = (int)(wgid / (uint32_t)n_pg);
  const int p0 = (int)(wgid % (uint32_t)n_pg) * pods_per_wave;
  if (tile >= nt_local || p0 >= nb) return;  // block-uniform
  const int p1 = (p0 + pods_per_wave) < nb ? (p0 + pods_per_wave) : nb;
  const int vbits = P.score_bits + 1;
  const int j = wave;
  int64_t local = (int64_t)tile * kTile + j * kWave + lane;
  asm volatile("" : "+v"(local));
  const bool in = local < n_local;
  // phase 1: Fit + LoadAware (the Row is dead afterwards but for the four NodeInfo terms NUMA reads)
  int64_t rq_c = 0, rq_m = 0, al_c = 0, al_m = 0;
  {
    Row row;
    row.flags = 0;
    if (in) row = load_row(T, node_base + local);
    for (int pi = p0; pi < p1; ++pi) {
      const DevPod p = pods[first + pi];
      int64_t t = 0;
      s_v[pi - p0][j][lane] = (in && eval_node(row, p, P, t)) ? (uint32_t)t + 1u : 0u;
    }
    rq_c = row.req_cpu;
    rq_m = row.req_mem;
    al_c = row.alloc_cpu;
    al_m = row.alloc_mem;
  }
  // phase 2: NodeNUMAResource on the pods Fit/LoadAware kept
  if (in) {
    const NumaView nv = make_view(NT.s + node_base + local, NT.m + node_base + local, NP);
    for (int pi = p0; pi < p1; ++pi) {
      const uint32_t v0 = s_v[pi - p0][j][lane];
      if (v0 == 0) continue;
      const NumaPod np = npods[first + pi];
      int64_t sc = 0;
      NumaHint aff;
      const bool ok = numa_eval(nv, np, NP, rq_c, rq_m, al_c, al_m, sc, aff);
      s_v[pi - p0][j][lane] = ok ? v0 + (uint32_t)(NP.score ? sc * NP.weight : 0) : 0u;
    }
  }
  __syncthreads();
  uint32_t gidx[kNPT];
#pragma unroll
  for (int jj = 0; jj < kNPT; ++jj) gidx[jj] = (uint32_t)(node_base + (int64_t)tile * kTile + jj * kWave + lane);
  for (int pi = p0 + wave; pi < p1; pi += kEvalWaves) {
    uint32_t v[kNPT];
#pragma unroll
    for (int jj = 0; jj < kNPT; ++jj) v[jj] = s_v[pi - p0][jj][lane];
    select_write(v, gidx, vbits, lists + ((size_t)pi * nt_local + tile) * kR, lane);
  }
}

// Single-wave FIFO resolver of a NUMA round (unpipelined).  Lane l < nM owns modified node l: its Row in
// registers, its NUMA state in LDS slot l.  Per pod: e = best unmodified candidate, mbest = exact re-score of
// every modified row; best < ub ends the round early (as resolve_round).  The winner's owner lane runs
// Reserve — the NUMA allocation with the exact cpuset (cpu accumulator); a failed Reserve leaves the pod
// unplaced (RunReservePluginsUnreserve) and the node unchanged.
constexpr int kNumaStaticWords = (int)(sizeof(NumaStatic) / 8), kNumaMutWords = (int)(sizeof(NumaMut) / 8);
constexpr int kNumaPodWords = (int)(sizeof(NumaPod) / 8);

__global__ __launch_bounds__(kWave) void resolve_round_numa(DevTable T, NumaTable NT, const DevPod* __restrict__ pods,
                                                             const NumaPod* __restrict__ npods,
                                                             int64_t* __restrict__ ctl, int64_t first, int nb,
                                                             const uint64_t* __restrict__ cand, EvalParams P,
                                                             NumaParams NP, uint64_t* __restrict__ out_keys,
                                                             uint64_t* __restrict__ out_cpus,
                                                             int64_t* __restrict__ out_nrec, int bitmap_words,
                                                             int32_t* __restrict__ poison, int64_t seq,
                                                             QuotaRow* __restrict__ quotas, int nq,
                                                             int32_t* __restrict__ modlists, int slot, int depth,
                                                             int n_prev, int wait) {
  extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
  const int lane = threadIdx.x;
  uint64_t* s_cand = smem;                                    // [nb][kCandStride]
  uint64_t* s_podw = s_cand + (size_t)nb * kCandStride;       // [nb] DevPod
  uint64_t* s_npw = s_podw + (size_t)nb * kPodWords;          // [nb] NumaPod
  uint64_t* s_nsw = s_npw + (size_t)nb * kNumaPodWords;       // [kWave] NumaStatic of the modified rows
  uint64_t* s_nmw = s_nsw + (size_t)kWave * kNumaStaticWords; // [kWave] NumaMut of the modified rows
  uint32_t* s_prevn = reinterpret_cast<uint32_t*>(s_nmw + (size_t)kWave * kNumaMutWords);  // [kWave] earlier winners
  uint32_t* bitmap = s_prevn + kWave;
  for (int w = lane; w < nb * kCandStride; w += kWave) s_cand[w] = cand[w];
  {
    const uint64_t* pw = reinterpret_cast<const uint64_t*>(pods + first);
    for (int w = lane; w < nb * kPodWords; w += kWave) s_podw[w] = pw[w];
    const uint64_t* nw = reinterpret_cast<const uint64_t*>(npods + first);
    for (int w = lane; w < nb * kNumaPodWords; w += kWave) s_npw[w] = nw[w];
  }
  for (int w = lane; w < bitmap_words; w += kWave) bitmap[w] = 0;
  __syncthreads();
  // (r5) pipelined rounds: chain on the previous round's resolver (its rows, cursor, poison and winner list are
  // published with a release of ctl[4] = its sequence number); bounded spin, as resolve_round
  int timed_out = 0;
  if (wait) {
    if (lane == 0) {
      int64_t it = 0;
      while (__hip_atomic_load(&ctl[4], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < seq - 1) {
        __builtin_amdgcn_s_sleep(1);
        if (++it > kSpinLimit) {
          timed_out = 1;
          break;
        }
      }
    }
    timed_out = __builtin_amdgcn_readfirstlane(timed_out);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  if (timed_out || *poison || ctl[0] != first) {
    if (lane == 0 && timed_out) ctl[5] = 1;
    publish_round(ctl, seq);
    return;
  }
  const uint64_t t_active = __builtin_amdgcn_s_memrealtime();  // the period decomposition's resolver time
  const DevPod* s_pods = reinterpret_cast<const DevPod*>(s_podw);
  const NumaPod* s_np = reinterpret_cast<const NumaPod*>(s_npw);
  NumaStatic* s_ns = reinterpret_cast<NumaStatic*>(s_nsw);
  NumaMut* s_nm = reinterpret_cast<NumaMut*>(s_nmw);
  uint32_t midx = 0xFFFFFFFFu;
  Row mrow;
  mrow.flags = 0;
  NumaView mv;
  bool touched = false;
  uint64_t my_out = 0;
  int nM = 0, consumed = 0;
  {  // the rows the n_prev earlier rounds modified (snapshot-stale: NUMA is not monotone, so every modified row is
     // re-scored for every pod anyway): de-duplicated into slots [0, nM), read after the chain wait
    int n = 0;
    for (int d = 1; d <= n_prev; ++d) {
      const int32_t* ml = modlists + (size_t)(((slot - d) % depth + depth) % depth) * kModListStride;
      const int c = ml[0];
      for (int t = lane; t < c; t += kWave) s_prevn[n + t] = (uint32_t)ml[1 + t];
      n += c;
    }
    __syncthreads();
    const uint32_t node = lane < n ? s_prevn[lane] : 0xFFFFFFFFu;
    bool dup = false;
    for (int k = 0; k < n; ++k) dup |= lane > k && node == (uint32_t)__builtin_amdgcn_readlane((int)node, k);
    const bool keep = lane < n && !dup;
    const uint64_t km = __ballot(keep);
    const uint64_t lane_lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const int sl = __popcll(km & lane_lt);
    __syncthreads();
    if (keep) s_prevn[sl] = node;
    __syncthreads();
    nM = __popcll(km);
    if (lane < nM) {
      midx = s_prevn[lane];
      mrow = load_row(T, midx);
      s_ns[lane] = NT.s[midx];
      s_nm[lane] = NT.m[midx];
      mv = make_view(&s_ns[lane], &s_nm[lane], NP);
      atomicOr(&bitmap[midx >> 5], 1u << (midx & 31));
    }
    __syncthreads();
  }
  DevQuota ql = quota_load(quotas, nq, lane);
  for (int j = 0; j < nb; ++j) {
    const uint64_t key = s_cand[(size_t)j * kCandStride + lane];
    const uint64_t ub = s_cand[(size_t)j * kCandStride + kC];
    const DevPod p = s_pods[j];
    const NumaPod np = s_np[j];
    KG_POD_DIAG(j, (uint64_t)nM);
    if (nq > 0 && !quota_admit(ql, p)) {  // ElasticQuota PreFilter rejects
      my_out = lane == j ? 0 : my_out;
      ++consumed;
      continue;
    }
    const uint32_t node = key_node(key);
    const bool unmod = (key != 0) && !((bitmap[node >> 5] >> (node & 31)) & 1u);
    const uint64_t um = __ballot(unmod);
    const int pos = um ? (int)__builtin_ctzll(um) : kC;
    uint64_t best = um ? readlane_u64(key, pos) : 0;
    // The best unmodified candidate e wins unless a modified row beats it: its row is brought into the spare slot
    // nM before the re-score, so its Filter (the affinity Reserve needs) runs alongside the modified rows' instead
    // of after the search on one lane.  Slot nM only becomes a modified row if e wins.
    if (lane == 0) KG_LANE_SUB(j, 0);
    if (um && lane == nM) {
      const uint32_t en = key_node(best);
      midx = en;
      mrow = load_row(T, en);
      s_ns[nM] = NT.s[en];
      s_nm[nM] = NT.m[en];
      mv = make_view(&s_ns[nM], &s_nm[nM], NP);
    }
    if (lane == 0) KG_LANE_SUB(j, 1);
    NumaHint maff{0, 1, 0, 0};  // the affinity of this lane's row (Reserve reuses it when the row wins)
    if (nM > 0 || um) {
      uint64_t mk = 0;
      if (lane < nM || (um && lane == nM)) {
        int64_t t = 0;
        if (eval_node_numa(mrow, mv, p, np, P, NP, t, maff) && lane < nM) mk = make_key(t, midx);
      }
      if (lane == 0) KG_LANE_SUB(j, 2);
      const uint64_t mbest = wave_max_key(mk);
      best = mbest > best ? mbest : best;
    }
    KG_POD_SUB(j, 0);
    if (best < ub) break;
    ++consumed;
    if (best == 0) {
      my_out = lane == j ? 0 : my_out;
      continue;
    }
    const uint32_t w = key_node(best);
    const uint64_t hit = __ballot((lane < nM) & (midx == w));
    const int owner = hit ? (int)__builtin_ctzll(hit) : nM;
    if (!hit) {  // w = e, already in slot nM = owner (with its affinity)
      if (lane == 0) bitmap[w >> 5] |= 1u << (w & 31);
      ++nM;
    }
    __syncthreads();
    KG_POD_SUB(j, 1);
    int placed = 0;
    {  // Reserve with the affinity Filter stored on the winner's row this pod, run wave-uniformly on the owner's
       // row (LDS slot `owner`): scalar mask arithmetic, the owner lane commits
      const NumaHint aff{(uint32_t)__builtin_amdgcn_readlane((int)maff.mask, owner),
                         __builtin_amdgcn_readlane(maff.nil, owner), __builtin_amdgcn_readlane(maff.preferred, owner),
                         __builtin_amdgcn_readlane(maff.score, owner)};
#ifdef KG_STAMPS
      if (j < 64 && lane == 0) g_pod_diag[j][5] = __builtin_amdgcn_s_memtime();
#endif
      CpuSet cpus;
      NumaAlloc rec;
      const NumaStatic ns = s_ns[owner];
      NumaMut nm = s_nm[owner];
      // the owner lane's view of its row is current (built when the row entered its slot, rebuilt after each of its
      // Reserves): read it across lanes instead of rebuilding it (a view build is ~5 k cycles)
      NumaView ov;
      {
        constexpr int kVw = (int)(sizeof(NumaView) / 4);
        static_assert(sizeof(NumaView) % 4 == 0, "NumaView in dwords");
        uint32_t vw[kVw];
        __builtin_memcpy(vw, &mv, sizeof(mv));
#pragma unroll
        for (int q = 0; q < kVw; ++q) vw[q] = (uint32_t)__builtin_amdgcn_readlane((int)vw[q], owner);
        __builtin_memcpy(&ov, vw, sizeof(ov));
      }
      if (lane == 0) KG_LANE_SUB(j, 3);
      placed = numa_reserve(ns, nm, ov, np, aff, cpus, rec) ? 1 : 0;
      if (lane == 0) KG_LANE_SUB(j, 4);
      if (placed && lane == owner) {
        s_nm[lane] = nm;
        mv = make_view(&s_ns[lane], &s_nm[lane], NP);
        mrow.req_cpu += p.req_cpu;  // assume: NodeInfo.AddPod + LoadAware assign cache
        mrow.req_mem += p.req_mem;
        mrow.nz_cpu += p.nz_cpu;
        mrow.nz_mem += p.nz_mem;
        mrow.la_used_cpu += p.est_cpu;
        mrow.la_used_mem += p.est_mem;
        if (p.flags & P_PROD) {
          mrow.la_pused_cpu += p.est_cpu;
          mrow.la_pused_mem += p.est_mem;
        }
        mrow.num_pods += 1;
        touched = true;
#pragma unroll
        for (int q = 0; q < kCpuWords; ++q) out_cpus[(size_t)(first + j) * kCpuWords + q] = cpus.w[q];
        int64_t* r = out_nrec + (size_t)(first + j) * kNumaRecWords;
        r[0] = rec.res;
#pragma unroll
        for (int i = 0; i < kNumaMax; ++i) {
          r[1 + i] = ((rec.res >> i) & 1u) ? rec.cpu[i] : 0;
          r[1 + kNumaMax + i] = ((rec.res >> i) & 1u) ? rec.mem[i] : 0;
        }
      }
    }
    KG_POD_SUB(j, 2);
    if (placed && nq > 0) quota_charge(ql, p, lane);
    my_out = lane == j ? (placed ? best : 0) : my_out;
    __syncthreads();
  }
  if (touched) {
    store_mutable(T, midx, mrow);
    NT.m[midx] = s_nm[lane];
  }
  if (lane < consumed) out_keys[first + lane] = my_out;
  quota_store(quotas, nq, lane, ql);
  {  // this round's modified rows (its placed pods' nodes; duplicates allowed) for the next rounds
    const bool mine = lane < consumed && my_out != 0;
    const uint64_t bm = __ballot(mine);
    const uint64_t lane_lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    int32_t* my_mod = modlists + (size_t)slot * kModListStride;
    if (mine) my_mod[1 + __popcll(bm & lane_lt)] = (int32_t)key_node(my_out);
    if (lane == 0) my_mod[0] = __popcll(bm);
  }
  if (lane == 0) {
    ctl[0] = first + consumed;
    ctl[1] += 1;
    ctl[2] += consumed;
    if (consumed < nb) *poison = 1;
    ctl[8] += (int64_t)(__builtin_amdgcn_s_memrealtime() - t_active);
  }
  publish_round(ctl, seq);
}

// (r6) Two-wave NUMA resolver: resolve_round_numa's chain split over the two waves of one workgroup.  Per pod j,
// phase A runs on both waves at once:
//   wave 0 (scorer):   pod j's exact key on every modified row (their committed states, i.e. after Reserve of pod
//                      j - 2) and the best unmodified candidate e's Filter (its affinity), e's row staged in the spare
//                      slot nM; keys and affinities go to LDS;
//   wave 1 (reserver): Reserve of pod j - 1 on its winner's slot (wave-uniform, on a copy), then pod j's exact key on
//                      that slot's new state — the one row whose state the scorer has not seen;
// after a barrier, phase B on the reserver: commit Reserve(j - 1)'s row, then pod j's decision (ElasticQuota admission,
// the early round end, e against the modified rows, the slot adopting e); a second barrier ends the pod.  The serial
// chain per pod becomes max(scorer, Reserve + one row) instead of their sum.  Same results as
// resolve_round_numa: the scorer's key of Reserve(j - 1)'s slot is replaced by the reserver's, every other slot's state
// is the one a sequential resolver would see.
constexpr int kRowWords = (int)(sizeof(Row) / 8);
static_assert(sizeof(Row) % 8 == 0, "Row in 8-byte words");
constexpr int kNuma2Threads = 2 * kWave;
// (r6) a row's view (make_view, ~3-4 k cycles on one lane) is built once per state and shared through LDS: the
// reserver publishes the view of the state it commits, the scorer the views of the rows it stages
constexpr int kViewWords = (int)(sizeof(NumaView) / 8);
static_assert(sizeof(NumaView) % 8 == 0, "NumaView in 8-byte words");
size_t numa2_extra_lds_bytes() {  // beyond resolve_numa_lds_bytes: slot Rows and views, reserver's NumaMut, keys, ...
  return ((size_t)kWave * (kRowWords + kViewWords + 1 + 2) + kNumaMutWords + 4) * 8 + (size_t)kWave * 4 * 2 + 16 * 4;
}
// the rows (and views) of each pod's first kNumaPre candidates, read into LDS once per round (after the chain wait, so
// an unmodified row's copy is current): the best unmodified candidate's staging then reads LDS instead of HBM and
// rebuilding its view on the serial path
constexpr int kNumaPre = 2;
constexpr int kPreWords = kRowWords + kNumaStaticWords + kNumaMutWords + kViewWords;
size_t numa2_pre_lds_bytes(int nb) { return (size_t)nb * kNumaPre * kPreWords * 8; }

__global__ __launch_bounds__(kNuma2Threads) void resolve_round_numa2(DevTable T, NumaTable NT,
                                                                      const DevPod* __restrict__ pods,
                                                                      const NumaPod* __restrict__ npods,
                                                                      int64_t* __restrict__ ctl, int64_t first, int nb,
                                                                      const uint64_t* __restrict__ cand, EvalParams P,
                                                                      NumaParams NP, uint64_t* __restrict__ out_keys,
                                                                      uint64_t* __restrict__ out_cpus,
                                                                      int64_t* __restrict__ out_nrec, int bitmap_words,
                                                                      int32_t* __restrict__ poison, int64_t seq,
                                                                      QuotaRow* __restrict__ quotas, int nq,
                                                                      int32_t* __restrict__ modlists, int slot,
                                                                      int depth, int n_prev, int wait, int npre) {
  extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
  const int tid = threadIdx.x, wave = tid / kWave, lane = tid % kWave;
  uint64_t* s_cand = smem;                                     // [nb][kCandStride]
  uint64_t* s_podw = s_cand + (size_t)nb * kCandStride;        // [nb] DevPod
  uint64_t* s_npw = s_podw + (size_t)nb * kPodWords;           // [nb] NumaPod
  uint64_t* s_nsw = s_npw + (size_t)nb * kNumaPodWords;        // [kWave] NumaStatic of the slots
  uint64_t* s_nmw = s_nsw + (size_t)kWave * kNumaStaticWords;  // [kWave] NumaMut of the slots (committed)
  uint64_t* s_roww = s_nmw + (size_t)kWave * kNumaMutWords;    // [kWave] Row of the slots (committed)
  uint64_t* s_vieww = s_roww + (size_t)kWave * kRowWords;      // [kWave] view of each slot's current state
  uint64_t* s_rnmw = s_vieww + (size_t)kWave * kViewWords;     // the reserver's NumaMut after its Reserve
  uint64_t* s_key = s_rnmw + kNumaMutWords;                    // [kWave] the scorer's keys of the current pod
  uint64_t* s_affw = s_key + kWave;                            // [kWave][2] the scorer's affinities (NumaHint)
  uint64_t* s_misc = s_affw + (size_t)kWave * 2;               // [4]: 0 = the current pod's e key (0 = none)
  uint32_t* s_ver = reinterpret_cast<uint32_t*>(s_misc + 4);   // [kWave] slot state versions
  uint32_t* s_node = s_ver + kWave;                            // [kWave] node of each slot
  int32_t* s_c = reinterpret_cast<int32_t*>(s_node + kWave);   // [16] 0 nM, 1 stop, 4 timed out, 5 abort
  uint32_t* bitmap = reinterpret_cast<uint32_t*>(s_c + 16);
  uint32_t* s_prevn = bitmap + bitmap_words;                   // [kWave] earlier rounds' winners (prologue)
  uint64_t* s_pre = reinterpret_cast<uint64_t*>(s_prevn + kWave);  // [nb][npre] Row, NumaStatic, NumaMut, view
  for (int w = tid; w < nb * kCandStride; w += kNuma2Threads) s_cand[w] = cand[w];
  {
    const uint64_t* pw = reinterpret_cast<const uint64_t*>(pods + first);
    for (int w = tid; w < nb * kPodWords; w += kNuma2Threads) s_podw[w] = pw[w];
    const uint64_t* nw = reinterpret_cast<const uint64_t*>(npods + first);
    for (int w = tid; w < nb * kNumaPodWords; w += kNuma2Threads) s_npw[w] = nw[w];
  }
  for (int w = tid; w < bitmap_words; w += kNuma2Threads) bitmap[w] = 0;
  if (tid < kWave) s_ver[tid] = 0;
  if (tid < 16) s_c[tid] = 0;
  __syncthreads();
  if (tid == 0) {  // (r5) pipelined rounds: chain on the previous round's resolver (bounded spin, as resolve_round)
    int timed_out = 0;
    if (wait) {
      int64_t it = 0;
      while (__hip_atomic_load(&ctl[4], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < seq - 1) {
        __builtin_amdgcn_s_sleep(1);
        if (++it > kSpinLimit) {
          timed_out = 1;
          break;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    s_c[4] = timed_out;
    s_c[5] = (timed_out || *poison || ctl[0] != first) ? 1 : 0;
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  if (s_c[5]) {
    if (tid == 0 && s_c[4]) ctl[5] = 1;
    publish_round(ctl, seq);
    return;
  }
  const uint64_t t_active = __builtin_amdgcn_s_memrealtime();
  for (int x = tid; x < nb * npre; x += kNuma2Threads) {  // the candidates' rows (one entry per thread)
    const uint64_t key = s_cand[(size_t)(x / npre) * kCandStride + x % npre];
    if (key == 0) continue;
    const uint32_t m = key_node(key);
    uint64_t* e = s_pre + (size_t)x * kPreWords;
    *reinterpret_cast<Row*>(e) = load_row(T, m);
    NumaStatic* es = reinterpret_cast<NumaStatic*>(e + kRowWords);
    NumaMut* em = reinterpret_cast<NumaMut*>(e + kRowWords + kNumaStaticWords);
    *es = NT.s[m];
    *em = NT.m[m];
    *reinterpret_cast<NumaView*>(e + kRowWords + kNumaStaticWords + kNumaMutWords) = make_view(es, em, NP);
  }
  const DevPod* s_pods = reinterpret_cast<const DevPod*>(s_podw);
  const NumaPod* s_np = reinterpret_cast<const NumaPod*>(s_npw);
  NumaStatic* s_ns = reinterpret_cast<NumaStatic*>(s_nsw);
  NumaMut* s_nm = reinterpret_cast<NumaMut*>(s_nmw);
  Row* s_row = reinterpret_cast<Row*>(s_roww);
  NumaMut* s_rnm = reinterpret_cast<NumaMut*>(s_rnmw);
  NumaView* s_view = reinterpret_cast<NumaView*>(s_vieww);
  // the rows the n_prev earlier rounds modified, de-duplicated into slots [0, nM) by wave 0 (as resolve_round_numa)
  {
    int n = 0;
    for (int d = 1; d <= n_prev; ++d) {
      const int32_t* ml = modlists + (size_t)(((slot - d) % depth + depth) % depth) * kModListStride;
      const int c = ml[0];
      if (wave == 0)
        for (int t = lane; t < c; t += kWave) s_prevn[n + t] = (uint32_t)ml[1 + t];
      n += c;
    }
    __syncthreads();
    const uint32_t node = (wave == 0 && lane < n) ? s_prevn[lane] : 0xFFFFFFFFu;
    bool dup = false;
    if (wave == 0)
      for (int k = 0; k < n; ++k) dup |= lane > k && node == (uint32_t)__builtin_amdgcn_readlane((int)node, k);
    const bool keep = wave == 0 && lane < n && !dup;
    const uint64_t km = __ballot(keep);
    const uint64_t lane_lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    __syncthreads();
    if (keep) s_prevn[__popcll(km & lane_lt)] = node;
    __syncthreads();
    if (wave == 0) {
      const int nM0 = __popcll(km);
      if (lane < nM0) {
        const uint32_t m = s_prevn[lane];
        s_node[lane] = m;
        s_row[lane] = load_row(T, m);
        s_ns[lane] = NT.s[m];
        s_nm[lane] = NT.m[m];
        atomicOr(&bitmap[m >> 5], 1u << (m & 31));
      }
      if (lane == 0) s_c[0] = nM0;
    }
    __syncthreads();
  }
  // scorer state (wave 0, lane = slot): the slot's node, Row and view, and the version they were built from
  uint32_t midx = 0xFFFFFFFFu, myver = 0;
  Row mrow;
  mrow.flags = 0;
  NumaView mv;
  if (wave == 0 && lane < s_c[0]) {
    midx = s_node[lane];
    mrow = s_row[lane];
    mv = make_view(&s_ns[lane], &s_nm[lane], NP);
    s_view[lane] = mv;
  }
  // reserver state (wave 1, uniform but my_out / quota lanes): the pending Reserve and the commit of the last one
  bool r_pend = false;
  int r_j = 0, r_slot = -1;
  uint64_t r_best = 0;
  NumaHint r_aff{0, 1, 0, 0};
  bool r_placed = false;  // this pod's phase A placed pod r_j (commit in phase B)
  int c_slot = -1;        // the slot that Reserve changed
  Row r_row;
  r_row.flags = 0;
  NumaView r_view;  // the view of c_slot's state after the last placed Reserve (published at its commit)
  uint64_t r_key = 0;           // pod j's key on c_slot's new state
  NumaHint r_aff2{0, 1, 0, 0};  // its affinity
  uint64_t touch = 0;           // slots with committed Reserves (written back at the end)
  uint64_t my_out = 0;
  int consumed = 0;
  DevQuota ql = quota_load(quotas, nq, wave == 1 ? lane : kWave);
  bool stop = false;
  for (int j = 0; j <= nb; ++j) {
    const bool live = j < nb && !stop;
#ifdef KG_STAMPS  // per pod: scorer phase A start / end, reserver phase A start / after Reserve / end, phase B end
#define KG_N2_STAMP(k) \
    if (lane == 0 && j < 64) g_pod_diag[j][k] = __builtin_amdgcn_s_memtime()
#define KG_N2_SUB(k) \
    if (lane == 0 && j < 64) g_lane_diag[j][k] = __builtin_amdgcn_s_memtime()
#else
#define KG_N2_STAMP(k)
#define KG_N2_SUB(k)
#endif
    if (wave == 0) {
      KG_N2_STAMP(0);
    } else {
      KG_N2_STAMP(2);
    }
    // ---- phase A ----
    if (wave == 0) {
      if (live) {
        const int nM = s_c[0];
        if (lane < nM && s_ver[lane] != myver) {  // the reserver committed a Reserve on this slot (and its view)
          myver = s_ver[lane];
          mrow = s_row[lane];
          mv = s_view[lane];
        }
        KG_N2_SUB(0);
        const uint64_t key = s_cand[(size_t)j * kCandStride + lane];
        const uint32_t node = key_node(key);
        const bool unmod = (key != 0) && !((bitmap[node >> 5] >> (node & 31)) & 1u);
        const uint64_t um = __ballot(unmod);
        const int pos = um ? (int)__builtin_ctzll(um) : kC;
        const uint64_t ekey = um ? readlane_u64(key, pos) : 0;
        const bool stage = um && nM < kWave;
        if (stage && pos < npre) {  // e's row from the round's LDS copy: the wave copies it into the spare slot nM
          const uint64_t* e = s_pre + ((size_t)j * npre + pos) * kPreWords;
          constexpr int kS = kRowWords, kM = kS + kNumaStaticWords, kV = kM + kNumaMutWords;
          for (int w = lane; w < kPreWords; w += kWave) {
            const uint64_t v = e[w];
            if (w < kS) s_roww[(size_t)nM * kRowWords + w] = v;
            else if (w < kM) s_nsw[(size_t)nM * kNumaStaticWords + (w - kS)] = v;
            else if (w < kV) s_nmw[(size_t)nM * kNumaMutWords + (w - kM)] = v;
            else s_vieww[(size_t)nM * kViewWords + (w - kV)] = v;
          }
          if (lane == nM) {  // its Filter gives the affinity Reserve needs (read from the copy: no cross-lane wait)
            midx = key_node(ekey);
            mrow = *reinterpret_cast<const Row*>(e);
            s_node[nM] = midx;
            myver = s_ver[nM];
            mv = *reinterpret_cast<const NumaView*>(e + kV);
          }
        } else if (stage && lane == nM) {  // e's row into the spare slot: its Filter gives the affinity Reserve needs
          const uint32_t en = key_node(ekey);
          midx = en;
          mrow = load_row(T, en);
          s_ns[nM] = NT.s[en];
          s_nm[nM] = NT.m[en];
          s_row[nM] = mrow;
          s_node[nM] = en;
          myver = s_ver[nM];
          mv = make_view(&s_ns[nM], &s_nm[nM], NP);
          s_view[nM] = mv;
        }
        const DevPod p = s_pods[j];
        const NumaPod np = s_np[j];
        uint64_t mk = 0;
        NumaHint maff{0, 1, 0, 0};
        KG_N2_SUB(1);
        if (lane < nM || (stage && lane == nM)) {
          int64_t t = 0;
          if (eval_node_numa(mrow, mv, p, np, P, NP, t, maff) && lane < nM) mk = make_key(t, midx);
        }
        KG_N2_SUB(2);
        if (lane <= nM && lane < kWave) {
          s_key[lane] = mk;
          s_affw[2 * lane] = (uint64_t)maff.mask | ((uint64_t)(uint32_t)maff.nil << 32);
          s_affw[2 * lane + 1] = (uint64_t)(uint32_t)maff.preferred | ((uint64_t)(uint32_t)maff.score << 32);
        }
        if (lane == 0) s_misc[0] = ekey;
      }
      KG_N2_STAMP(1);
    } else {
      r_placed = false;
      if (r_pend) {  // Reserve of pod r_j on slot r_slot (wave-uniform on copies; lane 0 writes the records)
        r_pend = false;
        const DevPod p = s_pods[r_j];
        const NumaPod np = s_np[r_j];
        const NumaStatic ns = s_ns[r_slot];
        NumaMut nm = s_nm[r_slot];
        // the slot's current view, published with its state (this wave's commit, or the scorer's staging of e)
        const NumaView ov = s_view[r_slot];
        CpuSet cpus;
        NumaAlloc rec;
        r_placed = numa_reserve(ns, nm, ov, np, r_aff, cpus, rec);
        if (r_placed) {
          c_slot = r_slot;
          r_row = s_row[r_slot];
          r_row.req_cpu += p.req_cpu;  // assume: NodeInfo.AddPod + LoadAware assign cache
          r_row.req_mem += p.req_mem;
          r_row.nz_cpu += p.nz_cpu;
          r_row.nz_mem += p.nz_mem;
          r_row.la_used_cpu += p.est_cpu;
          r_row.la_used_mem += p.est_mem;
          if (p.flags & P_PROD) {
            r_row.la_pused_cpu += p.est_cpu;
            r_row.la_pused_mem += p.est_mem;
          }
          r_row.num_pods += 1;
          *s_rnm = nm;  // every lane writes the same (uniform) state and reads back its own write
          if (lane == 0) {
#pragma unroll
            for (int q = 0; q < kCpuWords; ++q) out_cpus[(size_t)(first + r_j) * kCpuWords + q] = cpus.w[q];
            int64_t* r = out_nrec + (size_t)(first + r_j) * kNumaRecWords;
            r[0] = rec.res;
#pragma unroll
            for (int i = 0; i < kNumaMax; ++i) {
              r[1 + i] = ((rec.res >> i) & 1u) ? rec.cpu[i] : 0;
              r[1 + kNumaMax + i] = ((rec.res >> i) & 1u) ? rec.mem[i] : 0;
            }
          }
          if (nq > 0) quota_charge(ql, p, lane);
          KG_N2_STAMP(3);
          r_view = make_view(&s_ns[r_slot], s_rnm, NP);
          if (live) {  // pod j's key on the new state (the scorer saw the state before this Reserve)
            int64_t t = 0;
            r_aff2 = NumaHint{0, 1, 0, 0};
            r_key = eval_node_numa(r_row, r_view, s_pods[j], s_np[j], P, NP, t, r_aff2)
                        ? make_key(t, s_node[r_slot]) : 0;
          }
        }
        my_out = lane == r_j ? (r_placed ? r_best : 0) : my_out;
      }
      KG_N2_STAMP(4);
    }
    __syncthreads();
    // ---- phase B (reserver) ----
    if (wave == 1) {
      if (r_placed) {  // commit Reserve(r_j): the scorer rebuilds this slot from LDS at its next pod
        if (lane == 0) {
          s_nm[c_slot] = *s_rnm;
          s_row[c_slot] = r_row;
          s_view[c_slot] = r_view;
          s_ver[c_slot] += 1;
        }
        touch |= 1ull << c_slot;
      }
      if (live) {
        const DevPod p = s_pods[j];
        const int nM = s_c[0];
        if (nq > 0 && !quota_admit(ql, p)) {  // ElasticQuota PreFilter rejects
          my_out = lane == j ? 0 : my_out;
          ++consumed;
        } else {
          const uint64_t ekey = s_misc[0];
          const uint64_t ub = s_cand[(size_t)j * kCandStride + kC];
          uint64_t mk = lane < nM ? s_key[lane] : 0;
          if (r_placed && lane == c_slot) mk = r_key;  // the slot Reserve(j - 1) changed
          const uint64_t mbest = wave_max_key(mk);
          const uint64_t best = mbest > ekey ? mbest : ekey;
          if (best < ub) {
            stop = true;
            if (lane == 0) s_c[1] = 1;
          } else {
            ++consumed;
            if (best == 0) {
              my_out = lane == j ? 0 : my_out;
            } else {
              const uint32_t w = key_node(best);
              const uint64_t hit = __ballot(lane < nM && s_node[lane] == w);
              const int owner = hit ? (int)__builtin_ctzll(hit) : nM;
              if (!hit) {  // w = e, staged in slot nM: the slot becomes a modified row
                if (lane == 0) {
                  bitmap[w >> 5] |= 1u << (w & 31);
                  s_c[0] = nM + 1;
                }
              }
              if (r_placed && owner == c_slot) {
                r_aff = r_aff2;
              } else {
                const uint64_t a0 = s_affw[2 * owner], a1 = s_affw[2 * owner + 1];
                r_aff = NumaHint{(uint32_t)a0, (int)(uint32_t)(a0 >> 32), (int)(uint32_t)a1, (int)(uint32_t)(a1 >> 32)};
              }
              r_pend = true;
              r_j = j;
              r_slot = owner;
              r_best = best;
            }
          }
        }
      }
    }
    if (wave == 1) {
      KG_N2_STAMP(5);
    }
    __syncthreads();
    stop = s_c[1] != 0;
    if (!live) break;
#undef KG_N2_STAMP
#undef KG_N2_SUB
  }
  // write-back (reserver): the committed slots' rows, placements, quota, this round's modified-row list
  if (wave == 1) {
    if (lane < s_c[0] && ((touch >> lane) & 1ull)) {
      const uint32_t m = s_node[lane];
      store_mutable(T, m, s_row[lane]);
      NT.m[m] = s_nm[lane];
    }
    if (lane < consumed) out_keys[first + lane] = my_out;
    quota_store(quotas, nq, lane, ql);
    const bool mine = lane < consumed && my_out != 0;
    const uint64_t bm = __ballot(mine);
    const uint64_t lane_lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    int32_t* my_mod = modlists + (size_t)slot * kModListStride;
    if (mine) my_mod[1 + __popcll(bm & lane_lt)] = (int32_t)key_node(my_out);
    if (lane == 0) {
      my_mod[0] = __popcll(bm);
      ctl[0] = first + consumed;
      ctl[1] += 1;
      ctl[2] += consumed;
      if (consumed < nb) *poison = 1;
      ctl[8] += (int64_t)(__builtin_amdgcn_s_memrealtime() - t_active);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __syncthreads();
  publish_round(ctl, seq);
}

// kg_pods_evaluate_numa: NodeNUMAResource Filter + Score of one pod on every node (the plugin alone)
__global__ void evaluate_pod_numa(DevTable T, NumaTable NT, const DevPod* __restrict__ pod,
                                  const NumaPod* __restrict__ npod, int64_t n, NumaParams NP,
                                  int32_t* __restrict__ pass, int64_t* __restrict__ score,
                                  int64_t* __restrict__ affinity) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Row r = load_row(T, i);
  NumaParams q = NP;  // Filter only when the profile runs it (a Score-only profile scores the nil affinity)
  q.score = 1;
  int64_t sc = 0;
  NumaHint aff;
  const NumaView nv = make_view(NT.s + i, NT.m + i, q);
  const bool ok = numa_eval(nv, *npod, q, r.req_cpu, r.req_mem, r.alloc_cpu, r.alloc_mem, sc, aff);
  pass[i] = ok ? 1 : 0;
  score[i] = ok ? sc : 0;
  affinity[i] = aff.nil ? -1 : (int64_t)aff.mask;
}

// Scatter of upserted NUMA rows (static + NodeAllocation)
__global__ void scatter_numa(NumaTable NT, const NumaStatic* __restrict__ s, const NumaMut* __restrict__ m,
                             const int32_t* __restrict__ idx, int64_t n) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const int64_t i = idx[k];
  const_cast<NumaStatic*>(NT.s)[i] = s[k];
  NT.m[i] = m[k];
}

// ---- DeviceShare profiles (config C5) -------------------------------------------------------
// DeviceShare's Score is normalized per pod (DefaultNormalizeScore: 100·s / max over the feasible nodes), so a
// node's key depends on the maximum M over the whole cluster.  Per round:
//   ds_max_round   — every (pod, tile): max raw DeviceShare score over the tile's feasible nodes + how many hold it
//   ds_norm_reduce — per pod: M = max over tiles, c = #feasible nodes with raw == M (round-start snapshot)
//   eval_round_ds  — keys with that M (Fit + LoadAware + w·normalized DeviceShare), top-kR per tile
//   merge_round    — as for the other profiles
//   resolve_round_ds — FIFO replay; pod j keeps M_j = M only if an unmodified node or a modified row still holds
//                    M (counts of round-start holders among the modified rows); otherwise the round ends there.
// Rounds are unpipelined and driven by the device cursor: every kernel reads its first pod from ctl[0], so an
// early stop just makes the next round start at the cursor (no poison, no host round trip).
constexpr int kDsPpw = 8;

struct DsTable {
  DsNode* __restrict__ d;
};

__device__ __forceinline__ bool ds_round_range(const int64_t* ctl, int64_t end, int B, int64_t& first, int& nb) {
  first = ctl[0];
  const int64_t left = end - first;
  nb = left < B ? (int)left : B;
  return nb > 0;
}

template <int PF>
__global__ __launch_bounds__(kWave* kEvalWaves) void ds_max_round(DevTable T, DsTable DT,
                                                                   const DevPod* __restrict__ pods,
                                                                   const DsPod* __restrict__ dpods,
                                                                   const int64_t* __restrict__ ctl, int64_t end,
                                                                   int B, int pods_per_wave, int64_t base,
                                                                   int64_t n_local, int nt_local, EvalParams P,
                                                                   DsParams DP, uint64_t* __restrict__ dsmax,
                                                                   uint32_t* __restrict__ dsval) {
  int64_t first;
  int nb;
  if (!ds_round_range(ctl, end, B, first, nb)) return;
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int n_pg = (B + pods_per_wave - 1) / pods_per_wave;
  const uint32_t nwg = gridDim.x, bid = blockIdx.x, xcd = bid % 8u, q = nwg / 8u, r = nwg % 8u;
  const uint32_t wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8u;
  const int tile = (int)(wgid / (uint32_t)n_pg) * kEvalWaves + wave;
  const int p0 = (int)(wgid % (uint32_t)n_pg) * pods_per_wave;
  if (tile >= nt_local || p0 >= nb) return;
  const int np = ((p0 + pods_per_wave) < nb ? (p0 + pods_per_wave) : nb) - p0;
  uint32_t mx[kDsPpw], cnt[kDsPpw];
#pragma unroll
  for (int k = 0; k < kDsPpw; ++k) mx[k] = 0, cnt[k] = 0;
  for (int j = 0; j < kNPT; ++j) {
    const int64_t i = (int64_t)tile * kTile + j * kWave + lane;  // shard-local; the node is base + i
    if (i >= n_local) break;
    // Fit + LoadAware on the compact hoisted row of the C3 wide pass (eval_hot); a row outside its exact
    // domain (F_RARE) sends this node row of the wave to the reference-shaped eval_node
    const HotRow h = load_hot<PF>(T, base + i, P);
    const bool rare = __ballot((h.flags & F_RARE) != 0) != 0;
    Row row;
    row.flags = 0;
    if (rare) row = load_row(T, base + i);
    const DsNode d = DT.d[base + i];
#pragma unroll
    for (int k = 0; k < kDsPpw; ++k) {
      if (k >= np) break;
      int64_t t = 0, raw = 0;
      uint32_t packed = 0;
      const DevPod& pod = pods[first + p0 + k];
      bool ok;
      if (rare) {
        ok = eval_node(row, pod, P, t);
      } else {
        uint32_t t32 = 0;
        ok = eval_hot<PF>(h, pod, P, t32);
        t = t32;
      }
      if (ok && ds_eval(d, dpods[first + p0 + k], DP, raw)) {
        const uint32_t v = (uint32_t)raw + 1u;  // +1: a feasible node with raw 0 still counts
        cnt[k] = v > mx[k] ? 1u : cnt[k] + (v == mx[k] ? 1u : 0u);
        mx[k] = v > mx[k] ? v : mx[k];
        packed = (((uint32_t)t << 8) | (uint32_t)raw) + 1u;  // t < 2^23 (host check), raw ≤ 100
      }
      dsval[(size_t)(p0 + k) * ((size_t)nt_local * kTile) + i] = packed;  // eval_round_ds reads this back
    }
  }
#pragma unroll
  for (int k = 0; k < kDsPpw; ++k) {
    if (k >= np) break;
    const uint32_t m = wave_max_u32(mx[k]);
    const uint32_t c = wave_sum_u32(mx[k] == m ? cnt[k] : 0u);
    if (lane == 0) dsmax[(size_t)(p0 + k) * nt_local + tile] = ((uint64_t)m << 32) | c;
  }
}

// per pod: (M + 1) << 32 | c over the tiles (0: no feasible node)
__global__ __launch_bounds__(256) void ds_norm_reduce(const int64_t* __restrict__ ctl, int64_t end, int B,
                                                      const uint64_t* __restrict__ dsmax, int nt_local,
                                                      uint64_t* __restrict__ dsnorm) {
  __shared__ uint32_t s_m[256 / kWave], s_c[256 / kWave];
  int64_t first;
  int nb;
  if (!ds_round_range(ctl, end, B, first, nb)) return;
  const int pod = blockIdx.x;
  if (pod >= nb) return;
  const int tid = threadIdx.x, lane = tid % kWave, wave = tid / kWave;
  uint32_t m = 0, c = 0;
  for (int t = tid; t < nt_local; t += 256) {
    const uint64_t v = dsmax[(size_t)pod * nt_local + t];
    const uint32_t vm = (uint32_t)(v >> 32), vc = (uint32_t)v;
    c = vm > m ? vc : c + (vm == m ? vc : 0u);
    m = vm > m ? vm : m;
  }
  const uint32_t wm = wave_max_u32(m);
  const uint32_t wc = wave_sum_u32(m == wm ? c : 0u);
  if (lane == 0) s_m[wave] = wm, s_c[wave] = wc;
  __syncthreads();
  if (tid == 0) {
    uint32_t M = 0, C = 0;
    for (int w = 0; w < 256 / kWave; ++w) {
      C = s_m[w] > M ? s_c[w] : C + (s_m[w] == M ? s_c[w] : 0u);
      M = s_m[w] > M ? s_m[w] : M;
    }
    dsnorm[pod] = ((uint64_t)M << 32) | C;
  }
}

// several ranks: the global (M + 1, holders) per pod from the ranks' (all-gathered) shard values — the max of M,
// the holders summed over the ranks that hold it
__global__ __launch_bounds__(kMaxB) void ds_norm_combine(const int64_t* __restrict__ ctl, int64_t end, int B,
                                                         const uint64_t* __restrict__ all, int n_ranks,
                                                         uint64_t* __restrict__ dsnorm) {
  int64_t first;
  int nb;
  if (!ds_round_range(ctl, end, B, first, nb)) return;
  const int pod = threadIdx.x;
  if (pod >= nb) return;
  uint32_t M = 0, C = 0;
  for (int r = 0; r < n_ranks; ++r) {
    const uint64_t v = all[(size_t)r * B + pod];
    const uint32_t vm = (uint32_t)(v >> 32), vc = (uint32_t)v;
    C = vm > M ? vc : C + (vm == M ? vc : 0u);
    M = vm > M ? vm : M;
  }
  dsnorm[pod] = ((uint64_t)M << 32) | C;
}

__global__ __launch_bounds__(kWave* kEvalWaves) void eval_round_ds(const int64_t* __restrict__ ctl, int64_t end,
                                                                    int B, int pods_per_wave, int64_t base,
                                                                    int64_t n_local,
                                                                    int nt_local, EvalParams P, DsParams DP,
                                                                    const uint64_t* __restrict__ dsnorm,
                                                                    const uint32_t* __restrict__ dsval,
                                                                    uint64_t* __restrict__ lists) {
  // ds_max_round left every (pod, node)'s Fit + LoadAware total and raw DeviceShare score packed in dsval
  // ((t << 8 | raw) + 1, 0 = filtered out): this pass only normalizes with M and selects.
  int64_t first;
  int nb;
  if (!ds_round_range(ctl, end, B, first, nb)) return;
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int n_pg = (B + pods_per_wave - 1) / pods_per_wave;
  const uint32_t nwg = gridDim.x, bid = blockIdx.x, xcd = bid % 8u, q = nwg / 8u, r = nwg % 8u;
  const uint32_t wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8u;
  const int tile = (int)(wgid / (uint32_t)n_pg) * kEvalWaves + wave;
  const int p0 = (int)(wgid % (uint32_t)n_pg) * pods_per_wave;
  if (tile >= nt_local || p0 >= nb) return;
  const int np = ((p0 + pods_per_wave) < nb ? (p0 + pods_per_wave) : nb) - p0;
  const int vbits = P.score_bits + 1;
  const size_t stride = (size_t)nt_local * kTile;
  uint32_t gidx[kNPT], lidx[kNPT];  // global node index (the key), shard-local index (dsval)
#pragma unroll
  for (int j = 0; j < kNPT; ++j) {
    lidx[j] = (uint32_t)((int64_t)tile * kTile + j * kWave + lane);
    gidx[j] = (uint32_t)(base + lidx[j]);
  }
  for (int k = 0; k < np; ++k) {
    const uint32_t mm = (uint32_t)(dsnorm[p0 + k] >> 32);
    const uint32_t M = mm ? mm - 1u : 0u;
    uint32_t v[kNPT];
#pragma unroll
    for (int j = 0; j < kNPT; ++j) {
      const uint32_t pk = (int64_t)lidx[j] < n_local ? dsval[(size_t)(p0 + k) * stride + lidx[j]] : 0u;
      const uint32_t t = (pk - 1u) >> 8, raw = (pk - 1u) & 255u;
      v[j] = pk ? t + (DP.score ? (uint32_t)(DP.weight * ds_normalized(raw, M)) : 0u) + 1u : 0u;
    }
    select_write(v, gidx, vbits, lists + ((size_t)(p0 + k) * nt_local + tile) * kR, lane);
  }
}

// Single-wave FIFO resolver of a DeviceShare round.  Lane l < nM owns modified node l: its Row in registers and
// its DsNode in LDS, plus the round-start copies of both (what the wide passes saw).
constexpr int kDsNodeWords = (int)(sizeof(DsNode) / 8), kDsPodWords = (int)(sizeof(DsPod) / 8);

__global__ __launch_bounds__(kWave) void resolve_round_ds(DevTable T, DsTable DT, const DevPod* __restrict__ pods,
                                                           const DsPod* __restrict__ dpods,
                                                           int64_t* __restrict__ ctl, int64_t end, int B,
                                                           const uint64_t* __restrict__ cand,
                                                           const uint64_t* __restrict__ dsnorm,
                                                           const uint32_t* __restrict__ dsval, int64_t dsval_stride,
                                                           EvalParams P,
                                                           DsParams DP, uint64_t* __restrict__ out_keys,
                                                           int32_t* __restrict__ out_minors, int bitmap_words,
                                                           QuotaRow* __restrict__ quotas, int nq,
                                                           const int64_t* __restrict__ qdev, int sharded) {
  // sharded (several ranks): dsval holds only this rank's shard, so a modified row's round-start value is
  // re-evaluated from its round-start Row / DsNode copies (s_r0 / s_d0) instead of read from dsval
  extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
  const int lane = threadIdx.x;
  int64_t first;
  int nb;
  if (!ds_round_range(ctl, end, B, first, nb)) return;
  const uint64_t t_active = __builtin_amdgcn_s_memrealtime();  // the period decomposition's resolver time
  uint64_t* s_cand = smem;                                  // [nb][kCandStride]
  uint64_t* s_podw = s_cand + (size_t)nb * kCandStride;     // [nb] DevPod
  uint64_t* s_dpw = s_podw + (size_t)nb * kPodWords;        // [nb] DsPod
  uint64_t* s_cur = s_dpw + (size_t)nb * kDsPodWords;       // [kWave] DsNode, current
  uint64_t* s_stg = s_cur + (size_t)kWave * kDsNodeWords;   // [nb] DsNode of each pod's top candidate
  QuotaRow* s_q = reinterpret_cast<QuotaRow*>(s_stg + (size_t)nb * kDsNodeWords);  // [nq] quota rows
  int64_t* s_qdev = reinterpret_cast<int64_t*>(s_q + nq);   // [nb][kQuotaRes] device quota requests
  Row* s_srow = reinterpret_cast<Row*>(s_qdev + (size_t)nb * kQuotaRes);  // [nb] its Row
  DsNode* s_d0 = reinterpret_cast<DsNode*>(s_srow + nb);    // sharded: [kWave] round-start DsNode per modified lane
  Row* s_r0 = reinterpret_cast<Row*>(s_d0 + (sharded ? kWave : 0));  // sharded: [kWave] round-start Row
  uint32_t* bitmap = reinterpret_cast<uint32_t*>(s_r0 + (sharded ? kWave : 0));
  for (int w = lane; w < nb * kCandStride; w += kWave) s_cand[w] = cand[w];
  {
    const uint64_t* pw = reinterpret_cast<const uint64_t*>(pods + first);
    for (int w = lane; w < nb * kPodWords; w += kWave) s_podw[w] = pw[w];
    const uint64_t* dw = reinterpret_cast<const uint64_t*>(dpods + first);
    for (int w = lane; w < nb * kDsPodWords; w += kWave) s_dpw[w] = dw[w];
    if (nq > 0) {  // ElasticQuota rows (cpu, memory, device resources) + the pods' device requests
      const uint64_t* qw = reinterpret_cast<const uint64_t*>(quotas);
      uint64_t* sq = reinterpret_cast<uint64_t*>(s_q);
      for (int w = lane; w < nq * (int)(sizeof(QuotaRow) / 8); w += kWave) sq[w] = qw[w];
      for (int w = lane; w < nb * kQuotaRes; w += kWave) s_qdev[w] = qdev[(size_t)first * kQuotaRes + w];
    }
  }
  for (int w = lane; w < bitmap_words; w += kWave) bitmap[w] = 0;
  // stage the round-start row of every pod's top candidate (the usual winner): a first assume onto it then
  // reads LDS instead of waiting on HBM inside the serial loop
  uint32_t stg_node = 0xFFFFFFFFu;
  const uint64_t my_nrm = lane < nb ? dsnorm[lane] : 0;  // pod `lane`'s (M + 1, holders), read by readlane
  if (lane < nb) {
    const uint64_t k0 = cand[(size_t)lane * kCandStride];
    if (k0 != 0) {
      stg_node = key_node(k0);
      s_srow[lane] = load_row(T, stg_node);
      __builtin_memcpy(reinterpret_cast<DsNode*>(s_stg) + lane, DT.d + stg_node, sizeof(DsNode));
    }
  }
  __syncthreads();
  const DevPod* s_pods = reinterpret_cast<const DevPod*>(s_podw);
  const DsPod* s_dp = reinterpret_cast<const DsPod*>(s_dpw);
  DsNode* s_dc = reinterpret_cast<DsNode*>(s_cur);
  uint32_t midx = 0xFFFFFFFFu;
  Row mrow;
  mrow.flags = 0;
  bool touched = false;
  uint64_t my_out = 0;
  int32_t my_minors = 0;
  int nM = 0, consumed = 0;
  for (int j = 0; j < nb; ++j) {
    const uint64_t key = s_cand[(size_t)j * kCandStride + lane];
    const uint64_t ub = s_cand[(size_t)j * kCandStride + kC];
    const DevPod p = s_pods[j];
    const DsPod dp = s_dp[j];
    QuotaReq qr;
    if (p.quota >= 0) qr = quota_req(p, s_qdev + (size_t)j * kQuotaRes);
    if (p.quota >= 0 && !quota_row_admit(s_q[p.quota], qr, (p.flags & P_NONPREEMPT) != 0)) {  // PreFilter rejects
      my_out = lane == j ? 0 : my_out;
      my_minors = lane == j ? 0 : my_minors;
      ++consumed;
      continue;
    }
    const uint64_t nrm = readlane_u64(my_nrm, j);
    const uint32_t Mrs = (uint32_t)(nrm >> 32), Crs = (uint32_t)nrm;  // Mrs = max raw + 1 (0: no feasible node)
    // M_j: the round-start max survives while an unmodified node or a modified row still holds it.  At most nM
    // holders can have been modified, so with more than nM holders nothing needs checking.  A modified row's
    // round-start value for pod j is what ds_max_round packed for it (dsval): no re-score.
    // MostAllocated: an assume RAISES the node's raw score, so a modified row can also lift the max above M — the
    // modified rows are re-scored for every pod and the round ends when their max exceeds the round-start M.
    const bool most = DP.most != 0;
    bool cf = false, have_cur = false;
    int64_t ct = 0, craw = 0;
    if (DP.score && Mrs > 0 && (most ? nM > 0 : Crs <= (uint32_t)nM)) {
      uint32_t pk = 0;
      if (lane < nM) {
        if (sharded) {
          int64_t t0 = 0, raw0 = 0;
          pk = (eval_node(s_r0[lane], p, P, t0) && ds_eval(s_d0[lane], dp, DP, raw0)) ? (uint32_t)raw0 + 1u : 0u;
        } else {
          pk = dsval[(size_t)j * dsval_stride + midx];
        }
      }
      const bool rf = pk != 0;
      const int64_t rraw = (int64_t)((pk - 1u) & 255u);
      const uint32_t lost = (uint32_t)__popcll(__ballot(rf && (uint32_t)rraw + 1u == Mrs));
      if (most || lost >= Crs) {
        if (lane < nM) cf = eval_node(mrow, p, P, ct) && ds_eval(s_dc[lane], dp, DP, craw);
        have_cur = true;
        const uint32_t cm = wave_max_u32(cf ? (uint32_t)craw + 1u : 0u);
        // the normalization changed: every key of the round's lists is stale
        if (cm > Mrs || (lost >= Crs && cm != Mrs)) break;
      }
    }
    const uint32_t Mj = Mrs ? Mrs - 1u : 0u;
    const uint32_t node = key_node(key);
    const bool unmod = (key != 0) && !((bitmap[node >> 5] >> (node & 31)) & 1u);
    const uint64_t um = __ballot(unmod);
    const int pos = um ? (int)__builtin_ctzll(um) : kC;
    uint64_t best = um ? readlane_u64(key, pos) : 0;
    // With M_j = the round-start M every plugin term is monotone (an assume only lowers a node's key), so a
    // modified row can only beat the best unmodified candidate when that is not the pod's overall top key.
    if (nM > 0 && (pos != 0 || most)) {
      if (!have_cur && lane < nM) cf = eval_node(mrow, p, P, ct) && ds_eval(s_dc[lane], dp, DP, craw);
      const uint64_t mk = cf ? make_key(ct + (DP.score ? DP.weight * ds_normalized(craw, Mj) : 0), midx) : 0;
      const uint64_t mbest = wave_max_key(mk);
      best = mbest > best ? mbest : best;
    }
    if (best < ub) break;
    ++consumed;
    if (best == 0) {
      my_out = lane == j ? 0 : my_out;
      my_minors = lane == j ? 0 : my_minors;
      continue;
    }
    const uint32_t w = key_node(best);
    const uint64_t hit = __ballot((lane < nM) & (midx == w));
    const int owner = hit ? (int)__builtin_ctzll(hit) : nM;
    if (!hit) {
      const uint64_t sh = __ballot(stg_node == w);  // a pod whose top candidate is w staged its row
      const int src = sh ? (int)__builtin_ctzll(sh) : -1;
      if (lane == owner) {  // copy the row straight into the lane's LDS slots (memcpy: alias-safe, no private copy)
        midx = w;
        const DsNode* from = src >= 0 ? reinterpret_cast<const DsNode*>(s_stg) + src : DT.d + w;
        mrow = src >= 0 ? s_srow[src] : load_row(T, w);
        __builtin_memcpy(&s_dc[owner], from, sizeof(DsNode));
        if (sharded) {
          s_r0[owner] = mrow;
          __builtin_memcpy(&s_d0[owner], from, sizeof(DsNode));
        }
      }
      if (lane == 0) bitmap[w >> 5] |= 1u << (w & 31);
      ++nM;
    }
    __syncthreads();
    // Reserve: DeviceShare allocates the minors (wave-parallel: lane m scores minor m of the winner's row), then
    // the assume.  A failed Reserve leaves the pod unplaced and the node unchanged.
    int placed = 0, minors = 0;
    {
      DsNode& dn = s_dc[owner];
      if (dp.skip || !dn.has_device) {
        placed = 1;
      } else if (!dp.error) {
        const DsInst in = ds_instance(dn, dp);
        if (in.ok) {
          bool fit = false, nz = false;
          const int64_t sc = lane < kMinors ? ds_minor(dn, lane, in, DP, fit, nz) : 0;
          fit &= lane < kMinors;
          const uint64_t fits = __ballot(fit);
          if (__ballot(nz && lane < kMinors) != 0 && __popcll(fits) >= in.count) {
            uint32_t taken = 0;
            for (int k = 0; k < in.count; ++k) {  // (score desc, minor asc): max of score << 4 | (15 - minor)
              const bool cand = fit && !((taken >> (lane & 31)) & 1u);
              const uint32_t v = cand ? ((uint32_t)sc << 4) | (uint32_t)(15 - lane) : 0u;
              taken |= 1u << (15 - (int)(wave_max_u32(v) & 15u));
            }
            if (lane < kMinors && ((taken >> lane) & 1u)) {
              dn.ucore[lane] += (int32_t)in.core;
              dn.uratio[lane] += (int32_t)in.ratio;
              dn.umem[lane] += in.mem;
            }
            placed = 1;
            minors = (int)taken;
          }
        }
      }
    }
    if (placed && lane == owner) {
      mrow.req_cpu += p.req_cpu;  // NodeInfo.AddPod + LoadAware assign cache
      mrow.req_mem += p.req_mem;
      mrow.nz_cpu += p.nz_cpu;
      mrow.nz_mem += p.nz_mem;
      mrow.la_used_cpu += p.est_cpu;
      mrow.la_used_mem += p.est_mem;
      if (p.flags & P_PROD) {
        mrow.la_pused_cpu += p.est_cpu;
        mrow.la_pused_mem += p.est_mem;
      }
      mrow.num_pods += 1;
      touched = true;
    }
    placed = __builtin_amdgcn_readlane(placed, owner);
    minors = __builtin_amdgcn_readlane(minors, owner);
    if (placed && p.quota >= 0 && lane == 0) quota_row_charge(s_q[p.quota], qr, (p.flags & P_NONPREEMPT) != 0);
    my_out = lane == j ? (placed ? best : 0) : my_out;
    my_minors = lane == j ? (placed ? minors : 0) : my_minors;
    __syncthreads();
  }
  if (touched) {
    store_mutable(T, midx, mrow);
    __builtin_memcpy(DT.d + midx, &s_dc[lane], sizeof(DsNode));
  }
  if (lane < consumed) {
    out_keys[first + lane] = my_out;
    out_minors[first + lane] = my_minors;
  }
  if (nq > 0) {
    const uint64_t* sq = reinterpret_cast<const uint64_t*>(s_q);
    uint64_t* qw = reinterpret_cast<uint64_t*>(quotas);
    for (int w = lane; w < nq * (int)(sizeof(QuotaRow) / 8); w += kWave) qw[w] = sq[w];
  }
  __threadfence();
  if (lane == 0) {
    ctl[0] = first + consumed;
    ctl[1] += 1;
    ctl[2] += consumed;
    ctl[8] += (int64_t)(__builtin_amdgcn_s_memrealtime() - t_active);
  }
}

// kg_pods_evaluate_device: DeviceShare Filter + raw Score of one pod on every node (the plugin alone)
__global__ void evaluate_pod_ds(DsTable DT, const DsPod* __restrict__ pod, int64_t n, DsParams DP,
                                int32_t* __restrict__ pass, int64_t* __restrict__ score,
                                const DsXNode* __restrict__ dsx) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int64_t raw = 0, xraw = 0;
  const DsNode& d = DT.d[i];
  // (ABI 17) the RDMA / FPGA types too: AutopilotAllocator allocates every requested type, score sums them
  const bool ok = ds_eval(d, *pod, DP, raw) && ds_eval_x(dsx[i], d.has_device != 0, *pod, DP, xraw);
  raw += xraw;
  pass[i] = ok ? 1 : 0;
  score[i] = ok ? raw : 0;
}

// kg_pods_evaluate_reservation: the exact pass's per-node evaluation of one pod (restore, every Filter, nomination,
// raw Scores) with the restore's state; KG_RSV_EVAL_WORDS int64 per node
__global__ void evaluate_pod_rsv(DevTable T, const RsvNode* __restrict__ RN, const int32_t* __restrict__ rsv_n,
                                 const DevPod* __restrict__ pod, const RsvPod* __restrict__ rpod,
                                 const DsPod* __restrict__ dpod, const NumaPod* __restrict__ npod, int64_t n,
                                 EvalParams P, RsvParams RP, RsvExt X, int64_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  RsvDbg d;
  const RsvOut o = rsv_eval_node(T, RN, rsv_n, i, *pod, *rpod, P, RP, X, dpod, npod, &d);
  int64_t* w = out + (size_t)i * KG_RSV_EVAL_WORDS;
  w[0] = o.feas ? 1 : 0;
  w[1] = o.feas ? o.nom : -1;
  w[2] = o.feas ? o.raw : 0;
  w[3] = d.has_state;
  w[4] = d.matched;
  w[5] = d.req_cpu, w[6] = d.req_mem, w[7] = d.nz_cpu, w[8] = d.nz_mem, w[9] = d.num_pods;
  w[10] = d.pod_req_cpu, w[11] = d.pod_req_mem;
  w[12] = o.feas ? o.base : 0;
  w[13] = o.feas ? o.dsraw : 0;
  w[14] = o.order == 0x7fffffff ? 0 : o.order;
  w[15] = 0;
}

// The preemption dry run on the device (kg_pods_filter_preemption, r5 kg_pods_select_victims): a candidate node's
// restored NodeInfo copy minus its victims (NodeInfo.RemovePod) with the Reservation plugin's PreFilterExtensions
// (reservation/plugin.go:253-310: RemovePod adds a non-reserve victim's non-zero requests to state.preemptible[node], or
// to preemptibleInRRs[node][its reservation]; AddPod subtracts them again; either sets the map entry), then the pod's
// Filters on it: NodeResourcesFit + LoadAware (eval_node), the ephemeral-storage / scalar fit on the victim-free
// Requested, and the Reservation Filter with the preemptible amounts (:357-428, fitsNode :433-482).
struct Victim {
  int64_t req_cpu, req_mem, nz_cpu, nz_mem;
  int64_t aux[kAux];  // ephemeral-storage and the scalar resources (KG_RES_EPHEMERAL ..)
  int32_t slot;       // the node's reservation slot the victim was allocated from, -1 = none
  int32_t nonzero;    // counted by RemovePod / AddPod: !quotav1.IsZero(PodRequestsAndLimits) and not a reserve pod
  int32_t dminors;    // (r6) the minors of its DeviceShare allocation (nodeDevice.getUsed of the victim), 0 = none: GPU
                      // bits 0-7, (ABI 17) RDMA 8-15, FPGA 16-23
  int32_t reserve;    // (r6) a reserve pod (DeviceShare's AddPod / RemovePod return before counting it)
  DsPod dp;           // (r6) its DeviceShare request (the per-instance allocation on each minor, ds_instance)
};
// (r6) the dry run's Filters of the other accelerated plugins (nullptr: the plugin is not in the profile)
struct PreExt {
  const NumaStatic* __restrict__ ns;  // NodeNUMAResource: no PreFilterExtensions (plugin.go:272-274), so the victims'
  const NumaMut* __restrict__ nm;     // cpusets stay allocated; its Filter reads the victim-free NodeInfo.Requested
  NumaParams NP;
  NumaPod np;
  const DsNode* __restrict__ ds;      // DeviceShare: AddPod / RemovePod (deviceshare/plugin.go:163-278) move the
  const DsXNode* __restrict__ dsx;    // victims' allocations in / out of preemptibleDevices[node] ((ABI 17) RDMA /
  DsParams DP;                        // FPGA too)
  DsPod dp;
  const NodePred* __restrict__ pred;  // TaintToleration / NodeAffinity: node-static Filters
  DefParams DF;
  DefPod df;
};
struct PreNode {
  Row r;
  RsvNode rn;
  uint32_t mm;
  int nm;
  int64_t pr_c, pr_m, ra_c, ra_m;
  bool has_state;
  int64_t aux_req[kAux];                          // Requested of the aux resources, victims removed
  int64_t pre_c, pre_m, pre_aux[kAux];            // state.preemptible[node]
  int64_t rr_c[kRsvSlots], rr_m[kRsvSlots], rr_aux[kRsvSlots][kAux];  // preemptibleInRRs[node][slot]
  bool pre_set;
  uint32_t rr_set;
  int64_t dpre[kMinors][3];  // (r6) DeviceShare preemptibleDevices[node]: gpu-core, gpu-memory, gpu-memory-ratio
  int32_t xpre[kXTypes][kMinors];  // (ABI 17) and its RDMA / FPGA part
};

// BeforePreFilter's restore of node i for the pod (the same rsv_restore as the scheduling passes); false: invalid node
__device__ bool pre_node_init(PreNode& S, const DevTable& T, const RsvNode* __restrict__ RN,
                              const int32_t* __restrict__ rsv_n, const uint64_t* __restrict__ rsv_pred,
                              const RsvSel* __restrict__ rsel, int64_t i, const RsvPod& rp, int rsv_on) {
  S.r = load_row(T, i);
  if (!(S.r.flags & F_VALID)) return false;
  S.mm = 0;
  S.nm = 0;
  S.pr_c = S.pr_m = S.ra_c = S.ra_m = 0;
  S.has_state = false;
  const int ns = rsv_on ? rsv_n[i] : 0;
  if (ns > 0) {
    S.rn = RN[i];
    rsv_restore(S.rn, ns, rp, rsv_pred + (size_t)i * kRsvSlots, (rp.flags & RP_SEL) ? rsel : nullptr, S.r, S.mm, S.nm,
                S.pr_c, S.pr_m, S.ra_c, S.ra_m, S.has_state);
  }
#pragma unroll
  for (int q = 0; q < kAux; ++q) {
    S.aux_req[q] = T.aux ? T.aux[(size_t)(kAux + q) * T.cap + i] : 0;
    S.pre_aux[q] = 0;
  }
  S.pre_c = S.pre_m = 0;
  for (int s = 0; s < kRsvSlots; ++s) {
    S.rr_c[s] = S.rr_m[s] = 0;
#pragma unroll
    for (int q = 0; q < kAux; ++q) S.rr_aux[s][q] = 0;
  }
  S.pre_set = false;
  S.rr_set = 0;
#pragma unroll
  for (int m = 0; m < kMinors; ++m) S.dpre[m][0] = S.dpre[m][1] = S.dpre[m][2] = 0;
#pragma unroll
  for (int t = 0; t < kXTypes; ++t)
#pragma unroll
    for (int m = 0; m < kMinors; ++m) S.xpre[t][m] = 0;
  return true;
}

// sign +1: NodeInfo.RemovePod + RemovePod; −1: NodeInfo.AddPodInfo + AddPod
__device__ __forceinline__ void pre_node_apply(PreNode& S, const Victim& v, int64_t sign, const PreExt* X = nullptr,
                                               int64_t i = 0) {
  // (r6) DeviceShare's RemovePod / AddPod (deviceshare/plugin.go:163-278): a victim outside any reservation (rInfo nil)
  // moves its allocation into / out of preemptibleDevices[node] (appendAllocated / subtractAllocated), unless it is a
  // reserve pod or the preemptor requests no devices (state.skip)
  if (X && X->ds && !X->dp.skip && v.dminors != 0 && !v.reserve && v.slot < 0) {
    const int32_t gm = v.dminors & 0xFF;
    const DsInst in = gm && !v.dp.nogpu ? ds_instance(X->ds[i], v.dp) : DsInst{0, 0, 0, 0, 0};
    if (in.ok)
#pragma unroll
      for (int m = 0; m < kMinors; ++m)
        if ((gm >> m) & 1) {
          S.dpre[m][0] += sign * in.core;
          S.dpre[m][1] += sign * in.mem;
          S.dpre[m][2] += sign * in.ratio;
        }
#pragma unroll
    for (int t = 0; t < kXTypes; ++t) {  // (ABI 17) its RDMA / FPGA minors: the per-instance request on each
      const uint32_t xm = ((uint32_t)v.dminors >> (8 * (t + 1))) & 0xFFu;
      if (!xm || v.dp.xq[t] == 0) continue;
      int32_t count, per;
      dsx_inst(v.dp.xq[t], count, per);
#pragma unroll
      for (int m = 0; m < kMinors; ++m)
        if ((xm >> m) & 1u) S.xpre[t][m] += (int32_t)sign * per;
    }
  }
  S.r.req_cpu -= sign * v.req_cpu;
  S.r.req_mem -= sign * v.req_mem;
  S.r.nz_cpu -= sign * v.nz_cpu;
  S.r.nz_mem -= sign * v.nz_mem;
  S.r.num_pods -= sign;
#pragma unroll
  for (int q = 0; q < kAux; ++q) S.aux_req[q] -= sign * v.aux[q];
  if (!v.nonzero) return;
  if (v.slot >= 0 && v.slot < kRsvSlots) {
    S.rr_c[v.slot] += sign * v.req_cpu;
    S.rr_m[v.slot] += sign * v.req_mem;
#pragma unroll
    for (int q = 0; q < kAux; ++q) S.rr_aux[v.slot][q] += sign * v.aux[q];
    S.rr_set |= 1u << v.slot;
  } else {
    S.pre_c += sign * v.req_cpu;
    S.pre_m += sign * v.req_mem;
#pragma unroll
    for (int q = 0; q < kAux; ++q) S.pre_aux[q] += sign * v.aux[q];
    S.pre_set = true;
  }
}

// the pod's Filters on the candidate's current NodeInfo copy: 0 or KG_REJECT_* bits.  rq: the pod's kAux requests.
__device__ uint32_t pre_node_filter(const DevTable& T, const PreNode& S, int64_t i, const DevPod& p,
                                    const int64_t (&rq)[kAux], const RsvPod& rp, const EvalParams& P,
                                    const RsvParams& RP, int rsv_on, const PreExt* X = nullptr) {
  uint32_t rej = 0;
  int64_t t = 0;
  Row r = S.r;
  r.flags &= ~F_EPH_OVER;  // recomputed below from the victim-free Requested
  (void)eval_node(r, p, P, t, &rej);  // NodeResourcesFit + LoadAware Filter verdicts
  bool any_aux = false;
#pragma unroll
  for (int q = 0; q < kAux; ++q) any_aux |= rq[q] != 0;
  const bool zero = (p.flags & P_ZERO_REQ) != 0;
  if (P.fit_filter && !zero && T.aux) {  // fitsRequest: ephemeral-storage always, a scalar only when requested
#pragma unroll
    for (int q = 0; q < kAux; ++q)
      if ((q == 0 || rq[q] != 0) && rq[q] > T.aux[(size_t)q * T.cap + i] - S.aux_req[q]) rej |= KG_REJECT_FIT_OTHER;
  }
  if (rsv_on && RP.filter) {
    const RsvNode& rn = S.rn;
    const bool required = (rp.flags & RP_AFFINITY) != 0;
    const bool rzero = p.req_cpu == 0 && p.req_mem == 0 && !any_aux;
    // fitsNode with rInfo = slot s (s < 0: nil) and preemptible (pc, pm, pa); a node without state has no podRequested.
    // A reservation holds cpu / memory only (its Allocatable / Allocated of the aux resources are 0), and
    // podRequested's aux part is the node's Requested at restore time (T.aux), which the victims do not change.
    auto fits_node = [&](int s, int64_t pc, int64_t pm, const int64_t* pa) {
      if (r.num_pods - S.nm + 1 > r.alloc_pods) return false;
      if (rzero) return true;
      const int64_t rc = s >= 0 ? rsv_nn(rn.alloc_cpu[s], rn.allocd_cpu[s]) : 0;
      const int64_t rm = s >= 0 ? rsv_nn(rn.alloc_mem[s], rn.allocd_mem[s]) : 0;
      const int64_t prc = S.has_state ? S.pr_c : 0, prm = S.has_state ? S.pr_m : 0;
      if (p.req_cpu > r.alloc_cpu - (prc - rc - S.ra_c - pc)) return false;
      if (p.req_mem > r.alloc_mem - (prm - rm - S.ra_m - pm)) return false;
      if (T.aux) {
        for (int q = 0; q < kAux; ++q) {
          if (q > 0 && rq[q] == 0) continue;  // ScalarResources: the pod's request keys only
          const int64_t pra = S.has_state ? T.aux[(size_t)(kAux + q) * T.cap + i] : 0;
          if (rq[q] > T.aux[(size_t)q * T.cap + i] - (pra - pa[q])) return false;
        }
      }
      return true;
    };
    bool ok = true;
    if (S.mm == 0 || !S.has_state) {
      if (required) ok = false;
      else if (S.pre_set || S.rr_set) ok = fits_node(-1, S.pre_c, S.pre_m, S.pre_aux);
    } else {
      const bool kc = (p.flags & P_CPU_KEY) != 0, km = (p.flags & P_MEM_KEY) != 0;
      bool sat = false;
      for (int s = 0; s < kRsvSlots && !sat; ++s) {
        if (!(S.mm >> s & 1)) continue;
        const bool hc = rn.alloc_cpu[s] > 0, hm = rn.alloc_mem[s] > 0;
        if (!((kc && hc) || (km && hm))) continue;  // Intersection(rInfo.ResourceNames, pod request names) empty
        int64_t pa[kAux];
#pragma unroll
        for (int q = 0; q < kAux; ++q) pa[q] = S.rr_aux[s][q] + S.pre_aux[q];
        const bool fits = fits_node(s, S.rr_c[s] + S.pre_c, S.rr_m[s] + S.pre_m, pa);
        if (((rn.meta[s] >> 4) & 3) == KG_RSV_POLICY_RESTRICTED) {
          int64_t ac = rn.allocd_cpu[s], am = rn.allocd_mem[s];
          if (S.rr_set >> s & 1) {  // Allocated − preemptibleInRR, non-negative, masked to the reservation's keys
            ac = hc ? rsv_nn(ac, S.rr_c[s]) : 0;
            am = hm ? rsv_nn(am, S.rr_m[s]) : 0;
          }
          const int64_t rc = rsv_nn(rn.alloc_cpu[s], ac), rm = rsv_nn(rn.alloc_mem[s], am);
          sat = fits && (!hc || !kc || p.req_cpu <= rc) && (!hm || !km || p.req_mem <= rm);
        } else {
          sat = fits;
        }
      }
      ok = sat || !required;
    }
    if (!ok) rej |= KG_REJECT_RESERVATION;
  }
  if (X) {
    if (X->pred) {  // TaintToleration / NodeAffinity Filter (defaults_filter, split into their reject bits)
      const NodePred n = X->pred[i];
      const DefPod& d = X->df;
      if (X->DF.taint_filter && (n.hard & ~d.tol) != 0) rej |= KG_REJECT_TAINT;
      if (X->DF.aff_filter) {
        bool ok = (n.pred & d.sel) == d.sel;
        if (ok && d.nreq > 0) {
          bool any = false;
#pragma unroll
          for (int k = 0; k < kAffTerms; ++k) any |= k < d.nreq && term_holds(n.pred, d.req[k]);
          ok = any;
        }
        if (!ok) rej |= KG_REJECT_NODE_AFFINITY;
      }
    }
    if (X->ns && X->NP.filter) {  // NodeNUMAResource Filter on the node's own NodeAllocation, victim-free Requested
      const NumaView v = make_view(X->ns + i, X->nm + i, X->NP);
      NumaHint aff;
      if (!numa_filter(v, X->np, X->NP, aff, S.r.req_cpu, S.r.alloc_cpu)) rej |= KG_REJECT_NUMA;
    }
    if (X->ds && X->DP.filter && !X->dp.skip) {
      // calcFreeWithPreemptible (device_cache.go:314-342): free = total − max(0, used − preemptible) on every minor
      DsNode d = X->ds[i];
#pragma unroll
      for (int m = 0; m < kMinors; ++m) {
        const int64_t c = (int64_t)d.ucore[m] - S.dpre[m][0], b = d.umem[m] - S.dpre[m][1],
                      r = (int64_t)d.uratio[m] - S.dpre[m][2];
        d.ucore[m] = (int32_t)(c > 0 ? c : 0);
        d.umem[m] = b > 0 ? b : 0;
        d.uratio[m] = (int32_t)(r > 0 ? r : 0);
      }
      int64_t raw = 0;
      if (!ds_eval(d, X->dp, X->DP, raw)) rej |= KG_REJECT_DEVICE;
      else if (X->dsx && (X->dp.xq[0] | X->dp.xq[1]) &&
               !ds_eval_x(X->dsx[i], d.has_device != 0, X->dp, X->DP, raw, S.xpre))
        rej |= KG_REJECT_DEVICE;
    }
  }
  return rej;
}

// kg_pods_filter_preemption: one (pod, node) with every victim removed (one thread)
__global__ void filter_pod_preempt(DevTable T, const RsvNode* __restrict__ RN, const int32_t* __restrict__ rsv_n,
                                   const uint64_t* __restrict__ rsv_pred, const RsvSel* __restrict__ rsel, int64_t i,
                                   const DevPod* __restrict__ pod, const int64_t* __restrict__ pod_aux, RsvPod rp,
                                   EvalParams P, RsvParams RP, int rsv_on, const Victim* __restrict__ vic,
                                   int64_t n_vic, int32_t* __restrict__ out, PreExt X) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  PreNode S;
  if (!pre_node_init(S, T, RN, rsv_n, rsv_pred, rsel, i, rp, rsv_on)) {
    *out = KG_REJECT_INVALID_NODE;
    return;
  }
  const DevPod p = *pod;
  int64_t rq[kAux];
#pragma unroll
  for (int q = 0; q < kAux; ++q) rq[q] = pod_aux[q];
  for (int64_t k = 0; k < n_vic; ++k) pre_node_apply(S, vic[k], 1, &X, i);
  *out = (int32_t)pre_node_filter(T, S, i, p, rq, rp, P, RP, rsv_on, &X);
}

// (r5) kg_pods_select_victims: SelectVictimsOnNode for every candidate (one thread per candidate, the victims in the
// caller's reprieve order): remove every potential victim, Filter, then reprieve them one by one (add back, Filter,
// remove again as a victim when the pod no longer fits).  elasticquota/preempt.go:111-215; k8s defaultpreemption.
__global__ void select_victims(DevTable T, const RsvNode* __restrict__ RN, const int32_t* __restrict__ rsv_n,
                               const uint64_t* __restrict__ rsv_pred, const RsvSel* __restrict__ rsel,
                               const DevPod* __restrict__ pod, const int64_t* __restrict__ pod_aux, RsvPod rp,
                               EvalParams P, RsvParams RP, int rsv_on, int64_t n_cand, const int32_t* __restrict__ nodes,
                               const int64_t* __restrict__ off, const Victim* __restrict__ vic,
                               const uint8_t* __restrict__ violating, int32_t* __restrict__ out_reject,
                               uint8_t* __restrict__ out_victim, int32_t* __restrict__ out_violating, PreExt X) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n_cand) return;
  const int64_t i = nodes[c], k0 = off[c], k1 = off[c + 1];
  for (int64_t k = k0; k < k1; ++k) out_victim[k] = 0;
  out_violating[c] = 0;
  PreNode S;
  if (!pre_node_init(S, T, RN, rsv_n, rsv_pred, rsel, i, rp, rsv_on)) {
    out_reject[c] = KG_REJECT_INVALID_NODE;
    return;
  }
  if (k1 == k0) {  // "No victims found on node": UnschedulableAndUnresolvable, the node is not evaluated
    out_reject[c] = KG_REJECT_NO_VICTIMS;
    return;
  }
  const DevPod p = *pod;
  int64_t rq[kAux];
#pragma unroll
  for (int q = 0; q < kAux; ++q) rq[q] = pod_aux[q];
  for (int64_t k = k0; k < k1; ++k) pre_node_apply(S, vic[k], 1, &X, i);
  const uint32_t rej = pre_node_filter(T, S, i, p, rq, rp, P, RP, rsv_on, &X);
  out_reject[c] = (int32_t)rej;
  if (rej) return;
  int32_t nv = 0;
  for (int64_t k = k0; k < k1; ++k) {  // reprievePod, in order
    const Victim v = vic[k];
    pre_node_apply(S, v, -1, &X, i);
    if (pre_node_filter(T, S, i, p, rq, rp, P, RP, rsv_on, &X) != 0) {
      pre_node_apply(S, v, 1, &X, i);
      out_victim[k] = 1;
      nv += violating && violating[k] ? 1 : 0;
    }
  }
  out_violating[c] = nv;
}

// Scatter of upserted device rows
#include "xr_dev.h"

template <typename Rec>
__global__ void scatter_rows(Rec* __restrict__ dst, const Rec* __restrict__ src, const int32_t* __restrict__ idx,
                             int64_t n) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) dst[idx[k]] = src[k];
}

__global__ void scatter_ds(DsTable DT, const DsNode* __restrict__ s, const int32_t* __restrict__ idx, int64_t n) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  DT.d[idx[k]] = s[k];
}
__global__ void scatter_dsx(DsXNode* __restrict__ dst, const DsXNode* __restrict__ s, const int32_t* __restrict__ idx,
                            int64_t n) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  dst[idx[k]] = s[k];
}

// kg_pods_evaluate: one pod, every node, per-plugin outputs.
__global__ void evaluate_pod(DevTable T, const DevPod* __restrict__ pod, int64_t n, EvalParams P,
                             int32_t* __restrict__ reject, int64_t* __restrict__ fit, int64_t* __restrict__ la,
                             const int64_t* __restrict__ aux_req) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Row r = load_row(T, i);
  int64_t t = 0, fs = 0, ls = 0;
  uint32_t rej = 0;
  eval_node(r, *pod, P, t, &rej, &fs, &ls);
  if (P.fit_filter && (pod->flags & P_AUX) && (r.flags & F_VALID) && !aux_fits(T, i, aux_req)) rej |= 1u << 7;
  reject[i] = (int32_t)rej;
  fit[i] = fs;
  la[i] = ls;
}

// Scatter-add of mutable-column deltas (pod add/remove, NodeMetric usage changes).
struct RowDelta {
  int64_t idx;
  int64_t d[9];  // req_cpu, req_mem, nz_cpu, nz_mem, num_pods, la_used_cpu, la_used_mem, la_pused_cpu, la_pused_mem
  int64_t aux[kAux];  // Requested of the kAux resources
};
// The framework's Unreserve of placed staged pods idx[0..n) (kg_pods_unreserve), one thread in queue order: NodeInfo
// + the LoadAware assign cache, NodeNUMAResource Release, DeviceShare updateCacheUsed(add=false), Reservation
// forgetPod, ElasticQuota UnreservePod.  Each pod's decision is cleared, so a second Unreserve is a no-op.
__global__ void unreserve_pods(DevTable T, const DevPod* __restrict__ pods, const int64_t* __restrict__ idx, int64_t n,
                               uint64_t* __restrict__ out_keys, NumaMut* __restrict__ nm, uint64_t* __restrict__ out_cpus,
                               int64_t* __restrict__ out_nrec, DsNode* __restrict__ ds, const DsPod* __restrict__ dpods,
                               int32_t* __restrict__ out_minors, RsvNode* __restrict__ RN, int32_t* __restrict__ out_rslot,
                               QuotaRow* __restrict__ quotas, int nq, const int64_t* __restrict__ qdev,
                               const int64_t* __restrict__ paux, GroupTable G, const GroupPod* __restrict__ gpods,
                               int hard_w, RsvGpu* __restrict__ rg, RsvCpu* __restrict__ rcs,
                               DsXNode* __restrict__ dsx) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  for (int64_t k = 0; k < n; ++k) {
    const int64_t j = idx[k];
    const uint64_t key = out_keys[j];
    if (key == 0) continue;
    const int32_t gm = ds ? (out_minors[j] & 0xFF) : 0;  // the DeviceShare GPU allocation, before it is cleared below
    const uint32_t w = key_node(key);
    const DevPod p = pods[j];
    Row r = load_row(T, w);  // NodeInfo.RemovePod + podAssignCache.unAssign (pod_assign_cache.go:119-131)
    const int64_t prod = (p.flags & P_PROD) ? 1 : 0;
    r.req_cpu -= p.req_cpu;
    r.req_mem -= p.req_mem;
    r.nz_cpu -= p.nz_cpu;
    r.nz_mem -= p.nz_mem;
    r.la_used_cpu -= p.est_cpu;
    r.la_used_mem -= p.est_mem;
    r.la_pused_cpu -= prod * p.est_cpu;
    r.la_pused_mem -= prod * p.est_mem;
    r.num_pods -= 1;
    store_mutable(T, w, r);
    if (gpods) group_apply(G, w, gpods[j], -1, hard_w);  // the node's pod-group counters
    if (p.flags & P_AUX)  // ephemeral-storage / scalar Requested
      for (int q = 0; q < kAux; ++q) T.aux[(size_t)(kAux + q) * T.cap + w] -= paux[(size_t)j * kAux + q];
    uint64_t pc[kCpuWords] = {0, 0, 0, 0};  // the pod's cpuset, before it is cleared below
    if (nm) {  // nodenumaresource/plugin.go:417-425
      uint64_t* c = out_cpus + (size_t)j * kCpuWords;
      int64_t* rec = out_nrec + (size_t)j * kNumaRecWords;
      // (ABI 15) the cpus the node's reservations hold keep RefCount 1 (the reservation's)
      uint64_t keep[kCpuWords] = {0, 0, 0, 0};
      if (rcs && RN)
        for (int s = 0; s < kRsvSlots; ++s)
          if (RN[w].meta[s] & RS_CPUS)
            for (int q = 0; q < kCpuWords; ++q) keep[q] |= rcs[(size_t)w * kRsvSlots + s].r[q];
      for (int q = 0; q < kCpuWords; ++q) pc[q] = c[q];
      NumaMut m = nm[w];
      numa_release(m, c, rec, keep);
      nm[w] = m;
      for (int q = 0; q < kCpuWords; ++q) c[q] = 0;
      for (int q = 0; q < kNumaRecWords; ++q) rec[q] = 0;
    }
    if (ds && out_minors[j]) {  // deviceshare/plugin.go:440-455, SubtractWithNonNegativeResult per minor
      const DsPod dp = dpods[j];
      DsNode dn = ds[w];
      if (!dp.skip && !dp.error && !dp.nogpu && dn.has_device && gm) {
        const DsInst in = ds_instance(dn, dp);
        for (int m = 0; m < kMinors; ++m) {
          if (!((gm >> m) & 1)) continue;
          const int64_t c = dn.ucore[m] - in.core, q = dn.uratio[m] - in.ratio, b = dn.umem[m] - in.mem;
          dn.ucore[m] = (int32_t)(c > 0 ? c : 0);
          dn.uratio[m] = (int32_t)(q > 0 ? q : 0);
          dn.umem[m] = b > 0 ? b : 0;
        }
        ds[w] = dn;
      }
      // (ABI 17) the RDMA / FPGA minors of the packed record
      if (dsx && ((uint32_t)out_minors[j] >> 8)) ds_release_x(dsx[w], dp, out_minors[j]);
      out_minors[j] = 0;
    }
    if (RN && out_rslot[j] >= 0) {  // reservation/plugin.go:561-583 → RemoveAssignedPod (reservation_info.go:328-339)
      const int s = out_rslot[j];
      RsvNode& rn = RN[w];
      // (ABI 13) its allocation on a GPU-holding reservation's minors leaves the restore's `allocated`
      // (deviceshare/reservation.go:150-155)
      if (rg && gm > 0 && (rn.meta[s] & RS_GPU))
        rsv_gpu_assign(rg[(size_t)w * kRsvSlots + s], ds_instance(ds[w], dpods[j]), gm, -1);
      // (ABI 15) the pod leaves AssignedPods: its cpus are the reservation's reserved cpus again
      if (rcs && (rn.meta[s] & RS_CPUS))
        for (int q = 0; q < kCpuWords; ++q) rcs[(size_t)w * kRsvSlots + s].u[q] &= ~pc[q];
      if (rn.assigned[s] > 0) {
        if (rn.alloc_cpu[s] > 0) rn.allocd_cpu[s] = rn.allocd_cpu[s] > p.req_cpu ? rn.allocd_cpu[s] - p.req_cpu : 0;
        if (rn.alloc_mem[s] > 0) rn.allocd_mem[s] = rn.allocd_mem[s] > p.req_mem ? rn.allocd_mem[s] - p.req_mem : 0;
        rn.assigned[s] -= 1;
      }
      out_rslot[j] = -1;
    }
    if (nq > 0 && p.quota >= 0) {  // elasticquota/plugin.go:348-360 → UnreservePod (addUsedNonNegativeNoLock)
      const QuotaReq rq = quota_req(p, qdev ? qdev + (size_t)j * kQuotaRes : nullptr);
      QuotaRow& Q = quotas[p.quota];
      const bool np = (p.flags & P_NONPREEMPT) != 0;
      for (int d = 0; d < kQuotaRes; ++d) {
        Q.used[d] = Q.used[d] > rq.r[d] ? Q.used[d] - rq.r[d] : 0;
        if (np) Q.np[d] = Q.np[d] > rq.r[d] ? Q.np[d] - rq.r[d] : 0;
      }
    }
    out_keys[j] = 0;
  }
}

// F_EPH_OVER of every node from its ephemeral-storage Allocatable / Requested columns (aux slot 0)
__global__ void refresh_eph_flags(DevTable T, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const bool over = T.aux[(size_t)kAux * T.cap + i] > T.aux[i];
  T.flags[i] = (T.flags[i] & ~F_EPH_OVER) | (over ? F_EPH_OVER : 0u);
}

__global__ void apply_deltas(DevTable T, const RowDelta* __restrict__ d, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const RowDelta x = d[i];
  const int64_t k = x.idx;
  atomicAdd((unsigned long long*)&T.req_cpu[k], (unsigned long long)x.d[0]);
  atomicAdd((unsigned long long*)&T.req_mem[k], (unsigned long long)x.d[1]);
  atomicAdd((unsigned long long*)&T.nz_cpu[k], (unsigned long long)x.d[2]);
  atomicAdd((unsigned long long*)&T.nz_mem[k], (unsigned long long)x.d[3]);
  atomicAdd(&T.num_pods[k], (int32_t)x.d[4]);
  atomicAdd((unsigned long long*)&T.la_used_cpu[k], (unsigned long long)x.d[5]);
  atomicAdd((unsigned long long*)&T.la_used_mem[k], (unsigned long long)x.d[6]);
  atomicAdd((unsigned long long*)&T.la_pused_cpu[k], (unsigned long long)x.d[7]);
  atomicAdd((unsigned long long*)&T.la_pused_mem[k], (unsigned long long)x.d[8]);
#pragma unroll
  for (int r = 0; r < kAux; ++r)
    if (x.aux[r]) atomicAdd((unsigned long long*)&T.aux[(size_t)(kAux + r) * T.cap + k], (unsigned long long)x.aux[r]);
}

__device__ __forceinline__ bool eval_hot_rt(const DevTable& T, int64_t i, const DevPod& p, const EvalParams& P,
                                            uint32_t& t, bool& rare) {
  const int pf = (P.fit_filter ? PF_FIT_FILTER : 0) | (P.fit_score ? PF_FIT_SCORE : 0) |
                 (P.la_filter ? PF_LA_FILTER : 0) | (P.la_score ? PF_LA_SCORE : 0) |
                 (P.la_score && P.la_prod_score ? PF_LA_PROD : 0);
  switch (pf) {
#define KG_CASE(X)                                   \
  case X: {                                          \
    const HotRow h = load_hot<X>(T, i, P);           \
    rare = (h.flags & F_RARE) != 0;                  \
    return eval_hot<X>(h, p, P, t);                  \
  }
    KG_CASE(0) KG_CASE(1) KG_CASE(2) KG_CASE(3) KG_CASE(4) KG_CASE(5) KG_CASE(6) KG_CASE(7)
    KG_CASE(8) KG_CASE(9) KG_CASE(10) KG_CASE(11) KG_CASE(12) KG_CASE(13) KG_CASE(14) KG_CASE(15)
    KG_CASE(24) KG_CASE(25) KG_CASE(26) KG_CASE(27) KG_CASE(28) KG_CASE(29) KG_CASE(30) KG_CASE(31)
#undef KG_CASE
  }
  return false;
}

__device__ __forceinline__ bool eval_fast_rt(const EvalRow& n, const DevPod& p, const EvalParams& P, uint32_t& t,
                                             bool& rare) {
  const int pf = (P.fit_filter ? PF_FIT_FILTER : 0) | (P.fit_score ? PF_FIT_SCORE : 0) |
                 (P.la_filter ? PF_LA_FILTER : 0) | (P.la_score ? PF_LA_SCORE : 0);
  switch (pf) {
#define KG_CASE(X) \
  case X:          \
    return eval_fast<X>(n, p, P, t, rare);
    KG_CASE(0) KG_CASE(1) KG_CASE(2) KG_CASE(3) KG_CASE(4) KG_CASE(5) KG_CASE(6) KG_CASE(7)
    KG_CASE(8) KG_CASE(9) KG_CASE(10) KG_CASE(11) KG_CASE(12) KG_CASE(13) KG_CASE(14) KG_CASE(15)
#undef KG_CASE
  }
  return false;
}

// Both evaluation paths on every (pod, node): eval_node (reference-shaped) vs eval_fast (hoisted terms).
__global__ void debug_eval_paths(DevTable T, const DevPod* __restrict__ pods, int64_t n_pods, int64_t n,
                                 EvalParams P, unsigned long long* __restrict__ mismatches) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Row r = load_row(T, i);
  const EvalRow er = make_eval_row(r, P);
  unsigned long long bad = 0;
  for (int64_t k = 0; k < n_pods; ++k) {
    int64_t t1 = 0;
    uint32_t t2 = 0;
    const bool f1 = eval_node(r, pods[k], P, t1);
    bool rare = false;
    const bool f2 = eval_fast_rt(er, pods[k], P, t2, rare);
    bad += !rare && ((f1 != f2) || (f1 && (uint32_t)t1 != t2));
    uint32_t t3 = 0;
    bool rare3 = false;
    const bool f3 = eval_hot_rt(T, i, pods[k], P, t3, rare3);
    bad += !rare3 && ((f1 != f3) || (f1 && (uint32_t)t1 != t3));
  }
  if (bad) atomicAdd(mismatches, bad);
}

// kg_debug_numa_merge: one case per thread through policy_merge, the merge numa_admit runs.  Case layout
// (KG_DBG_MERGE_WORDS int64): policy, NUMA node count, list count (1..2), then per list {positions, preferred
// positions, nil, nil preferred, empty}, then the hint score of each mask 0..15.  Out: admit, nil, mask, preferred,
// score (8 words per case).
__global__ void debug_numa_merge(const int64_t* __restrict__ in, int64_t n, int64_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t* c = in + (size_t)i * KG_DBG_MERGE_WORDS;
  HintList L[2];
#pragma unroll
  for (int l = 0; l < 2; ++l)
    L[l] = HintList{(uint32_t)c[3 + 5 * l], (uint32_t)c[4 + 5 * l], (int)c[5 + 5 * l], (int)c[6 + 5 * l],
                    (int)c[7 + 5 * l]};
  const int64_t* sc = c + 13;
  const auto score_of = [&](uint32_t m) -> int { return (int)sc[m & 15u]; };
  NumaHint best;
  const bool admit = policy_merge((int)c[0], (1u << (int)c[1]) - 1u, L[0], L[1], (int)c[2], score_of, best);
  int64_t* o = out + (size_t)i * 8;
  o[0] = admit;
  o[1] = best.nil;
  o[2] = best.mask;
  o[3] = best.preferred;
  o[4] = best.score;
}

__global__ void debug_least_requested(const int64_t* req, const int64_t* cap, int64_t* out, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = least_requested(req[i], cap[i]);
}

__global__ void debug_fast_lrs(const int64_t* req, const int64_t* cap, int64_t* out_cpu, int64_t* out_mem, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t c = cap[i], fr = c - req[i];
  // the wide pass's in-kernel estimates (load_hot), and for memory also the correctly rounded column value the exact
  // paths use: both must give the same quotient (-2 flags a disagreement)
  const double invd = c > 0 ? 100.0 / (double)c : 0.0;
  out_cpu[i] = cpu_dom(c, fr) ? lrs_cpu((int32_t)fr, (int32_t)c, inv100_f32(c)) : -1;
  if (mem_dom(c, fr)) {
    const int32_t a = lrs_mem((double)fr, (double)c, inv100_f64(c)), b = lrs_mem((double)fr, (double)c, invd);
    out_mem[i] = a == b ? a : -2;
  } else {
    out_mem[i] = -1;
  }
}

// ------------------------------------------------------------------------------------------------
// Host side
// ------------------------------------------------------------------------------------------------

// KG_DEBUG_POISON=1 (debug runs only): every fresh device buffer is filled with 0xA5 bytes before use, so a read of
// memory the engine never wrote shows up as a wrong answer instead of inheriting a freed buffer's old contents.
bool debug_poison() {
  const char* v = std::getenv("KG_DEBUG_POISON");
  return v && v[0] == '1';
}

template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  int ensure(size_t want) {
    if (want <= n) return 0;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    if (hipMalloc(&p, std::max<size_t>(want, 1) * sizeof(T)) != hipSuccess) return fail(KG_E_NOMEM, "hipMalloc %zu", want);
    n = want;
    if (debug_poison() && (hipMemset(p, 0xA5, n * sizeof(T)) != hipSuccess || hipDeviceSynchronize() != hipSuccess))
      return fail(KG_E_DEVICE, "poison fill");
    return 0;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
};

int64_t bits_for(int64_t v) {
  int b = 1;
  while (b < 32 && (int64_t(1) << b) <= v) ++b;
  return b;
}

}  // namespace

// In-process rank group (test hook, kg_engine_create_loopback): the ranks' exchange buffers and events, and a
// host barrier that pairs their exchanges call by call.
struct kg_loopback {
  int n = 0;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  bool failed = false;
  std::vector<kg_engine*> ranks;
  std::vector<const uint64_t*> buf;  // this exchange: each rank's buffer holding its record at [rank · cnt]
  std::vector<hipEvent_t> ready, done;
};

struct kg_engine {
  kg_config cfg;
  int rank = 0, n_ranks = 1;
  kg_loopback* lb = nullptr;  // test hook: exchanges through device copies instead of RCCL
  kg_exchange_fn xfn = nullptr;  // host collective (kg_engine_create_hosted): exchanges through the caller
  void* xuser = nullptr;
  std::vector<uint64_t> xsend, xrecv;
  hipEvent_t lb_ready = nullptr, lb_done = nullptr;
  int device = 0;
  hipStream_t stream = nullptr;
  ncclComm_t comm = nullptr;
  int64_t capacity = 0;
  int64_t n_nodes = 0;  // highest upserted index + 1
  EvalParams P{};
  // host mirror of static / ingest state
  std::vector<kg_node> nodes;
  std::vector<kg_node_metric> metrics;
  std::vector<int64_t> folded_usage;  // node-level term currently folded into la_used (2 per node): NodeUsage, or with
                                      // PodsMetric NodeUsage minus the estimated pods' usage + the pods' corrections
  std::vector<int64_t> folded_prod;   // the same for la_pused (the ScoreAccordingProdUsage view), 2 per node
  // podAssignCache mirror (pod_assign_cache.go:35-45) and NodeMetric.Status.PodsMetric per node: the PodsMetric
  // LoadAware Score terms (load_aware.go:283-376) are host-side functions of these, folded into la_used / la_pused
  struct AssignedPod {
    int64_t uid, time, est[2];
    int32_t prod;
  };
  struct PodMetricRec {
    int64_t uid, usage[2], present;
    int32_t prod;
  };
  std::vector<std::vector<AssignedPod>> assigned;
  std::vector<std::vector<PodMetricRec>> pmetrics;
  int64_t pm_nodes = 0;                  // nodes with a non-empty PodsMetric list
  std::vector<AssignedPod> staged_info;  // the staged pods' (uid, est, prod) for the mirror
  struct PendingPlace {
    int64_t first, count, time;
  };
  std::vector<PendingPlace> pending_place;  // scheduled staged ranges not yet in the mirror (flush_placements)
  std::vector<int64_t> now_of;        // metric ingest time per node
  bool static_dirty = true;
  // F_EPH_OVER (ephemeral-storage Requested > Allocatable) must be recomputed on the device: eph_any once any
  // ephemeral Requested delta was pushed, eph_dirty until the flags column has been refreshed since
  bool eph_any = false, eph_dirty = false;
  int64_t rounds_ahead = 256;  // rounds one host batch launches (adapted to how often rounds stop early)
  // scheduler clock for isNodeMetricExpired (kg_engine_set_clock): 0 = the newest now given to
  // kg_node_metrics_update, 1 = fixed, 2 = the host's real-time clock at every call
  int clock_mode = 0;
  int64_t clock_fixed = 0, clock_metrics = 0, clock_now = 0;
  DevBuf<int64_t> uidx;  // kg_pods_unreserve: staged pod indices
  // device
  DevTable T{};
  DevBuf<int64_t> cols64;
  std::vector<int64_t> h_aux;  // staging of the kAux Allocatable columns
  DevBuf<int64_t> paux;        // [pods][kAux] the staged pods' requests of the kAux resources
  DevBuf<int64_t> paux1;       // [kAux] the pod of a kg_pods_evaluate call
  DevBuf<int32_t> cols32;
  DevBuf<DevPod> pods;
  int64_t n_staged = 0;
  DevBuf<uint64_t> lists;     // [D][B][nt_local][kR] tile candidate lists (this rank), by round slot r % D
  DevBuf<uint64_t> gathered;  // [D][n_ranks][B][kCandStride] per-rank merged records (n_ranks > 1), by round slot
  DevBuf<uint64_t> cand;      // [D][B][kCandStride] final merged candidates, by round slot
  DevBuf<uint64_t> out_keys;
  DevBuf<int64_t> cursor;     // [0] cursor, [1] rounds, [2] consumed, [3] poison (int32 in its low word),
                              // [4] last published resolver sequence, [5] device error (chain wait timed out),
                              // [6] pods re-scored on the chain, [7] chain waits on a helper, [8] resolver active
                              // time (s_memrealtime ticks)
  DevBuf<int32_t> modlists;   // [kMaxDepth][kModListStride]: rows each round modified ([0] = count), by round slot
  DevBuf<uint32_t> tickets;   // (r5) [kMaxDepth][kMaxB]: fused-merge tickets per (round slot, pod group)
  // round r runs on rs[r % D] (eval → merge → [RCCL on comms[r % D]] → resolve); `stream` runs ingest
  hipStream_t rs[kMaxDepth] = {};
  ncclComm_t comms[kMaxDepth] = {};  // comms[0] = comm; one communicator per round stream
  hipEvent_t ev_res[kMaxDepth] = {};
  DevBuf<RowDelta> deltas;
  DevBuf<int64_t> scratch64;
  DevBuf<int32_t> scratch32;
  std::vector<int64_t> h_static64;
  std::vector<int32_t> h_static32;
  std::vector<double> h_static_f64;
  // NodeNUMAResource (profile enables it): per-node state, per-pod preFilterState, Reserve's cpusets
  bool numa_on = false;
  NumaParams NP{};
  DevBuf<NumaStatic> numa_s;
  DevBuf<NumaMut> numa_m;
  DevBuf<NumaPod> npods;
  DevBuf<uint64_t> out_cpus;  // [staged + kMaxB][4]
  DevBuf<int64_t> out_nrec;   // [staged + kMaxB][kNumaRecWords]: each pod's NUMA allocation (for Unreserve)
  // DeviceShare (profile enables it): per-node GPU state, per-pod preFilterState, Reserve's minors, round scratch
  bool ds_on = false;
  DsParams DP{};
  DevBuf<DsNode> ds_d;
  std::vector<DsNode> ds_host;
  DevBuf<DsXNode> dsx_d;                         // (ABI 17) RDMA / FPGA devices [cap]
  bool dsx_q = false;                            // (ABI 17) the staged queue holds RDMA / FPGA requests: per-pod pass
  DevBuf<DsPod> dpods;
  DevBuf<int32_t> out_minors;  // [staged + kMaxB]
  DevBuf<uint64_t> dsmax;      // [B][nt_local]
  DevBuf<uint64_t> dsnorm;     // [B]
  DevBuf<uint64_t> dsnorm_all; // [n_ranks][B]: every rank's shard maxima (several ranks)
  DevBuf<uint32_t> dsval;      // [B][nt_local·256]: packed (Fit+LoadAware total, raw DeviceShare) per (pod, node)
  // ElasticQuota admission table (kg_quotas_set)
  DevBuf<QuotaRow> quotas;     // [KG_MAX_QUOTAS] full kg_quota rows (cpu, memory, device resources)
  DevBuf<int64_t> qdev;        // [staged + kMaxB][kQuotaRes]: the pod's device requests (quota dims 2..7)
  int nq = 0;
  // Reservation (profile enables it): per-node slots, per-pod owner/affinity, Reserve's slots, pass scratch
  bool rsv_on = false;
  // the per-pod exact pass (rsv_eval / rsv_select / rsv_apply) runs the profile: Reservation, or NodeNUMAResource
  // together with DeviceShare (the reference's shipped profile, config/manager/scheduler-config.yaml:66-117)
  bool exact_on = false;
  DevBuf<uint32_t> numa_aff;  // exact pass: the NUMA affinity Filter stored per node for the pass's pod
  RsvParams RP{};
  DevBuf<RsvNode> rsv_d;
  DevBuf<RsvGpu> rsv_g;                         // (ABI 13) [cap][kRsvSlots] GPU holdings, allocated at the first GPU slot
  std::vector<uint8_t> rsv_gnode;               // per node: it has an RS_GPU slot
  int64_t rgpu_nodes = 0;                       // nodes with an RS_GPU slot (> 0 routes queues to the per-pod pass)
  int replica_ranks = 1;                        // (r6) ranks of the caller's group when this engine runs as a replica
  DevBuf<RsvCpu> rsv_c;                         // (ABI 15) [cap][kRsvSlots] cpusets, allocated at the first cpu slot
  std::vector<uint8_t> rsv_cnode;               // per node: it has an RS_CPUS slot
  int64_t rcpu_nodes = 0;                       // nodes with an RS_CPUS slot (> 0 routes queues to the per-pod pass)
  DevBuf<uint64_t> rsv_pd;      // [cap][kRsvSlots] (ABI 12) the slots' fakeNode predicates
  DevBuf<int32_t> rsv_nd;       // slots in use per node
  DevBuf<RsvPod> rpods;
  DevBuf<RsvSel> rsel;          // (ABI 12) [staged + kMaxB] reservation-affinity selectors (RsvPod::aux)
  DevBuf<int32_t> out_rslot;    // [staged + kMaxB]
  DevBuf<uint64_t> rsv_val;     // [capacity] packed per-node pass-1 values
  DevBuf<unsigned long long> rsv_ws;  // [8]: [3] = pod cursor, [4] = the call's end (graph launches)
  // the instantiated reservation group graph, reused while its launch arguments are unchanged
  hipGraphExec_t rsv_exec = nullptr;   // a group of kRsvGroup passes + rsv_apply
  std::vector<unsigned char> rsv_exec_sig;
  hipGraphExec_t rsv_exec1 = nullptr;  // one pass + rsv_apply (single-pod calls)
  std::vector<unsigned char> rsv_exec1_sig;
  DevBuf<uint64_t> rsv_part;    // [13][blocks] per-block partials (preferred-node key, max raw, max key, max ds raw,
                                // max taint count, max affinity sum; (ABI 12) group_pre's min match / total, the
                                // filtered-node count and the spread count / InterPodAffinity raw extremes)
  // TaintToleration / NodeAffinity / NodeResourcesBalancedAllocation (exact pass)
  bool def_on = false, def_score = false;
  DefParams DF{};
  DevBuf<NodePred> npred;       // [cap] kg_node_predicates
  // (ABI 11) what the node rows and the staged queue were compiled against (the caller's tables only grow): per node
  // the highest taint id it carries + 1, and the predicate / image table sizes its row decides; per staged queue the
  // fewest taints a pod's tolerations were compiled against and the highest predicate / image id + 1 it references
  std::vector<int16_t> np_taint_top, np_pred_cnt, np_img_cnt;
  bool np_dirty = true;
  int64_t np_taint_top_max = 0, np_pred_cnt_min = 64, np_img_cnt_min = 64;
  int64_t sq_taint_min = 64, sq_pred_top = 0, sq_img_top = 0;
  std::vector<int16_t> rsv_pcnt;                // (ABI 12) per node: predicates its slots were compiled against (64: no slots)
  int64_t rsv_pcnt_min = 64, sq_rsv_top = 0;    // min over the nodes; the staged reservation affinities' top id + 1
  bool rsv_ext_q = false;                       // the queue holds reserve / operating-mode / selector pods: per-pod pass
  bool aux_q = false;  // (r5) a staged pod requests ephemeral-storage / a scalar resource: eval_round<PF, true>
  bool rsv_pdirty = false;
  DevBuf<DefPod> defpods;       // [staged + kMaxB]
  DevBuf<uint32_t> rsv_val2;    // [cap] raw taint count << 24 | raw affinity sum (their Scores on)
  // (ABI 12) PodTopologySpread / InterPodAffinity, hostname key (groups_dev.h): one pod per exact pass
  bool grp_on = false;
  GroupParams GP{};
  DevBuf<int32_t> grp_d;        // [kGroupArrays][kGroups][cap] per-node group counters
  DevBuf<GroupPod> gpods;       // [staged + kMaxB]
  DevBuf<double> logw;          // [cap + 1] log(F + 2)
  DevBuf<uint64_t> gval;        // [cap] InterPodAffinity raw << 32 | spread count
  DevBuf<GroupPod> gdelta;      // kg_pods_add / kg_pods_remove: the pods' group view, their nodes and signs
  DevBuf<int32_t> gdelta_ns;
  DevBuf<int32_t> gz;           // [2][2][kSpread][kZones] zone sums, by pod parity
  DevBuf<uint64_t> gzm;         // [2] present zones
  // batched exact rounds (xr_dev.h): kXrPods pods per round
  bool xr_on = true;            // KG_EXACT_ROUNDS=0: one pod per pass only
  DevBuf<uint64_t> xr_val;      // [kXrPods][cap]
  DevBuf<uint32_t> xr_val2;     // [kXrPods][cap] (TaintToleration / NodeAffinity Scores on)
  DevBuf<uint32_t> xr_aff;      // [kXrPods][cap] (NodeNUMAResource on)
  DevBuf<uint64_t> xr_part;     // [kXrPods][tiles][kXrNorm]
  DevBuf<uint64_t> xr_norm_d;   // [kXrPods][kXrNorm]
  DevBuf<uint64_t> xr_lists;    // [kXrPods][tiles][kR]
  DevBuf<uint64_t> xr_cand;     // [kXrPods][kCandStride]
  DevBuf<uint64_t> xr_norm_all; // (r5) [n_ranks][kXrPods][kXrNorm]: every rank's shard statistics (several ranks)
  DevBuf<uint64_t> xr_rec_all;  // (r5) [n_ranks][kXrPods][kCandStride]: every rank's merged record (several ranks)
  hipGraphExec_t xr_exec = nullptr;  // kXrGraphRounds rounds
  std::vector<unsigned char> xr_exec_sig;
  double xr_avg = kXrPods;      // pods a round consumed on average (sizes the launches between host checks)
  // live kernel timing (kg_profile_enable): HIP event pairs around every launch of the round runners, on the
  // launch's own stream, folded into per-kind totals after each batch synchronises
  bool prof_on = false;
  std::vector<hipEvent_t> prof_pool;
  size_t prof_used = 0;
  struct ProfRec {
    int kind;
    size_t a, b;  // prof_pool indices of the begin / end events
  };
  std::vector<ProfRec> prof_recs;
  double prof_ms[KG_PROF_KINDS] = {};
  int64_t prof_n[KG_PROF_KINDS] = {};
};

namespace {

// ---- live kernel timing (kg_profile_enable) ----
constexpr size_t kNoProf = ~size_t(0);
size_t prof_mark(kg_engine* e, hipStream_t st) {
  if (e->prof_used == e->prof_pool.size()) {
    hipEvent_t ev = nullptr;
    if (hipEventCreate(&ev) != hipSuccess) return kNoProf;
    e->prof_pool.push_back(ev);
  }
  const size_t i = e->prof_used++;
  return hipEventRecord(e->prof_pool[i], st) == hipSuccess ? i : kNoProf;
}
size_t prof_begin(kg_engine* e, hipStream_t st) { return e->prof_on ? prof_mark(e, st) : kNoProf; }
void prof_end(kg_engine* e, int kind, size_t a, hipStream_t st) {
  if (a == kNoProf) return;
  const size_t b = prof_mark(e, st);
  if (b != kNoProf) e->prof_recs.push_back({kind, a, b});
}
// after the streams of the recorded launches have synchronised
int prof_collect(kg_engine* e) {
  for (const auto& r : e->prof_recs) {
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, e->prof_pool[r.a], e->prof_pool[r.b]));
    e->prof_ms[r.kind] += ms;
    e->prof_n[r.kind] += 1;
  }
  e->prof_recs.clear();
  e->prof_used = 0;
  return 0;
}

int validate_config(const kg_config* c) {
  if (!c) return fail(KG_E_INVALID, "config is NULL");
  if (c->abi_version != KG_ABI_VERSION) return fail(KG_E_INVALID, "abi_version %lld != %d", (long long)c->abi_version, KG_ABI_VERSION);
  for (int r = 2; r < KG_RES_MAX; ++r) {
    if (c->fit_score && c->fit_resource_weights[r] != 0)
      return fail(KG_E_UNSUPPORTED, "NodeResourcesFit scoring resource slot %d: only cpu/memory are accelerated", r);
    if (c->la_score && c->la_resource_weights[r] != 0)
      return fail(KG_E_UNSUPPORTED, "LoadAware resourceWeights slot %d: only cpu/memory are accelerated", r);
  }
  for (int r = 0; r < 2; ++r) {
    if (c->fit_resource_weights[r] < 0 || c->fit_resource_weights[r] > 1000000) return fail(KG_E_INVALID, "fit weight out of range");
    if (c->la_resource_weights[r] < 0 || c->la_resource_weights[r] > 1000000) return fail(KG_E_INVALID, "loadaware weight out of range");
  }
  if ((c->la_score || c->la_filter) && c->la_resource_weights[0] + c->la_resource_weights[1] <= 0)
    return fail(KG_E_INVALID, "LoadAwareSchedulingArgs.resourceWeights must not be empty");
  if (c->weight_fit < 0 || c->weight_fit > 1000000 || c->weight_loadaware < 0 || c->weight_loadaware > 1000000)
    return fail(KG_E_INVALID, "plugin weight out of range");
  if (c->batch_pods < 0 || c->batch_pods > kMaxB) return fail(KG_E_INVALID, "batch_pods must be in [1,%d]", kMaxB);
  if (c->la_agg_usage_type < KG_AGG_NONE || c->la_agg_usage_type > KG_AGG_P99 || c->la_agg_score_type < KG_AGG_NONE ||
      c->la_agg_score_type > KG_AGG_P99 || c->la_agg_usage_duration_ns < 0 || c->la_agg_score_duration_ns < 0)
    return fail(KG_E_INVALID, "LoadAwareSchedulingArgs.Aggregated: aggregation type / duration");
  if (c->weight_taint < 0 || c->weight_taint > 1000000 || c->weight_affinity < 0 || c->weight_affinity > 1000000 ||
      c->weight_balanced < 0 || c->weight_balanced > 1000000 || c->weight_image < 0 || c->weight_image > 1000000)
    return fail(KG_E_INVALID,
                "TaintToleration / NodeAffinity / NodeResourcesBalancedAllocation / ImageLocality weight out of range");
  if (c->weight_spread < 0 || c->weight_spread > 1000000 || c->weight_interpod < 0 || c->weight_interpod > 1000000)
    return fail(KG_E_INVALID, "PodTopologySpread / InterPodAffinity weight out of range");
  if ((c->interpod_filter || c->interpod_score) && (c->hard_pod_affinity_weight < 0 || c->hard_pod_affinity_weight > 100))
    return fail(KG_E_INVALID, "InterPodAffinityArgs.HardPodAffinityWeight must be in [0, 100]");
  if (c->balanced_score && (c->balanced_resources & ~3ll))
    return fail(KG_E_UNSUPPORTED, "NodeResourcesBalancedAllocation resources: cpu / memory are accelerated");
  if (c->reservation_filter || c->reservation_score) {
    if (c->weight_reservation < 0 || c->weight_reservation > 1000000) return fail(KG_E_INVALID, "Reservation weight out of range");
  }
  if (c->ds_filter || c->ds_score) {
    if (c->weight_deviceshare < 0 || c->weight_deviceshare > 1000000) return fail(KG_E_INVALID, "DeviceShare weight out of range");
    if (c->ds_scoring_strategy != KG_STRATEGY_LEAST_ALLOCATED && c->ds_scoring_strategy != KG_STRATEGY_MOST_ALLOCATED)
      return fail(KG_E_UNSUPPORTED, "DeviceShare scoring strategy: LeastAllocated / MostAllocated");
    for (int r = 0; r < 3; ++r)
      if (c->ds_scoring_weights[r] < 0 || c->ds_scoring_weights[r] > 1000000) return fail(KG_E_INVALID, "DeviceShare scoring weight");
    if (c->ds_score && !c->ds_filter)
      return fail(KG_E_UNSUPPORTED, "DeviceShare at Score needs DeviceShare at Filter (Score errors on unfiltered nodes)");
    if (c->batch_pods > 32) return fail(KG_E_UNSUPPORTED, "DeviceShare profiles: batch_pods <= 32");
    if (100 * ((c->fit_score ? c->weight_fit : 0) + (c->la_score ? c->weight_loadaware : 0)) >= (1 << 23))
      return fail(KG_E_UNSUPPORTED, "DeviceShare profiles: Fit + LoadAware weights must keep totals below 2^23");
  }
  if (c->numa_filter || c->numa_score) {
    if (c->weight_numa < 0 || c->weight_numa > 1000000) return fail(KG_E_INVALID, "NodeNUMAResource weight out of range");
    if ((c->numa_scoring_strategy != KG_STRATEGY_LEAST_ALLOCATED && c->numa_scoring_strategy != KG_STRATEGY_MOST_ALLOCATED) ||
        (c->numa_numa_scoring_strategy != KG_STRATEGY_LEAST_ALLOCATED &&
         c->numa_numa_scoring_strategy != KG_STRATEGY_MOST_ALLOCATED))
      return fail(KG_E_UNSUPPORTED, "NodeNUMAResource scoring strategy: LeastAllocated / MostAllocated");
    for (int r = 0; r < 2; ++r)
      if (c->numa_scoring_weights[r] < 0 || c->numa_scoring_weights[r] > 1000000 || c->numa_numa_scoring_weights[r] < 0 ||
          c->numa_numa_scoring_weights[r] > 1000000)
        return fail(KG_E_INVALID, "NodeNUMAResource scoring weight out of range");
    if (c->numa_default_cpu_bind_policy < KG_BIND_NONE || c->numa_default_cpu_bind_policy > KG_BIND_CONSTRAINED_BURST)
      return fail(KG_E_INVALID, "DefaultCPUBindPolicy");
  }
  return 0;
}

// EstimateNode (estimator/default_estimator.go:110-129)
int64_t estimate_node(const kg_node& n, int r) {
  if ((n.flags & KG_NODE_HAS_RAW_ALLOCATABLE) && n.raw_allocatable_present[r]) return n.raw_allocatable[r];
  return n.allocatable[r];
}

// isNodeMetricExpired (loadaware/helper.go:36-41)
bool metric_expired(const kg_node_metric& m, int64_t exp_s, int64_t now) {
  if (!m.present || !m.has_update_time) return true;
  return exp_s > 0 && (now - m.update_time_unix_nano) >= exp_s * 1000000000LL;
}

int64_t milli_of(int r, int64_t v) { return r == KG_RES_CPU ? v : v * 1000; }

// int64(math.Round(float64(used.MilliValue()) / float64(total.MilliValue()) * 100)) (load_aware.go:214,248)
int64_t usage_percent(int r, int64_t used, int64_t total) {
  volatile double q = (double)milli_of(r, used) / (double)milli_of(r, total);
  volatile double pct = q * 100.0;
  return (int64_t)std::round(pct);
}

// LoadAware Filter verdict for one node, for a non-prod (prod=false) or prod pod (load_aware.go:123-254).
// Pod-invariant apart from {prod, daemonset}: Filter ignores estimated/assigned pods (":198 TODO").
// getTargetAggregatedUsage (loadaware/helper.go:58-92): the AggregatedNodeUsages entry whose Usage[type] is
// read, -1 = nil (no NodeMetric, no entries, or the chosen entry's map is empty)
int agg_index(const kg_node_metric& m, int64_t dur_ns, int64_t type) {
  if (!m.has_node_metric || m.agg_count <= 0 || type < 1 || type > KG_AGG_TYPES) return -1;
  const int n = (int)std::min<int64_t>(m.agg_count, KG_MAX_AGG);
  if (dur_ns == 0) {  // no period: the longest one recorded (the first of equals)
    int64_t maxd = 0;
    int maxi = 0;
    for (int i = 0; i < n; ++i)
      if (m.agg_duration_ns[i] > maxd) maxd = m.agg_duration_ns[i], maxi = i;
    return m.agg_present[maxi][type - 1] ? maxi : -1;
  }
  for (int i = 0; i < n; ++i)
    if (m.agg_duration_ns[i] == dur_ns && m.agg_present[i][type - 1]) return i;
  return -1;
}
int64_t agg_value(const kg_node_metric& m, int i, int64_t type, int r) {
  return (r < 2 && ((m.agg_present[i][type - 1] >> r) & 1)) ? m.agg_usage[i][type - 1][r] : 0;
}

// generateUsageThresholdsFilterProfile's AggregatedUsage (helper.go:102-140): the node annotation's when complete,
// else the args' when filterWithAggregation.  False = nil.
bool agg_filter_profile(const kg_config& c, const kg_node& n, int64_t thr[KG_RES_MAX], int64_t& type, int64_t& dur) {
  int nargs = 0, ncust = 0;
  for (int r = 0; r < KG_RES_MAX; ++r) {
    nargs += c.la_agg_usage_thresholds[r] != 0;
    ncust += n.custom_agg_thresholds[r] >= 0;
  }
  if ((n.flags & KG_NODE_HAS_CUSTOM_THRESHOLDS) && ncust > 0 && n.custom_agg_type != KG_AGG_NONE) {
    for (int r = 0; r < KG_RES_MAX; ++r) thr[r] = std::max<int64_t>(n.custom_agg_thresholds[r], 0);
    type = n.custom_agg_type;
    dur = n.custom_agg_duration_ns;
    return true;
  }
  if (nargs > 0 && c.la_agg_usage_type != KG_AGG_NONE) {
    for (int r = 0; r < KG_RES_MAX; ++r) thr[r] = c.la_agg_usage_thresholds[r];
    type = c.la_agg_usage_type;
    dur = c.la_agg_usage_duration_ns;
    return true;
  }
  return false;
}

bool la_filter_pass(const kg_config& c, const kg_node& n, const kg_node_metric& m, int64_t now, bool prod) {
  if (!m.present) return true;
  if (c.la_filter_expired_node_metrics && c.la_node_metric_expiration_seconds >= 0 &&
      metric_expired(m, c.la_node_metric_expiration_seconds, now))
    return true;
  const bool custom = (n.flags & KG_NODE_HAS_CUSTOM_THRESHOLDS) != 0;
  int nc = 0, ncp = 0, nprod_args = 0;
  for (int r = 0; r < KG_RES_MAX; ++r) {
    nc += custom && n.custom_usage_thresholds[r] >= 0;
    ncp += custom && n.custom_prod_usage_thresholds[r] >= 0;
    nprod_args += c.la_prod_usage_thresholds[r] != 0;
  }
  auto thr = [&](int r) { return nc > 0 ? std::max<int64_t>(n.custom_usage_thresholds[r], 0) : c.la_usage_thresholds[r]; };
  auto pthr = [&](int r) { return ncp > 0 ? std::max<int64_t>(n.custom_prod_usage_thresholds[r], 0) : c.la_prod_usage_thresholds[r]; };
  if (prod && (ncp > 0 ? ncp : nprod_args) > 0) {  // filterProdUsage (load_aware.go:226-254)
    if (m.pods_metric_count == 0) return true;
    for (int r = 0; r < KG_RES_MAX; ++r) {
      const int64_t t = pthr(r);
      if (t == 0) continue;
      const int64_t total = estimate_node(n, r);
      if (total == 0) continue;
      if (usage_percent(r, m.prod_pods_usage[r], total) >= t) return false;
    }
    return true;
  }
  int64_t athr[KG_RES_MAX], atype = 0, adur = 0;
  const bool agg = agg_filter_profile(c, n, athr, atype, adur);
  if (!m.has_node_metric) return true;  // filterNodeUsage (load_aware.go:173-224)
  const int ai = agg ? agg_index(m, adur, atype) : -1;
  for (int r = 0; r < KG_RES_MAX; ++r) {
    const int64_t t = agg ? athr[r] : thr(r);
    if (t == 0) continue;
    const int64_t total = estimate_node(n, r);
    if (total == 0) continue;
    if (agg && ai < 0) continue;  // aggregated usage nil
    const int64_t used = agg ? agg_value(m, ai, atype, r) : (m.node_usage_present[r] ? m.node_usage[r] : 0);
    if (usage_percent(r, used, total) >= t) return false;
  }
  return true;
}

// TranslateResourceNameByPriorityClass (apis/extension/resource.go:53-58); -1 = "".
int translate_resource(int64_t prio, int r) {
  if (prio == KG_PRIO_PROD || prio == KG_PRIO_NONE) return r;
  if (prio == KG_PRIO_BATCH) return r == KG_RES_CPU ? KG_RES_BATCH_CPU : (r == KG_RES_MEMORY ? KG_RES_BATCH_MEMORY : -1);
  if (prio == KG_PRIO_MID) return r == KG_RES_CPU ? KG_RES_MID_CPU : (r == KG_RES_MEMORY ? KG_RES_MID_MEMORY : -1);
  return -1;
}

// estimatedUsedByResource (estimator/default_estimator.go:73-108)
int64_t estimate_resource(const kg_pod& p, int real, int64_t factor) {
  const int64_t limit = real >= 0 ? p.limits[real] : 0;
  const int64_t request = real >= 0 ? p.requests[real] : 0;
  int64_t q = request;
  if (limit > request) {
    factor = 100;
    q = limit;
  }
  if (q == 0) {
    if (real == KG_RES_CPU || real == KG_RES_BATCH_CPU) return 250;                 // DefaultMilliCPURequest
    if (real == KG_RES_MEMORY || real == KG_RES_BATCH_MEMORY) return 200LL << 20;   // DefaultMemoryRequest
    return 0;
  }
  volatile double prod = (double)q * (double)factor;
  int64_t est = (int64_t)std::round(prod / 100.0);
  if (limit > 0 && est > limit) est = limit;
  return est;
}

// EstimatePod (default_estimator.go:57-70) for the cpu/memory weight keys.
void estimate_pod(const kg_config& c, const kg_pod& p, int64_t est[2]) {
  for (int r = 0; r < 2; ++r) {
    est[r] = 0;
    if (c.la_resource_weights[r] == 0) continue;
    est[r] = estimate_resource(p, translate_resource(p.priority_class, r), c.la_estimated_scaling_factors[r]);
  }
}

int decode_pod(const kg_engine* e, const kg_pod& p, DevPod& d) {
  const kg_config& c = e->cfg;
  bool zero = true;
  for (int r = 0; r < KG_RES_MAX; ++r) {
    if (p.requests[r] < 0 || p.limits[r] < 0) return fail(KG_E_INVALID, "negative pod quantity");
    zero &= p.requests[r] == 0;
    if (c.fit_filter && r >= kAuxFirst + kAux && p.requests[r] != 0)
      return fail(KG_E_UNSUPPORTED, "pod requests resource slot %d outside the accelerated NodeResourcesFit set", r);
    if (c.fit_filter && r >= kAuxFirst && p.requests[r] != 0 && (e->numa_on || e->ds_on) && !e->exact_on)
      return fail(KG_E_UNSUPPORTED, "pod requests ephemeral-storage / a scalar resource (slot %d): accelerated in the "
                  "NodeResourcesFit + LoadAware profiles only", r);
  }
  if (p.priority_class < KG_PRIO_NONE || p.priority_class > KG_PRIO_FREE) return fail(KG_E_INVALID, "priority_class");
  d.req_cpu = p.requests[KG_RES_CPU];
  d.req_mem = p.requests[KG_RES_MEMORY];
  d.nz_cpu = p.nonzero_requests[0];
  d.nz_mem = p.nonzero_requests[1];
  int64_t est[2];
  estimate_pod(c, p, est);
  d.est_cpu = est[0];
  d.est_mem = est[1];
  d.nz_mem_d = (double)d.nz_mem;
  d.est_mem_d = (double)d.est_mem;
  d.nz_cpu32 = (int32_t)std::min<int64_t>(d.nz_cpu, kPodCpu32Max);
  d.est_cpu32 = (int32_t)std::min<int64_t>(d.est_cpu, kPodCpu32Max);
  d.req_cpu32 = (int32_t)std::min<int64_t>(d.req_cpu, kFreeCpuAbs + 1);
  d.req_mem_d = (double)std::min<int64_t>(d.req_mem, int64_t(1) << 53);
  d.flags = (zero ? P_ZERO_REQ : 0) | ((p.flags & KG_POD_DAEMONSET) ? P_DAEMONSET : 0) |
            (p.priority_class == KG_PRIO_PROD ? P_PROD : 0) |
            (p.priority_class == KG_PRIO_PROD && c.la_score_according_prod_usage ? P_LA_PROD_SCORE : 0);
  d.pad = 0;
  d.quota = (int32_t)std::min<int64_t>(std::max<int64_t>(p.quota_id, 0), 1 << 20) - 1;
  if (p.flags & KG_POD_NON_PREEMPTIBLE) d.flags |= P_NONPREEMPT;
  // request-key presence (PodRequestsAndLimits keys): explicit with KG_POD_REQUEST_KEYS, else by value
  const bool kc = (p.flags & KG_POD_REQUEST_KEYS) ? (p.flags & KG_POD_CPU_KEY) != 0 : d.req_cpu != 0;
  const bool km = (p.flags & KG_POD_REQUEST_KEYS) ? (p.flags & KG_POD_MEM_KEY) != 0 : d.req_mem != 0;
  d.flags |= (kc ? P_CPU_KEY : 0u) | (km ? P_MEM_KEY : 0u);
  for (int r = 0; r < KG_QUOTA_RES - 2; ++r)
    if (p.device_requests[r] != 0) d.flags |= P_QDEV;
  for (int r = 0; r < kAux; ++r)
    if (c.fit_filter && p.requests[kAuxFirst + r] != 0) d.flags |= P_AUX;
  return 0;
}

// NodeNUMAResource preFilterState (plugin.go:220-270; AllowUseCPUSet util.go:42-49)
int decode_numa_pod(const kg_config& c, const kg_pod& p, NumaPod& d) {
  std::memset(&d, 0, sizeof(d));
  if (p.qos < KG_QOS_NONE || p.qos > KG_QOS_SYSTEM) return fail(KG_E_INVALID, "pod qos");
  if (p.required_cpu_bind_policy < KG_BIND_NONE || p.required_cpu_bind_policy > KG_BIND_CONSTRAINED_BURST ||
      p.preferred_cpu_bind_policy < KG_BIND_NONE || p.preferred_cpu_bind_policy > KG_BIND_CONSTRAINED_BURST)
    return fail(KG_E_INVALID, "pod cpu bind policy");
  if (p.preferred_cpu_exclusive_policy < KG_EXCL_NONE || p.preferred_cpu_exclusive_policy > KG_EXCL_NUMA_NODE_LEVEL)
    return fail(KG_E_INVALID, "pod cpu exclusive policy");
  d.req_cpu = p.requests[KG_RES_CPU];
  d.req_mem = p.requests[KG_RES_MEMORY];
  d.allow = (p.qos == KG_QOS_LSE || p.qos == KG_QOS_LSR) && p.priority_class == KG_PRIO_PROD;  // PreRestoreReservation
  bool zero = true;
  for (int r = 0; r < KG_RES_MAX; ++r) zero &= p.requests[r] == 0;
  if (zero) {
    d.skip = 1;
    return 0;
  }
  if (!d.allow) return 0;
  int bind = (int)p.preferred_cpu_bind_policy;
  if (bind == KG_BIND_NONE || bind == KG_BIND_DEFAULT) bind = (int)c.numa_default_cpu_bind_policy;
  int required = (int)p.required_cpu_bind_policy;
  if (required == KG_BIND_DEFAULT) required = (int)c.numa_default_cpu_bind_policy;
  if (required != KG_BIND_NONE) bind = required;
  if (bind == KG_BIND_FULL_PCPUS || bind == KG_BIND_SPREAD_BY_PCPUS) {
    if (d.req_cpu % 1000 != 0) {  // "the requested CPUs must be integer": every node rejects
      d.prefilter_error = 1;
      return 0;
    }
    if (d.req_cpu > 0) {
      d.cpu_bind = 1;
      d.required = required;
      d.preferred = bind;
      d.needed = (int32_t)std::min<int64_t>(d.req_cpu / 1000, 1 << 20);
      d.excl = (int32_t)p.preferred_cpu_exclusive_policy;  // plugin.go:261
    }
  }
  return 0;
}

// TopologyOptions + NodeAllocation of one node → device rows
int decode_node_numa(const kg_node_numa& n, NumaStatic& s, NumaMut& m) {
  std::memset(&s, 0, sizeof(s));
  std::memset(&m, 0, sizeof(m));
  if (n.num_numa < 0 || n.num_numa > KG_MAX_NUMA) return fail(KG_E_UNSUPPORTED, "num_numa %lld > %d", (long long)n.num_numa, KG_MAX_NUMA);
  if (n.numa_policy < KG_NUMA_POLICY_NONE || n.numa_policy > KG_NUMA_POLICY_SINGLE_NUMA_NODE) return fail(KG_E_INVALID, "numa_policy");
  if (n.node_cpu_bind_policy < KG_NODE_BIND_NONE || n.node_cpu_bind_policy > KG_NODE_BIND_SPREAD_BY_PCPUS)
    return fail(KG_E_INVALID, "node_cpu_bind_policy");
  if (n.numa_allocate_strategy < -1 || n.numa_allocate_strategy > KG_STRATEGY_MOST_ALLOCATED)
    return fail(KG_E_INVALID, "numa_allocate_strategy");
  if (n.has_topology) {
    if (n.sockets < 0 || n.nodes_per_socket < 0 || n.cores_per_node < 0 || n.cpus_per_core < 0)
      return fail(KG_E_INVALID, "negative topology");
    const int64_t cpus = n.sockets * n.nodes_per_socket * n.cores_per_node * n.cpus_per_core;
    if (cpus > KG_MAX_CPUS || n.sockets > 8 || n.sockets * n.nodes_per_socket > 8)
      return fail(KG_E_UNSUPPORTED, "cpu topology beyond %d cpus / 8 NUMA nodes", KG_MAX_CPUS);
    if (n.cpus_per_core > 2) return fail(KG_E_UNSUPPORTED, "cpus_per_core %lld > 2", (long long)n.cpus_per_core);
    s.sockets = (int32_t)n.sockets;
    s.nps = (int32_t)n.nodes_per_socket;
    s.cpn = (int32_t)n.cores_per_node;
    s.cpc = (int32_t)n.cpus_per_core;
    s.valid = cpus > 0 ? 1 : 0;  // CPUTopology.IsValid: every count non-zero
  }
  s.policy = (int32_t)n.numa_policy;
  s.node_bind = (int32_t)n.node_cpu_bind_policy;
  s.strategy = (int32_t)n.numa_allocate_strategy;
  s.num_numa = (int32_t)n.num_numa;
  for (int i = 0; i < KG_MAX_NUMA; ++i) {
    if (n.numa_cpu[i] < 0 || n.numa_mem[i] < 0 || n.numa_alloc_cpu[i] < 0 || n.numa_alloc_mem[i] < 0)
      return fail(KG_E_INVALID, "negative NUMA quantity");
    s.numa_cpu[i] = i < n.num_numa ? n.numa_cpu[i] : 0;
    s.numa_mem[i] = i < n.num_numa ? n.numa_mem[i] : 0;
    m.alloc_cpu[i] = i < n.num_numa ? n.numa_alloc_cpu[i] : 0;
    m.alloc_mem[i] = i < n.num_numa ? n.numa_alloc_mem[i] : 0;
    if (m.alloc_cpu[i] != 0 || m.alloc_mem[i] != 0) m.present |= 1u << i;
  }
  if (!(n.cpu_amplification_ratio >= 0.0) || n.cpu_amplification_ratio > 1000.0)
    return fail(KG_E_INVALID, "cpu_amplification_ratio outside [0, 1000]");
  s.cpu_amp = n.cpu_amplification_ratio;
  for (int w = 0; w < KG_MAX_CPUS / 64; ++w) {
    s.reserved[w] = n.reserved_cpus[w];
    m.allocated[w] = n.allocated_cpus[w];
    m.excl_pcpu[w] = n.exclusive_pcpu_cpus[w] & n.allocated_cpus[w];
    m.excl_numa[w] = n.exclusive_numa_cpus[w] & n.allocated_cpus[w];
  }
  return 0;
}

// DeviceShare preFilterState for the GPU type: GetPodDeviceRequests (deviceshare/utils.go:232-252) =
// RemoveZeros → Mask(GPU names) → ValidateDeviceRequest (:158-179, percentage units :151-156) →
// ConvertDeviceRequest (:181-192 with the mapper table :92-149).
// TaintToleration / NodeAffinity view of one pod (k: its index, for the error)
int decode_def_pod(const kg_pod& p, DefPod& d, int64_t k) {
  d = DefPod{};
  if (p.n_required_terms < 0 || p.n_required_terms > kAffTerms || p.n_preferred_terms < 0 ||
      p.n_preferred_terms > kAffTerms)
    return fail(KG_E_UNSUPPORTED, "pod %lld: more than %d node affinity terms (the pod stays on the Go path)",
                (long long)k, kAffTerms);
  d.tol = p.tolerated_taints;
  d.sel = p.node_selector;
  d.nreq = (int32_t)p.n_required_terms;
  d.npref = (int32_t)p.n_preferred_terms;
  for (int t = 0; t < kAffTerms; ++t) {
    d.req[t] = t < d.nreq ? p.required_terms[t] : 0;
    d.pref[t] = t < d.npref ? p.preferred_terms[t] : 0;
    if (t < d.npref && (p.preferred_weights[t] < 0 || p.preferred_weights[t] > 100))
      return fail(KG_E_INVALID, "pod %lld: preferred term weight %lld outside [0, 100]", (long long)k,
                  (long long)p.preferred_weights[t]);
    d.w[t] = t < d.npref ? (int32_t)p.preferred_weights[t] : 0;
  }
  // ImageLocality: containers grouped by image bit (sumImageScores adds an image once per container using it)
  if (p.n_containers < 0 || p.n_containers > kContainers)
    return fail(KG_E_UNSUPPORTED, "pod %lld: more than %d containers for ImageLocality (the pod stays on the Go path)",
                (long long)k, kContainers);
  d.ncont = (int32_t)p.n_containers;
  for (int c = 0; c < d.ncont; ++c) {
    const int64_t b = p.container_image_bit[c], w = p.container_image_score[c];
    if (b < -1 || b > 63 || w < 0)
      return fail(KG_E_INVALID, "pod %lld: container %d image bit %lld / score %lld out of range", (long long)k, c,
                  (long long)b, (long long)w);
    if (b < 0) continue;  // no node holds the image
    int at = 0;
    while (at < d.nimg && d.img_bit[at] != (uint8_t)b) ++at;
    if (at == d.nimg) {
      d.img_bit[d.nimg] = (uint8_t)b;
      d.img_w[d.nimg++] = 0;
    }
    d.img_w[at] += w;
  }
  return 0;
}

// (ABI 12) PodTopologySpread / InterPodAffinity view of one pod (groups 1-based in the ABI)
int decode_group_pod(const kg_pod& p, GroupPod& d, int64_t k) {
  d = GroupPod{};
  auto grp = [&](int64_t g, int32_t& out, const char* what) -> int {
    if (g < 0 || g > kGroups) return fail(KG_E_INVALID, "pod %lld: %s group %lld outside [0, %d]", (long long)k, what,
                                          (long long)g, kGroups);
    out = (int32_t)g - 1;
    return 0;
  };
  const uint64_t all = kGroups >= 64 ? ~0ull : ((1ull << kGroups) - 1);
  if (((uint64_t)p.match_groups | (uint64_t)p.pod_affinity_terms | (uint64_t)p.pod_anti_affinity |
       (uint64_t)p.pod_affinity_terms_zone | (uint64_t)p.pod_anti_affinity_zone) & ~all)
    return fail(KG_E_INVALID, "pod %lld: a group bit beyond %d", (long long)k, kGroups);
  d.match = (uint32_t)p.match_groups;
  d.aff_terms = (uint32_t)p.pod_affinity_terms;
  d.anti = (uint32_t)p.pod_anti_affinity;
  d.aff_terms_z = (uint32_t)p.pod_affinity_terms_zone;
  d.anti_z = (uint32_t)p.pod_anti_affinity_zone;
  if (int rc = grp(p.pod_affinity_group, d.req, "pod affinity")) return rc;
  if ((d.req >= 0) != ((d.aff_terms | d.aff_terms_z) != 0))
    return fail(KG_E_INVALID, "pod %lld: required pod affinity needs both its conjunction group and its terms",
                (long long)k);
  if (p.n_spread < 0 || p.n_spread > kSpread)
    return fail(KG_E_UNSUPPORTED, "pod %lld: more than %d topology spread constraints (the pod stays on the Go path)",
                (long long)k, kSpread);
  d.nsp = (int32_t)p.n_spread;
  uint32_t seen = 0;
  for (int c = 0; c < d.nsp; ++c) {
    int32_t g = -1;
    if (int rc = grp(p.spread_group[c], g, "topology spread")) return rc;
    const int64_t fa = p.spread_flags[c], f = fa & 3ll;
    if (g < 0 || p.spread_max_skew[c] < 1 || p.spread_max_skew[c] > INT32_MAX || (fa & ~7ll))
      return fail(KG_E_INVALID, "pod %lld: spread constraint %d: group %lld, maxSkew %lld, flags %lld", (long long)k, c,
                  (long long)p.spread_group[c], (long long)p.spread_max_skew[c], (long long)fa);
    // (ABI 13) system defaults: every constraint of the pod or none, ScheduleAnyway only
    const bool sd = (fa & KG_SPREAD_SYSTEM_DEFAULT) != 0;
    if (sd != ((p.spread_flags[0] & KG_SPREAD_SYSTEM_DEFAULT) != 0) || (sd && (f & KG_SPREAD_HARD)))
      return fail(KG_E_INVALID, "pod %lld: KG_SPREAD_SYSTEM_DEFAULT on some constraints only, or on a DoNotSchedule one",
                  (long long)k);
    if (sd) d.zone_keys |= kSpreadSysDefault;
    if ((seen >> f) & 1u)  // the API allows one constraint per {topologyKey, whenUnsatisfiable}
      return fail(KG_E_INVALID, "pod %lld: duplicate {topologyKey, whenUnsatisfiable} spread constraints", (long long)k);
    seen |= 1u << f;
    d.sp_g[c] = g;
    d.sp_skew[c] = (int32_t)p.spread_max_skew[c];
    d.sp_flags[c] = (uint32_t)f;
    if (f & KG_SPREAD_ZONE) d.zone_keys |= (f & KG_SPREAD_HARD) ? 1u : 2u;
  }
  if (p.n_pod_preferred < 0 || p.n_pod_preferred > kPodPref)
    return fail(KG_E_UNSUPPORTED, "pod %lld: more than %d preferred pod (anti-)affinity terms (the pod stays on the Go "
                "path)", (long long)k, kPodPref);
  d.npref = (int32_t)p.n_pod_preferred;
  for (int t = 0; t < d.npref; ++t) {
    int32_t g = -1;
    if (int rc = grp(p.pod_preferred_group[t], g, "preferred term")) return rc;
    const int64_t w = p.pod_preferred_weight[t];
    if (g < 0 || w < -100 || w > 100 || w == 0)
      return fail(KG_E_INVALID, "pod %lld: preferred term %d: group %lld weight %lld (weights in [1, 100], negative for "
                  "anti-affinity)", (long long)k, t, (long long)p.pod_preferred_group[t], (long long)w);
    d.pref_g[t] = g;
    d.pref_w[t] = (int32_t)w;
  }
  if ((uint64_t)p.pod_preferred_zone >> d.npref)
    return fail(KG_E_INVALID, "pod %lld: pod_preferred_zone bit beyond n_pod_preferred", (long long)k);
  d.pref_zone = (uint32_t)p.pod_preferred_zone;
  return 0;
}

int decode_ds_pod(const kg_pod& p, DsPod& d) {
  std::memset(&d, 0, sizeof(d));
  const int64_t* q = p.device_requests;
  for (int r = 0; r < KG_DEV_RES_MAX; ++r)
    if (q[r] < 0) return fail(KG_E_INVALID, "negative device request");
  auto pct_ok = [](int64_t v) { return !(v > 100 && v % 100 != 0); };
  // (ABI 17) RDMA / FPGA (utils.go:47-58: one resource each, ValidatePercentageResource): the default handler's types
  const int64_t xq[kXTypes] = {q[KG_DEV_RDMA], q[KG_DEV_FPGA]};
  for (int t = 0; t < kXTypes; ++t) {
    if (xq[t] > (1 << 20)) return fail(KG_E_UNSUPPORTED, "RDMA / FPGA request beyond the accelerated range");
    if (xq[t] && !pct_ok(xq[t])) d.error = 1;  // "invalid resource unit"
    d.xq[t] = (int32_t)xq[t];
  }
  enum { NV = 1, DCU = 2, KG = 4, CORE = 8, MEM = 16, RATIO = 32 };
  unsigned comb = 0;
  for (int r = 0; r < 6; ++r)
    if (q[r]) comb |= 1u << r;  // KG_DEV_* order = flag order
  if (!comb) {
    d.nogpu = 1;
    d.skip = (xq[0] | xq[1]) == 0 ? 1 : 0;  // state.skip: no device request of any type
    return 0;
  }
  if ((q[KG_DEV_KOORD_GPU] && !pct_ok(q[KG_DEV_KOORD_GPU])) || (q[KG_DEV_GPU_CORE] && !pct_ok(q[KG_DEV_GPU_CORE])) ||
      (q[KG_DEV_GPU_MEMORY_RATIO] && !pct_ok(q[KG_DEV_GPU_MEMORY_RATIO]))) {
    d.error = 1;
    return 0;
  }
  if (q[KG_DEV_NVIDIA_GPU] > (1 << 20) || q[KG_DEV_HYGON_DCU] > (1 << 20) || q[KG_DEV_KOORD_GPU] > (1 << 27) ||
      q[KG_DEV_GPU_CORE] > (1 << 27) || q[KG_DEV_GPU_MEMORY_RATIO] > (1 << 27) || q[KG_DEV_GPU_MEMORY] > (1ll << 50))
    return fail(KG_E_UNSUPPORTED, "device request beyond the accelerated range");
  switch (comb) {
    case NV: d.core = d.ratio = q[KG_DEV_NVIDIA_GPU] * 100; break;
    case DCU: d.core = d.ratio = q[KG_DEV_HYGON_DCU] * 100; break;
    case KG: d.core = d.ratio = q[KG_DEV_KOORD_GPU]; break;
    case MEM: d.mem = q[KG_DEV_GPU_MEMORY]; d.has_mem = 1; break;
    case RATIO: d.ratio = q[KG_DEV_GPU_MEMORY_RATIO]; break;
    case CORE | MEM: d.core = q[KG_DEV_GPU_CORE]; d.mem = q[KG_DEV_GPU_MEMORY]; d.has_mem = 1; break;
    case CORE | RATIO: d.core = q[KG_DEV_GPU_CORE]; d.ratio = q[KG_DEV_GPU_MEMORY_RATIO]; break;
    default: d.error = 1;  // "invalid resource device requests"
  }
  return 0;
}

// One node's Device object + deviceUsed → device row (buildDeviceResources, device_cache.go:505-523)
int decode_node_device(const kg_node_device& n, DsNode& d, DsXNode& x) {
  std::memset(&x, 0, sizeof(x));
  if (n.has_device)  // (ABI 17) RDMA / FPGA DeviceInfos (buildDeviceResources: an unhealthy device has no resources)
    for (int t = 0; t < kXTypes; ++t)
      for (int m = 0; m < KG_MAX_MINORS; ++m) {
        if (!n.x_present[t][m]) continue;
        if (n.x_total[t][m] < 0 || n.x_used[t][m] < 0) return fail(KG_E_INVALID, "negative device quantity");
        if (n.x_total[t][m] >= (1 << 30) || n.x_used[t][m] >= (1 << 30))
          return fail(KG_E_UNSUPPORTED, "device quantity beyond the accelerated range");
        x.listed[t] |= 1u << m;
        x.t[t][m] = n.x_healthy[t][m] ? (int32_t)n.x_total[t][m] : 0;
        x.u[t][m] = (int32_t)n.x_used[t][m];
      }
  std::memset(&d, 0, sizeof(d));
  d.first = -1;
  d.has_device = n.has_device ? 1 : 0;
  if (!n.has_device) return 0;
  for (int m = 0; m < KG_MAX_MINORS; ++m) {
    if (!n.present[m]) continue;
    const int64_t v[6] = {n.total_core[m], n.total_ratio[m], n.used_core[m], n.used_ratio[m], n.total_memory[m], n.used_memory[m]};
    for (int k = 0; k < 6; ++k) {
      if (v[k] < 0) return fail(KG_E_INVALID, "negative device quantity");
      if (v[k] >= (k < 4 ? (1ll << 30) : (1ll << 50))) return fail(KG_E_UNSUPPORTED, "device quantity beyond the accelerated range");
    }
    d.present |= 1 << m;
    if (n.healthy[m]) {
      d.tcore[m] = (int32_t)n.total_core[m];
      d.tratio[m] = (int32_t)n.total_ratio[m];
      d.tmem[m] = n.total_memory[m];
    }
    d.ucore[m] = (int32_t)n.used_core[m];
    d.uratio[m] = (int32_t)n.used_ratio[m];
    d.umem[m] = n.used_memory[m];
    if (d.first < 0 && (d.tcore[m] || d.tratio[m] || d.tmem[m])) {
      if (d.tmem[m] == 0) return fail(KG_E_UNSUPPORTED, "first healthy GPU without gpu-memory (fillGPUTotalMem divides by it)");
      d.first = m;
    }
  }
  return 0;
}

// Static columns (alloc_cpu, alloc_mem, la_alloc_cpu, la_alloc_mem | alloc_pods, flags) from host mirror.
uint32_t node_flags(const kg_engine* e, int64_t i) {
  const kg_node& n = e->nodes[i];
  if (!(n.flags & KG_NODE_VALID)) return 0;
  const kg_node_metric& m = e->metrics[i];
  const int64_t now = e->clock_now;  // isNodeMetricExpired: time.Since(updateTime) at this scheduling call
  uint32_t f = F_VALID;
  const kg_config& c = e->cfg;
  if (m.present && !(c.la_node_metric_expiration_seconds >= 0 && metric_expired(m, c.la_node_metric_expiration_seconds, now)))
    f |= F_LA_SCORE;
  if (la_filter_pass(c, n, m, now, false)) f |= F_LA_PASS;
  if (la_filter_pass(c, n, m, now, true)) f |= F_LA_PASS_PROD;
  if (estimate_node(n, KG_RES_CPU) == n.allocatable[KG_RES_CPU] &&
      estimate_node(n, KG_RES_MEMORY) == n.allocatable[KG_RES_MEMORY])
    f |= F_LA_ALLOC_EQ;
  return f;
}

int64_t clock_read(const kg_engine* e) {
  if (e->clock_mode == 1) return e->clock_fixed;
  if (e->clock_mode == 2)
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::system_clock::now().time_since_epoch()).count();
  return e->clock_metrics;
}

// Moves the scheduler clock to this call's now: the static flags are rebuilt only when some node's
// isNodeMetricExpired verdict (loadaware/helper.go:36-41) differs between the old and the new now.
void clock_refresh(kg_engine* e) {
  const int64_t now = clock_read(e);
  if (now == e->clock_now) return;
  const int64_t exp_s = e->cfg.la_node_metric_expiration_seconds;
  bool flip = false;
  for (int64_t i = 0; i < e->n_nodes && !flip && exp_s > 0; ++i) {
    const kg_node_metric& m = e->metrics[i];
    if (m.present && m.has_update_time)
      flip = metric_expired(m, exp_s, now) != metric_expired(m, exp_s, e->clock_now);
  }
  e->clock_now = now;
  if (flip) e->static_dirty = true;
}

int refresh_eph(kg_engine* e) {
  if (!e->eph_dirty) return 0;
  e->eph_dirty = false;
  if (e->n_nodes == 0) return 0;
  refresh_eph_flags<<<(unsigned)((e->n_nodes + 255) / 256), 256, 0, e->stream>>>(e->T, e->n_nodes);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(e->stream));
  return 0;
}

int sync_static(kg_engine* e) {
  clock_refresh(e);
  if (!e->static_dirty) return refresh_eph(e);
  e->eph_dirty |= e->eph_any;  // the flags column below is rewritten without F_EPH_OVER
  const int64_t cap = e->capacity;
  auto& h64 = e->h_static64;
  auto& h32 = e->h_static32;
  h64.assign(4 * cap, 0);
  h32.assign(4 * cap, 0);
  auto& hd = e->h_static_f64;
  hd.assign(2 * cap, 0.0);
  // 100 / capacity: only estimates of leastRequestedScore's quotient (corrected exactly on device); f32 for the
  // cpu terms, f64 (correctly rounded) for the memory terms
  auto inv100 = [](int64_t c) -> float { return c > 0 ? (float)(100.0 / (double)c) : 0.0f; };
  auto inv100d = [](int64_t c) -> double { return c > 0 ? 100.0 / (double)c : 0.0; };
  for (int64_t i = 0; i < e->n_nodes; ++i) {
    const kg_node& n = e->nodes[i];
    h64[0 * cap + i] = n.allocatable[KG_RES_CPU];
    h64[1 * cap + i] = n.allocatable[KG_RES_MEMORY];
    h64[2 * cap + i] = estimate_node(n, KG_RES_CPU);
    h64[3 * cap + i] = estimate_node(n, KG_RES_MEMORY);
    h32[0 * cap + i] = (int32_t)std::min<int64_t>(n.allowed_pods, INT32_MAX);
    h32[1 * cap + i] = (int32_t)node_flags(e, i);
    const float f[2] = {inv100(h64[0 * cap + i]), inv100(h64[2 * cap + i])};
    for (int q = 0; q < 2; ++q) std::memcpy(&h32[(2 + q) * cap + i], &f[q], 4);
    hd[0 * cap + i] = inv100d(h64[1 * cap + i]);
    hd[1 * cap + i] = inv100d(h64[3 * cap + i]);
  }
  HIP_TRY(hipMemcpyAsync(e->T.alloc_cpu, &h64[0 * cap], cap * 8, hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipMemcpyAsync(e->T.alloc_mem, &h64[1 * cap], cap * 8, hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipMemcpyAsync(e->T.la_alloc_cpu, &h64[2 * cap], cap * 8, hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipMemcpyAsync(e->T.la_alloc_mem, &h64[3 * cap], cap * 8, hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipMemcpyAsync(e->T.alloc_pods, &h32[0 * cap], cap * 4, hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipMemcpyAsync(e->T.flags, (uint32_t*)&h32[1 * cap], cap * 4, hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipMemcpyAsync(e->T.inv_cpu, &h32[2 * cap], 2 * cap * 4, hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipMemcpyAsync(e->T.inv_mem, hd.data(), 2 * cap * 8, hipMemcpyHostToDevice, e->stream));
  {  // Allocatable of the NodeResourcesFit-only resources (ephemeral-storage, batch / mid cpu / memory)
    auto& ha = e->h_aux;
    ha.assign((size_t)kAux * cap, 0);
    for (int64_t i = 0; i < e->n_nodes; ++i)
      for (int r = 0; r < kAux; ++r) ha[(size_t)r * cap + i] = e->nodes[i].allocatable[kAuxFirst + r];
    HIP_TRY(hipMemcpyAsync(e->T.aux, ha.data(), (size_t)kAux * cap * 8, hipMemcpyHostToDevice, e->stream));
  }
  HIP_TRY(hipStreamSynchronize(e->stream));
  e->static_dirty = false;
  return refresh_eph(e);
}

int push_deltas(kg_engine* e, const std::vector<RowDelta>& d) {
  if (d.empty()) return 0;
  if (int rc = e->deltas.ensure(d.size())) return rc;
  HIP_TRY(hipMemcpyAsync(e->deltas.p, d.data(), d.size() * sizeof(RowDelta), hipMemcpyHostToDevice, e->stream));
  const int64_t n = (int64_t)d.size();
  apply_deltas<<<(unsigned)((n + 255) / 256), 256, 0, e->stream>>>(e->T, e->deltas.p, n);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(e->stream));
  return 0;
}

// NodeUsage folded into la_used (non-prod view): load_aware.go:307-326 with an empty PodsMetric — the aggregated
// usage of ScoreAggregationType when scoreWithAggregation (nil: no node usage at all).
void usage_for_score(const kg_config& c, const kg_node_metric& m, int64_t u[2]) {
  if (c.la_agg_score_type != KG_AGG_NONE) {
    const int i = m.present ? agg_index(m, c.la_agg_score_duration_ns, c.la_agg_score_type) : -1;
    for (int r = 0; r < 2; ++r) u[r] = i >= 0 ? agg_value(m, i, c.la_agg_score_type, r) : 0;
    return;
  }
  for (int r = 0; r < 2; ++r) u[r] = (m.present && m.has_node_metric && m.node_usage_present[r]) ? m.node_usage[r] : 0;
}

// The node-level LoadAware Score terms with PodsMetric (load_aware.go:283-376), relative to what the device adds per
// assigned pod (its EstimatePod): out[0..1] = the non-prod view folded into la_used, out[2..3] = the prod view
// (ScoreAccordingProdUsage) folded into la_pused.  An assigned pod is estimated when its usage is not reported,
// or it was assigned after the metric's update time, or within the report interval before it, or the aggregated
// score usage is missing (estimatedAssignedPodUsed :337-376); it then counts max(EstimatePod, reported usage) and its
// reported usage leaves NodeUsage when NodeUsage covers it (:307-326); otherwise its usage is already in NodeUsage
// (non-prod view) or in the prod pods' reported usages (prod view), and its EstimatePod is taken back out.
void la_node_terms(const kg_engine* e, int64_t i, int64_t out[4]) {
  const kg_config& c = e->cfg;
  const kg_node_metric& m = e->metrics[i];
  int64_t u[2];
  usage_for_score(c, m, u);
  const auto& pm = e->pmetrics[i];
  out[0] = u[0], out[1] = u[1], out[2] = 0, out[3] = 0;
  if (pm.empty() || !m.present) return;  // nil podMetrics: every assigned pod is estimated (:355)
  const int64_t upd = m.has_update_time ? m.update_time_unix_nano : INT64_MIN;  // zero time: before every assign
  const int64_t interval = m.report_interval_ns > 0 ? m.report_interval_ns : 60ll * 1000000000ll;
  const bool agg_nil = c.la_agg_score_type != KG_AGG_NONE && agg_index(m, c.la_agg_score_duration_ns, c.la_agg_score_type) < 0;
  for (int view = 0; view < 2; ++view) {  // 0: all pods (non-prod), 1: prod pods only (buildPodMetricMap filterProdPod)
    int64_t corr[2] = {0, 0}, est_usage[2] = {0, 0}, act_usage[2] = {0, 0};
    std::vector<char> estimated(pm.size(), 0);
    for (const auto& a : e->assigned[i]) {
      if (view == 1 && !a.prod) continue;
      int hit = -1;
      if (a.uid != 0)
        for (size_t q = 0; q < pm.size(); ++q)
          if (pm[q].uid == a.uid && (view == 0 || pm[q].prod)) {
            hit = (int)q;
            break;
          }
      const bool reported = hit >= 0 && pm[hit].present != 0;
      const bool missed = a.time > upd;
      const bool in_interval = a.time < upd && upd - a.time < interval;
      if (!reported || missed || in_interval || agg_nil) {
        for (int r = 0; r < 2; ++r) {
          int64_t v = a.est[r];
          if (reported && ((pm[hit].present >> r) & 1) && pm[hit].usage[r] > v) v = pm[hit].usage[r];
          corr[r] += v - a.est[r];
        }
        if (hit >= 0) estimated[hit] = 1;
      } else {
        for (int r = 0; r < 2; ++r) corr[r] -= a.est[r];
      }
    }
    for (size_t q = 0; q < pm.size(); ++q) {  // sumPodUsages (helper.go:172-186)
      if (view == 1 && !pm[q].prod) continue;
      for (int r = 0; r < 2; ++r) {
        if (!((pm[q].present >> r) & 1)) continue;
        (estimated[q] ? est_usage : act_usage)[r] += pm[q].usage[r];
      }
    }
    if (view == 0) {
      for (int r = 0; r < 2; ++r) {
        int64_t nu = u[r];
        if (est_usage[r] != 0 && nu >= est_usage[r]) nu -= est_usage[r];
        out[r] = nu + corr[r];
      }
    } else {
      for (int r = 0; r < 2; ++r) out[2 + r] = act_usage[r] + corr[r];
    }
  }
}

// Re-folds node i's LoadAware terms into la_used / la_pused (a delta against what is folded now)
void la_refold(kg_engine* e, int64_t i, std::vector<RowDelta>& d) {
  int64_t t[4];
  la_node_terms(e, i, t);
  RowDelta x{};
  x.idx = i;
  x.d[5] = t[0] - e->folded_usage[2 * i];
  x.d[6] = t[1] - e->folded_usage[2 * i + 1];
  x.d[7] = t[2] - e->folded_prod[2 * i];
  x.d[8] = t[3] - e->folded_prod[2 * i + 1];
  e->folded_usage[2 * i] = t[0];
  e->folded_usage[2 * i + 1] = t[1];
  e->folded_prod[2 * i] = t[2];
  e->folded_prod[2 * i + 1] = t[3];
  if (x.d[5] || x.d[6] || x.d[7] || x.d[8]) d.push_back(x);
}

// podAssignCache mirror: assign (Reserve / informer add) and unAssign (Unreserve / delete) of one pod
void mirror_assign(kg_engine* e, int64_t i, const kg_engine::AssignedPod& a) { e->assigned[i].push_back(a); }
void mirror_unassign(kg_engine* e, int64_t i, int64_t uid, const int64_t est[2]) {
  auto& v = e->assigned[i];
  for (size_t q = 0; q < v.size(); ++q)
    if ((uid != 0 && v[q].uid == uid) || (uid == 0 && v[q].uid == 0 && v[q].est[0] == est[0] && v[q].est[1] == est[1])) {
      v.erase(v.begin() + (long)q);
      return;
    }
}

struct RoundGeom {
  int64_t N, shard, base, n_local;
  int nt_local, B, ppw, bitmap_words;
  int nte;     // (r4) eval_round tiles of kETile nodes in this shard
  int nl_max;  // list slots per pod in the lists buffer: max(nt_local, nte)
  int depth;  // rounds in flight: eval(r) reads the table right after resolve(r - depth) (1 = unpipelined)
};

RoundGeom geometry(const kg_engine* e) {
  RoundGeom g;
  g.N = e->n_nodes;
  g.shard = (g.N + e->n_ranks - 1) / e->n_ranks;
  g.base = std::min<int64_t>(g.N, (int64_t)e->rank * g.shard);
  g.n_local = std::min<int64_t>(g.shard, g.N - g.base);
  g.nt_local = (int)std::max<int64_t>(1, (g.shard + kTile - 1) / kTile);
  g.nte = (int)std::max<int64_t>(1, (g.shard + kETile - 1) / kETile);
  g.nl_max = std::max(g.nt_local, g.nte);
  g.B = (int)(e->cfg.batch_pods > 0 ? e->cfg.batch_pods : 32);
  g.ppw = (int)(e->cfg.pods_per_wave > 0 ? std::min<int64_t>(e->cfg.pods_per_wave, g.B) : 8);
  g.bitmap_words = (int)(((std::max<int64_t>(g.N, 1) + 127) / 128) * 4);  // whole 16-B stores
  // pipelining needs the monotone profile (a row read mid-update reads ≥ its current key) and depth·B modified-row
  // slots in the resolver; several ranks keep one communicator per round stream
  int d = (int)(e->cfg.pipeline_depth > 0 ? e->cfg.pipeline_depth : 2);
  d = std::min(d, kMaxDepth);
  while (d > 1 && d * g.B > kMaxMod) --d;
  // (r5) the NUMA rounds pipeline too: their resolver re-scores every row modified since the snapshot (the earlier
  // rounds' winners included) for every pod, so no monotonicity is needed; its slots are one wave's lanes, one of
  // them spare for the best unmodified candidate
  const bool numa_rounds = e->numa_on && !e->ds_on && !e->rsv_on;
  if (numa_rounds)
    while (d > 1 && d * g.B >= kWave) --d;
  g.depth = (e->P.monotone || numa_rounds) ? d : 1;
  if (e->numa_on) g.ppw = std::min(g.ppw, kNumaPpw);  // eval_round_numa parks ≤ kNumaPpw pods' values in LDS
  if (e->ds_on) g.ppw = std::min(g.ppw, kDsPpw);      // the DeviceShare passes keep ≤ kDsPpw pods in registers
  return g;
}

size_t resolve_lds_bytes(const RoundGeom& g, int nb) {
  return ((size_t)nb * (kCandStride + kPodWords) + kParWords) * 8 + (size_t)(kModHash + kMaxMod) * 4 +
         (size_t)g.bitmap_words * 4;
}
constexpr size_t kMaxLds = 160 * 1024;
size_t resolve_numa_lds_bytes(const RoundGeom& g, int nb) {
  return ((size_t)nb * (kCandStride + kPodWords + kNumaPodWords) + (size_t)kWave * (kNumaStaticWords + kNumaMutWords)) * 8 +
         (size_t)kWave * 4 + (size_t)g.bitmap_words * 4;
}
NumaTable numa_table(kg_engine* e) { return NumaTable{e->numa_s.p, e->numa_m.p}; }

size_t eval_lds_bytes(const RoundGeom& g) { return (size_t)kEW * std::max(g.ppw * kR, kC) * 8; }
// eval_round's 1-D grid: tile groups of kEW tiles × pod groups, swizzled over XCDs inside the kernel
dim3 eval_grid_e(const RoundGeom& g, int nb) {
  return dim3((unsigned)(((g.nte + kEW - 1) / kEW) * ((nb + g.ppw - 1) / g.ppw)));
}
dim3 eval_grid(const RoundGeom& g, int nb) {
  // 1-D grid: tile groups × pod groups, swizzled over XCDs inside eval_round
  return dim3((unsigned)(((g.nt_local + kEvalWaves - 1) / kEvalWaves) * ((nb + g.ppw - 1) / g.ppw)));
}

int profile_bits(const EvalParams& P) {
  return (P.fit_filter ? PF_FIT_FILTER : 0) | (P.fit_score ? PF_FIT_SCORE : 0) | (P.la_filter ? PF_LA_FILTER : 0) |
         (P.la_score ? PF_LA_SCORE : 0) | (P.la_score && P.la_prod_score ? PF_LA_PROD : 0);
}

#ifdef KG_DEV_PF  // iteration builds only (make dev): one profile instantiated; engine_create refuses every other one
#define KG_PF_SWITCH(pf, CALL) \
  if ((pf) == KG_DEV_PF) {     \
    CALL(KG_DEV_PF);           \
  }
#else
#define KG_PF_SWITCH(pf, CALL)                                                                   \
  switch (pf) {                                                                                \
    case 0: CALL(0); break;   case 1: CALL(1); break;   case 2: CALL(2); break;   case 3: CALL(3); break;     \
    case 4: CALL(4); break;   case 5: CALL(5); break;   case 6: CALL(6); break;   case 7: CALL(7); break;     \
    case 8: CALL(8); break;   case 9: CALL(9); break;   case 10: CALL(10); break; case 11: CALL(11); break;   \
    case 12: CALL(12); break; case 13: CALL(13); break; case 14: CALL(14); break; case 15: CALL(15); break;   \
    case 24: CALL(24); break; case 25: CALL(25); break; case 26: CALL(26); break; case 27: CALL(27); break;   \
    case 28: CALL(28); break; case 29: CALL(29); break; case 30: CALL(30); break; case 31: CALL(31); break;   \
  }
#endif

int32_t* poison_ptr(kg_engine* e) { return reinterpret_cast<int32_t*>(e->cursor.p + 3); }
uint64_t* lists_slot(kg_engine* e, const RoundGeom& g, int slot) {
  return e->lists.p + (size_t)slot * g.B * g.nl_max * kR;
}

constexpr int kCombineTiles = 16 * kEW;  // combined lists from 16 tile groups on (128 keys ≥ kC per pod)
bool eval_combine(const RoundGeom& g) { return g.nte >= kCombineTiles; }
int eval_lists(kg_engine* e, const RoundGeom& g);
uint64_t* cand_slot(kg_engine* e, const RoundGeom& g, int slot);
bool merge_block();
// (r5) KG_FUSE=1: the merge fused into eval_round's tail (merge_tail; one rank, the Fit + LoadAware round engine,
// ≤ 2·kWave lists per pod, ≤ 131k nodes).  A/B option only: measured at C3 the tail merge made eval + merge 2.5 µs
// longer than the two launches (40.8 vs 28.0 + 10.2 µs, profiles/r05/timeline_*.txt) — the boundary it removes costs
// ~0.9 µs (scripts/micro/handoff.hip) and every block pays a release before its ticket.
bool fused_merge(kg_engine* e, const RoundGeom& g) {
  static const bool on = KG_FUSE_TAIL && std::getenv("KG_FUSE") && std::string(std::getenv("KG_FUSE")) == "1";
  return on && e->n_ranks == 1 && !e->numa_on && !e->ds_on && !merge_block() && eval_lists(e, g) <= 2 * kWave;
}
uint32_t* tickets_slot(kg_engine* e, int slot) { return e->tickets.p + (size_t)slot * kMaxB; }
// (r5) eval_round<PF, AUX>: the ephemeral-storage / scalar check only in the instantiation a queue with such a pod
// runs (profiles with NodeResourcesFit's Filter)
template <int X>
void launch_eval_round(kg_engine* e, const RoundGeom& g, int64_t first, int nb, int slot, hipStream_t st, bool fuse) {
  auto go = [&](auto kern) {
    kern<<<eval_grid_e(g, nb), kWave * kEW, eval_lds_bytes(g), st>>>(e->T, e->pods.p, first, nb, g.ppw, g.base,
                                                                    g.n_local, g.nte, e->P, lists_slot(e, g, slot),
                                                                    poison_ptr(e), e->paux.p,
                                                                    eval_combine(g) ? 1 : 0,
                                                                    fuse ? tickets_slot(e, slot) : nullptr,
                                                                    cand_slot(e, g, slot));
  };
  if constexpr ((X & PF_FIT_FILTER) != 0) {
    if (e->aux_q) {
      go(eval_round<X, true>);
      return;
    }
  }
  go(eval_round<X, false>);
}

void launch_eval(kg_engine* e, const RoundGeom& g, int64_t first, int nb, int slot, hipStream_t st, bool fuse = false) {
  if (e->numa_on) {  // one block per (tile, pod group)
    const dim3 grid((unsigned)(g.nt_local * ((nb + g.ppw - 1) / g.ppw)));
    eval_round_numa<<<grid, kWave * kEvalWaves, 0, st>>>(e->T, numa_table(e), e->pods.p, e->npods.p, first, nb,
                                                                      g.ppw, g.base, g.n_local, g.nt_local, e->P,
                                                                      e->NP, lists_slot(e, g, slot), poison_ptr(e));
    return;
  }
#define KG_EVAL(X) launch_eval_round<X>(e, g, first, nb, slot, st, fuse)
  KG_PF_SWITCH(profile_bits(e->P), KG_EVAL)
#undef KG_EVAL
}

// candidate lists per pod of the round's wide pass: eval_round writes one per tile group of kEvalWaves tiles, the
// NUMA and DeviceShare passes one per tile
int eval_lists(kg_engine* e, const RoundGeom& g) {
  if (e->numa_on || e->ds_on) return g.nt_local;
  return eval_combine(g) ? (g.nte + kEW - 1) / kEW : g.nte;
}

// local merge: this rank's tile lists → per-pod record (single rank: the final candidates)
uint64_t* cand_slot(kg_engine* e, const RoundGeom& g, int slot) { return e->cand.p + (size_t)slot * g.B * kCandStride; }
uint64_t* gathered_slot(kg_engine* e, const RoundGeom& g, int slot) {
  return e->gathered.p + (size_t)slot * e->n_ranks * g.B * kCandStride;
}

// KG_MERGE=block: the block-per-pod merge_round for eval_round's lists too (A/B measurements only)
bool merge_block() {
  static const bool on = std::getenv("KG_MERGE") && std::string(std::getenv("KG_MERGE")) == "block";
  return on;
}

void launch_merge_local(kg_engine* e, const RoundGeom& g, int nb, int slot, hipStream_t st) {
  uint64_t* dst = e->n_ranks > 1 ? gathered_slot(e, g, slot) + (size_t)e->rank * g.B * kCandStride : cand_slot(e, g, slot);
  const int nl = eval_lists(e, g);
  // eval_round's tile-group lists hold kRG keys, its tile lists (a shard of fewer than kCombineTiles tiles) and the
  // NUMA / DeviceShare passes' lists kR
  const bool grp = !e->numa_on && !e->ds_on && eval_combine(g);
  const int ll = grp ? kRG : kR;
  if (!e->numa_on && !e->ds_on && !merge_block()) {  // (r4) one wavefront per pod
    const unsigned blocks = (unsigned)((nb + 3) / 4);
    const int64_t ps = (int64_t)nl * ll;
#define KG_MW(LW, LLV) \
  merge_wave<LW, LLV><<<blocks, kWave * 4, 0, st>>>(e->T, e->P, lists_slot(e, g, slot), ps, nl, nb, poison_ptr(e), dst)
#define KG_MW_L(LLV)                    \
  if (nl <= kWave) KG_MW(1, LLV);       \
  else if (nl <= 2 * kWave) KG_MW(2, LLV); \
  else if (nl <= 4 * kWave) KG_MW(4, LLV); \
  else KG_MW(8, LLV);
    if (grp) {
      KG_MW_L(kRG)
    } else {
      KG_MW_L(kR)
    }
#undef KG_MW_L
#undef KG_MW
    return;
  }
  merge_round<false><<<nb, kMergeThreads, 0, st>>>(e->T, e->P, lists_slot(e, g, slot), (int64_t)nl * ll, ll, nl, ll,
                                                   nb, poison_ptr(e), dst);
}

void launch_merge_ranks(kg_engine* e, const RoundGeom& g, int nb, int slot, hipStream_t st) {
  merge_round<true><<<nb, kMergeThreads, 0, st>>>(e->T, e->P, gathered_slot(e, g, slot), kCandStride,
                                                  (int64_t)g.B * kCandStride, e->n_ranks, kC, nb, poison_ptr(e),
                                                  cand_slot(e, g, slot));
}

// KG_RESOLVER=mw: the look-ahead resolve_mw (A/B measurements only).  The single-wave resolve_round is the default:
// on MI355X at 100k nodes, depth 2, it runs the C3 queue at 869k pods/s against resolve_mw's 671k
bool resolver_one_wave() {
  static const bool on = !(std::getenv("KG_RESOLVER") && std::string(std::getenv("KG_RESOLVER")) == "mw");
  return on;
}

void launch_resolve(kg_engine* e, const RoundGeom& g, int64_t first, int nb, int slot, int n_prev,
                    int64_t seq, int wait, hipStream_t st) {
  // (r6) the two-wave resolver while the engine's round streams have hardware queues of their own (one rank, depth
  // ≤ 3: with the main stream ≤ 4 streams, GPU_MAX_HW_QUEUES); KG_NUMA_RESOLVER=1 keeps the one-wave chain (A/B runs).
  // Where streams share a queue — depth 4, or several loopback ranks in one process — the two-wave kernel's chain
  // wait outlasted its spin limit in r6 (test_c4_pipelined_parity[8-4], test_numa_ranks); the one-wave kernel is the
  // measured-safe choice there
  static const bool numa_one_wave = std::getenv("KG_NUMA_RESOLVER") && std::getenv("KG_NUMA_RESOLVER")[0] == '1';
  const size_t lds2 = resolve_numa_lds_bytes(g, nb) + numa2_extra_lds_bytes();
  if (e->numa_on && !numa_one_wave && e->n_ranks == 1 && g.depth <= 3 && lds2 <= kMaxLds) {
    const bool pre = lds2 + numa2_pre_lds_bytes(nb) <= kMaxLds;
    resolve_round_numa2<<<1, kNuma2Threads, lds2 + (pre ? numa2_pre_lds_bytes(nb) : 0), st>>>(
        e->T, numa_table(e), e->pods.p, e->npods.p, e->cursor.p, first, nb, cand_slot(e, g, slot), e->P, e->NP,
        e->out_keys.p, e->out_cpus.p, e->out_nrec.p, g.bitmap_words, poison_ptr(e), seq, e->quotas.p, e->nq,
        e->modlists.p, slot, g.depth, n_prev, wait, pre ? kNumaPre : 0);
  } else if (e->numa_on) {
    resolve_round_numa<<<1, kWave, resolve_numa_lds_bytes(g, nb), st>>>(e->T, numa_table(e), e->pods.p, e->npods.p,
                                                                        e->cursor.p, first, nb, cand_slot(e, g, slot),
                                                                        e->P, e->NP, e->out_keys.p, e->out_cpus.p,
                                                                        e->out_nrec.p,
                                                                        g.bitmap_words, poison_ptr(e), seq, e->quotas.p,
                                                                        e->nq, e->modlists.p, slot, g.depth, n_prev,
                                                                        wait);
    return;
  }
#define KG_RESOLVE_T(X, Q)                                                                                       \
  resolve_round<X, Q><<<1, kWave, resolve_lds_bytes(g, nb), st>>>(e->T, e->pods.p, e->cursor.p, first, nb,           \
                                                                  cand_slot(e, g, slot), e->P, e->out_keys.p,       \
                                                                  g.bitmap_words, e->modlists.p, slot, g.depth,     \
                                                                  n_prev, poison_ptr(e), seq, wait, e->quotas.p,    \
                                                                  e->nq, e->paux.p)
#define KG_RESOLVE(X) KG_RESOLVE_T(X, false)
#define KG_RESOLVE_Q(X) KG_RESOLVE_T(X, true)
#define KG_RESOLVE_MW_T(X, Q)                                                                                   \
  resolve_mw<X, Q><<<1, kMwThreads, mw_lds_bytes(nb), st>>>(e->T, e->pods.p, e->cursor.p, first, nb,              \
                                                            cand_slot(e, g, slot), e->P, e->out_keys.p,         \
                                                            e->modlists.p, slot, g.depth, n_prev, poison_ptr(e), \
                                                            seq, wait, e->quotas.p, e->nq, e->paux.p)
#define KG_RESOLVE_MW(X) KG_RESOLVE_MW_T(X, false)
#define KG_RESOLVE_MW_Q(X) KG_RESOLVE_MW_T(X, true)
  if (!resolver_one_wave()) {
    if (e->nq > 0) {
      KG_PF_SWITCH(profile_bits(e->P), KG_RESOLVE_MW_Q)
    } else {
      KG_PF_SWITCH(profile_bits(e->P), KG_RESOLVE_MW)
    }
  } else if (e->nq > 0) {
    KG_PF_SWITCH(profile_bits(e->P), KG_RESOLVE_Q)
  } else {
    KG_PF_SWITCH(profile_bits(e->P), KG_RESOLVE)
  }
#undef KG_RESOLVE_MW_Q
#undef KG_RESOLVE_MW
#undef KG_RESOLVE_MW_T
#undef KG_RESOLVE_Q
#undef KG_RESOLVE_T
#undef KG_RESOLVE
}

int lb_barrier(kg_loopback* lb) {
  std::unique_lock<std::mutex> lk(lb->mu);
  const uint64_t g = lb->gen;
  if (lb->failed) return fail(KG_E_COLLECTIVE, "loopback group failed");
  if (++lb->arrived == lb->n) {
    lb->arrived = 0;
    ++lb->gen;
    lb->cv.notify_all();
    return 0;
  }
  if (!lb->cv.wait_for(lk, std::chrono::seconds(60), [&] { return lb->gen != g || lb->failed; })) {
    lb->failed = true;
    lb->cv.notify_all();
    return fail(KG_E_COLLECTIVE, "loopback exchange: a peer rank did not arrive within 60 s");
  }
  return lb->failed ? fail(KG_E_COLLECTIVE, "loopback group failed") : 0;
}

// All-gather of `cnt` words per rank in `all` ([n_ranks][cnt], this rank's part already written on stream st):
// ncclAllGather over RCCL, or — loopback test hook — device copies from the peers' buffers, ordered by events.
int rank_allgather(kg_engine* e, uint64_t* all, size_t cnt, int slot, hipStream_t st) {
  if (e->xfn) {  // host collective: this rank's part back to the host, the caller's all-gather, every part up again
    e->xsend.resize(cnt);
    e->xrecv.resize(cnt * (size_t)e->n_ranks);
    HIP_TRY(hipMemcpyAsync(e->xsend.data(), all + (size_t)e->rank * cnt, cnt * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (int rc = e->xfn(e->xuser, e->xsend.data(), e->xrecv.data(), (int64_t)(cnt * 8)))
      return fail(KG_E_COLLECTIVE, "host exchange returned %d", rc);
    HIP_TRY(hipMemcpyAsync(all, e->xrecv.data(), cnt * 8 * (size_t)e->n_ranks, hipMemcpyHostToDevice, st));
    HIP_TRY(hipStreamSynchronize(st));  // the host buffers are reused by the next exchange
    return 0;
  }
  if (!e->lb) {
    NCCL_TRY(ncclAllGather(all + (size_t)e->rank * cnt, all, cnt, ncclUint64, e->comms[slot], st));
    return 0;
  }
  kg_loopback* lb = e->lb;
  HIP_TRY(hipEventRecord(e->lb_ready, st));
  lb->buf[e->rank] = all;
  if (int rc = lb_barrier(lb)) return rc;
  for (int q = 0; q < lb->n; ++q) {
    if (q == e->rank) continue;
    HIP_TRY(hipStreamWaitEvent(st, lb->ready[q], 0));
    HIP_TRY(hipMemcpyAsync(all + (size_t)q * cnt, lb->buf[q] + (size_t)q * cnt, cnt * 8, hipMemcpyDeviceToDevice, st));
  }
  HIP_TRY(hipEventRecord(e->lb_done, st));
  if (int rc = lb_barrier(lb)) return rc;
  // a peer's later writes into its buffer (same stream as its reads of it) wait for this rank's copies
  for (int q = 0; q < lb->n; ++q)
    if (q != e->rank) HIP_TRY(hipStreamWaitEvent(st, lb->done[q], 0));
  return 0;
}

// merge → [all-gather + merge of the rank records] of one round, on stream st
int launch_merge(kg_engine* e, const RoundGeom& g, int nb, int slot, hipStream_t st) {
  launch_merge_local(e, g, nb, slot, st);
  HIP_TRY(hipGetLastError());
  if (e->n_ranks > 1) {
    const size_t cnt = (size_t)g.B * kCandStride;
    uint64_t* all = gathered_slot(e, g, slot);
    if (int rc = rank_allgather(e, all, cnt, slot, st)) return rc;
    launch_merge_ranks(e, g, nb, slot, st);
    HIP_TRY(hipGetLastError());
  }
  return 0;
}

// One batch of rounds over pods [cur, end).  Round r runs on stream rs[r % D]: eval(r) → merge(r) →
// [RCCL all-gather on that stream's communicator] → resolve(r), the resolve waiting on resolve(r-1) (another
// stream) through the device sequence word, so its launch and prologue overlap the previous resolver instead of
// waiting on a cross-stream event.  Stream order makes eval(r) start right after resolve(r-D): it overlaps
// resolve(r-D+1 .. r-1), whose rows resolve(r) treats as modified; merge(r) also runs off the
// serial chain.  The first round of a batch starts from a fully written table (the host synchronised), so it has
// no previous-round rows.  (r4: a split — resolvers on streams of their own, dispatched ahead and waiting on the
// device for their merge — measured slower at every depth: the cross-stream event before each wide pass costs more
// than the early dispatch saves)
int run_batch(kg_engine* e, const RoundGeom& g, int64_t cur, int64_t end, int64_t n_rounds) {
  const int D = g.depth;
  const bool fuse = fused_merge(e, g);
  HIP_TRY(hipMemsetAsync(e->cursor.p + 3, 0, 3 * 8, e->rs[0]));  // poison, resolver sequence, device error
  if (fuse) HIP_TRY(hipMemsetAsync(e->tickets.p, 0, (size_t)kMaxDepth * kMaxB * 4, e->rs[0]));
  if (D > 1) {  // the other round streams must not start before that reset
    HIP_TRY(hipEventRecord(e->ev_res[0], e->rs[0]));
    for (int k = 1; k < D; ++k) HIP_TRY(hipStreamWaitEvent(e->rs[k], e->ev_res[0], 0));
  }
  for (int64_t r = 0; r < n_rounds; ++r) {
    const int64_t first = cur + r * g.B;
    const int nb = (int)std::min<int64_t>(g.B, end - first);
    const int slot = (int)(r % D);
    hipStream_t st = e->rs[slot];
    size_t t = prof_begin(e, st);
    launch_eval(e, g, first, nb, slot, st, fuse);
    HIP_TRY(hipGetLastError());
    prof_end(e, KG_PROF_EVAL, t, st);
    if (!fuse) {
      t = prof_begin(e, st);
      if (int rc = launch_merge(e, g, nb, slot, st)) return rc;
      prof_end(e, KG_PROF_MERGE, t, st);
    }
    const int n_prev = (int)std::min<int64_t>(r, D - 1);
    t = prof_begin(e, st);
    launch_resolve(e, g, first, nb, slot, n_prev, r + 1, D > 1 && r > 0, st);
    HIP_TRY(hipGetLastError());
    prof_end(e, KG_PROF_RESOLVE, t, st);
  }
  for (int k = 0; k < D; ++k) HIP_TRY(hipStreamSynchronize(e->rs[k]));
  return prof_collect(e);
}

// ---- DeviceShare rounds: cursor-driven, unpipelined, all on rs[0] ----
size_t resolve_ds_lds_bytes(const RoundGeom& g, int nb, int nq, bool sharded) {
  return ((size_t)nb * (kCandStride + kPodWords + kDsPodWords + kDsNodeWords + kQuotaRes) + (size_t)kWave * kDsNodeWords) * 8 +
         (size_t)nq * sizeof(QuotaRow) + (size_t)nb * sizeof(Row) +
         (sharded ? (size_t)kWave * (sizeof(DsNode) + sizeof(Row)) : 0) + (size_t)g.bitmap_words * 4;
}

int launch_round_ds(kg_engine* e, const RoundGeom& g, int64_t end, hipStream_t st, int which = -1) {
  const DsTable DT{e->ds_d.p};
  const bool sharded = e->n_ranks > 1;
  const dim3 grid = eval_grid(g, g.B);
  size_t t;
  if (which < 0 || which == 3) {
    t = prof_begin(e, st);
#define KG_DSMAX(X)                                                                                             \
  ds_max_round<X><<<grid, kWave * kEvalWaves, 0, st>>>(e->T, DT, e->pods.p, e->dpods.p, e->cursor.p, end, g.B, g.ppw, \
                                                       g.base, g.n_local, g.nt_local, e->P, e->DP, e->dsmax.p,     \
                                                       e->dsval.p)
    KG_PF_SWITCH(profile_bits(e->P), KG_DSMAX)
#undef KG_DSMAX
    prof_end(e, KG_PROF_DS_MAX, t, st);
  }
  if (which < 0 || which == 4) {
    t = prof_begin(e, st);
    uint64_t* mine = sharded ? e->dsnorm_all.p + (size_t)e->rank * g.B : e->dsnorm.p;
    ds_norm_reduce<<<g.B, 256, 0, st>>>(e->cursor.p, end, g.B, e->dsmax.p, g.nt_local, mine);
    if (sharded) {  // the per-pod normalization maxima over every rank's shard
      if (int rc = rank_allgather(e, e->dsnorm_all.p, (size_t)g.B, 0, st)) return rc;
      ds_norm_combine<<<1, kMaxB, 0, st>>>(e->cursor.p, end, g.B, e->dsnorm_all.p, e->n_ranks, e->dsnorm.p);
    }
    prof_end(e, KG_PROF_DS_NORM, t, st);
  }
  if (which < 0 || which == 0) {
    t = prof_begin(e, st);
    eval_round_ds<<<grid, kWave * kEvalWaves, 0, st>>>(e->cursor.p, end, g.B, g.ppw, g.base, g.n_local, g.nt_local,
                                                        e->P, e->DP, e->dsnorm.p, e->dsval.p, lists_slot(e, g, 0));
    prof_end(e, KG_PROF_EVAL, t, st);
  }
  if (which < 0 || which == 1) {
    t = prof_begin(e, st);
    if (int rc = launch_merge(e, g, g.B, 0, st)) return rc;
    prof_end(e, KG_PROF_MERGE, t, st);
  }
  if (which < 0 || which == 2) {
    t = prof_begin(e, st);
    resolve_round_ds<<<1, kWave, resolve_ds_lds_bytes(g, g.B, e->nq, sharded), st>>>(e->T, DT, e->pods.p, e->dpods.p,
                                                                            e->cursor.p, end, g.B, cand_slot(e, g, 0),
                                                                            e->dsnorm.p, e->dsval.p,
                                                                            (int64_t)g.nt_local * kTile, e->P, e->DP,
                                                                            e->out_keys.p, e->out_minors.p,
                                                                            g.bitmap_words, e->quotas.p, e->nq,
                                                                            e->qdev.p, (int)sharded);
    prof_end(e, KG_PROF_RESOLVE, t, st);
  }
  return 0;
}

int run_batch_ds(kg_engine* e, const RoundGeom& g, int64_t end, int64_t n_rounds) {
  for (int64_t r = 0; r < n_rounds; ++r) {
    if (int rc = launch_round_ds(e, g, end, e->rs[0])) return rc;
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(hipStreamSynchronize(e->rs[0]));
  return prof_collect(e);
}

int prepare_rounds(kg_engine* e, RoundGeom& g) {
  if (int rc = sync_static(e)) return rc;
  g = geometry(e);
  if (g.N > kMaxNodes) return fail(KG_E_UNSUPPORTED, "n_nodes %lld > %lld", (long long)g.N, (long long)kMaxNodes);
  if (g.nt_local > kMergeThreads * kMergeChunks)
    return fail(KG_E_UNSUPPORTED, "%lld nodes per rank exceed one merge block (%d)", (long long)g.shard,
                kMergeThreads * kMergeChunks * kTile);
  if (e->ds_on && resolve_ds_lds_bytes(g, g.B, e->nq, e->n_ranks > 1) > kMaxLds)
    return fail(KG_E_UNSUPPORTED, "DeviceShare resolver LDS %zu B > %zu B: fewer nodes or a smaller batch_pods",
                resolve_ds_lds_bytes(g, g.B, e->nq, e->n_ranks > 1), kMaxLds);
  if (!e->numa_on && !e->ds_on && resolve_lds_bytes(g, g.B) > kMaxLds)
    return fail(KG_E_UNSUPPORTED, "resolver LDS %zu B > %zu B: fewer nodes or a smaller batch_pods",
                resolve_lds_bytes(g, g.B), kMaxLds);
  if (!e->numa_on && !e->ds_on && !resolver_one_wave() && mw_lds_bytes(g.B) > kMaxLds)
    return fail(KG_E_UNSUPPORTED, "resolver LDS %zu B > %zu B: a smaller batch_pods", mw_lds_bytes(g.B), kMaxLds);
  const size_t D = (size_t)g.depth;
  const size_t lists_n = e->lists.n;
  if (int rc = e->lists.ensure(D * g.B * g.nl_max * kR)) return rc;
  if (e->lists.n != lists_n)  // fresh lists hold no keys (DeviceShare rounds merge every one of the B slots)
    HIP_TRY(hipMemsetAsync(e->lists.p, 0, e->lists.n * 8, e->stream));
  const size_t cand_n = e->cand.n;
  if (int rc = e->cand.ensure(D * g.B * kCandStride)) return rc;
  if (e->cand.n != cand_n) HIP_TRY(hipMemsetAsync(e->cand.p, 0, e->cand.n * 8, e->stream));
  if (e->n_ranks > 1)
    if (int rc = e->gathered.ensure(D * e->n_ranks * g.B * kCandStride)) return rc;
  if (e->ds_on) {
    if (int rc = e->dsmax.ensure((size_t)g.B * g.nt_local)) return rc;
    if (int rc = e->dsnorm.ensure((size_t)g.B)) return rc;
    if (e->n_ranks > 1)
      if (int rc = e->dsnorm_all.ensure((size_t)e->n_ranks * g.B)) return rc;
    if (int rc = e->dsval.ensure((size_t)g.B * g.nt_local * kTile)) return rc;
  }
  return 0;
}

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}


// Reservation profile: one FIFO pod per device pass (rsv_eval → rsv_select; Reserve in the next rsv_eval),
// kRsvGroup passes + the group-closing rsv_apply per hipGraph launch.  The pod index lives in the device cursor ws[3]; passes past `end` are no-ops.
constexpr int kRsvGroup = 32;
constexpr int64_t kExactSmall = 2;  // schedule calls of at most this many pods take the exact pass (single-pod path)
RsvExt rsv_ext(kg_engine* e) {
  RsvExt X;
  X.ds = e->ds_on ? e->ds_d.p : nullptr;
  X.dsx = e->ds_on ? e->dsx_d.p : nullptr;
  X.dpods = e->ds_on ? e->dpods.p : nullptr;
  X.DP = e->DP;
  X.quotas = e->quotas.p;
  X.qdev = e->qdev.p;
  X.out_minors = e->ds_on ? e->out_minors.p : nullptr;
  X.nq = e->nq;
  X.ns = e->numa_on ? e->numa_s.p : nullptr;
  X.nm = e->numa_on ? e->numa_m.p : nullptr;
  X.npods = e->numa_on ? e->npods.p : nullptr;
  X.NP = e->NP;
  X.aff = e->numa_on ? e->numa_aff.p : nullptr;
  X.out_cpus = e->numa_on ? e->out_cpus.p : nullptr;
  X.out_nrec = e->numa_on ? e->out_nrec.p : nullptr;
  X.paux = e->paux.p;
  X.pred = e->def_on ? e->npred.p : nullptr;
  X.defp = e->def_on ? e->defpods.p : nullptr;
  X.DF = e->DF;
  X.val2 = e->def_score ? e->rsv_val2.p : nullptr;
  X.G = GroupTable{e->grp_d.p, e->capacity};
  X.gpods = e->grp_on ? e->gpods.p : nullptr;
  X.GP = e->GP;
  X.logw = e->logw.p;
  X.gval = e->gval.p;
  X.gz = e->gz.p;
  X.gzm = e->gzm.p;
  X.rsv_pred = e->rsv_pd.p;
  X.rsv_sel = e->rsel.p;
  X.rgpu = e->ds_on && e->rgpu_nodes > 0 ? e->rsv_g.p : nullptr;
  X.rpods = e->rpods.p;
  X.rsv_n = e->rsv_nd.p;
  X.rcpu = e->numa_on && e->rcpu_nodes > 0 ? e->rsv_c.p : nullptr;
  return X;
}

// the rsv_eval variant for the pass's extension pointers (RSV_F_*: plugins absent from the profile compile out)
int rsv_eval_flags(const RsvExt& X) {
  return (X.dsx || X.rcpu ? RSV_F_XF : 0) | (X.ns ? RSV_F_NUMA : 0) | (X.ds ? RSV_F_DS : 0);
}
// the combinations a profile yields (XF needs NUMA or DeviceShare); the rest take the full kernel
#define KG_RSV_VARIANT(K, f)                                           \
  switch (f) {                                                        \
    case 0: return K<0>;                                              \
    case RSV_F_NUMA: return K<RSV_F_NUMA>;                            \
    case RSV_F_DS: return K<RSV_F_DS>;                                \
    case RSV_F_NUMA | RSV_F_DS: return K<RSV_F_NUMA | RSV_F_DS>;      \
    default: return K<RSV_F_XF | RSV_F_NUMA | RSV_F_DS>;              \
  }
using RsvEvalFn = decltype(&rsv_eval<0>);
RsvEvalFn rsv_eval_kernel(int f) { KG_RSV_VARIANT(rsv_eval, f) }
using GroupPreFn = decltype(&group_pre<0>);
GroupPreFn group_pre_kernel(int f) { KG_RSV_VARIANT(group_pre, f) }
using RsvApplyFn = decltype(&rsv_apply<0>);
RsvApplyFn rsv_apply_kernel(int f) { KG_RSV_VARIANT(rsv_apply, f) }
#undef KG_RSV_VARIANT

int run_rsv(kg_engine* e, int64_t first, int64_t count, kg_stats* stats, double t0) {
  if (int rc = sync_static(e)) return rc;
  const int64_t n = e->n_nodes, end = first + count;
  if (count > 0 && n > 0) {
    const unsigned blocks = (unsigned)((n + kRsvThreads - 1) / kRsvThreads);
    RsvExt X = rsv_ext(e);
    if (!e->dsx_q) X.dsx = nullptr;  // (r6) no RDMA / FPGA request staged: the lean rsv_eval variant (part of the graph key)
    const int rf = rsv_eval_flags(X);
    const unsigned long long init[5] = {0, 0, 0, (unsigned long long)first, (unsigned long long)end};
    HIP_TRY(hipMemcpyAsync(e->rsv_ws.p, init, sizeof(init), hipMemcpyHostToDevice, e->stream));
    if (e->grp_on) {  // the zone sums start from zero (then each pod's rsv_select clears the next pod's)
      HIP_TRY(hipMemsetAsync(e->gz.p, 0, (size_t)2 * kZoneSumWords * 4, e->stream));
      HIP_TRY(hipMemsetAsync(e->gzm.p, 0, 16, e->stream));
    }
    // `end_arg` < 0: the kernels read the call's end from the workspace (a graph stays valid across calls);
    // `passes` < kRsvGroup: a short call issues exactly its passes, no empty ones
    auto issue_group = [&](int64_t end_arg, int passes) {
      for (int g = 0; g < passes; ++g) {
        size_t t = prof_begin(e, e->stream);
        if (e->grp_on)  // Reserve of the previous pod + the group reductions this pod's Filters need
          group_pre_kernel(rf)<<<blocks, kRsvThreads, 0, e->stream>>>(e->T, e->rsv_d.p, e->pods.p, end_arg, n, g, X, e->rsv_val.p,
                                                           e->rsv_part.p, e->out_keys.p, e->out_rslot.p, e->rsv_ws.p);
        rsv_eval_kernel(rf)<<<blocks, kRsvThreads, 0, e->stream>>>(
            e->T, e->rsv_d.p, e->rsv_nd.p, e->pods.p, e->rpods.p, end_arg, n, g, e->P, e->RP, X, e->rsv_val.p,
            e->rsv_part.p, e->out_keys.p, e->out_rslot.p, e->rsv_ws.p);
        prof_end(e, KG_PROF_RSV_EVAL, t, e->stream);
        t = prof_begin(e, e->stream);
        rsv_select<<<blocks, kRsvThreads, 0, e->stream>>>(e->rsv_val.p, e->pods.p, end_arg, n, g, e->RP, X, e->rsv_part.p,
                                                           e->rsv_ws.p);
        if (e->grp_on)  // the keys, after PodTopologySpread's raw scores and their extremes
          rsv_select2<<<blocks, kRsvThreads, 0, e->stream>>>(e->rsv_val.p, end_arg, n, g, e->RP, X, e->rsv_part.p,
                                                             e->rsv_ws.p);
        prof_end(e, KG_PROF_RSV_SELECT, t, e->stream);
      }
      size_t t = prof_begin(e, e->stream);
      rsv_apply_kernel(rf)<<<1, kWave, 0, e->stream>>>(e->T, e->rsv_d.p, e->rsv_val.p, e->pods.p, end_arg, (int)blocks, passes - 1,
                                            X, e->rsv_part.p, e->out_keys.p, e->out_rslot.p, e->rsv_ws.p);
      prof_end(e, KG_PROF_RSV_APPLY, t, e->stream);
    };
    // KG_RSV_NO_GRAPH=1: plain stream launches (profilers whose kernel tracing does not follow graph launches);
    // live kernel timing also uses plain launches (its events bracket each launch)
    static const bool no_graph = std::getenv("KG_RSV_NO_GRAPH") && std::getenv("KG_RSV_NO_GRAPH")[0] == '1';
    // graphs of `passes` passes (kRsvGroup, or 1 for single-pod calls), keyed on their launch arguments (table /
    // buffer pointers, sizes, profile parameters) and re-instantiated when one changes
    auto graph = [&](int passes, hipGraphExec_t& exec, std::vector<unsigned char>& exec_sig) -> int {
      std::vector<unsigned char> sig;
      auto put = [&](const void* q, size_t len) {
        const unsigned char* b = static_cast<const unsigned char*>(q);
        sig.insert(sig.end(), b, b + len);
      };
      put(&e->T, sizeof(e->T));
      const void* ptrs[] = {e->rsv_d.p, e->rsv_nd.p, e->pods.p, e->rpods.p, e->rsv_val.p, e->rsv_part.p,
                            e->out_keys.p, e->out_rslot.p, e->rsv_ws.p};
      put(ptrs, sizeof(ptrs));
      put(&n, sizeof(n));
      put(&e->P, sizeof(e->P));
      put(&e->RP, sizeof(e->RP));
      put(&X, sizeof(X));
      if (exec && sig == exec_sig) return 0;
      if (exec) (void)hipGraphExecDestroy(exec);
      exec = nullptr;
      hipGraph_t gr = nullptr;
      HIP_TRY(hipStreamBeginCapture(e->stream, hipStreamCaptureModeThreadLocal));
      issue_group(-1, passes);
      const hipError_t ce = hipStreamEndCapture(e->stream, &gr);
      if (ce != hipSuccess) return fail(KG_E_DEVICE, "hipStreamEndCapture: %s", hipGetErrorString(ce));
      const hipError_t ie = hipGraphInstantiate(&exec, gr, nullptr, nullptr, 0);
      (void)hipGraphDestroy(gr);
      if (ie != hipSuccess) {
        exec = nullptr;
        return fail(KG_E_DEVICE, "exact pass graph: %s", hipGetErrorString(ie));
      }
      exec_sig = sig;
      return 0;
    };
    if (no_graph || e->prof_on || (count > 1 && count < kRsvGroup)) {
      for (int64_t c = 0; c < count; c += kRsvGroup) issue_group(end, (int)std::min<int64_t>(kRsvGroup, count - c));
      HIP_TRY(hipGetLastError());
      HIP_TRY(hipStreamSynchronize(e->stream));
      if (e->prof_on)
        if (int rc = prof_collect(e)) return rc;
    } else {
      hipGraphExec_t ex = nullptr;
      if (count == 1) {
        if (int rc = graph(1, e->rsv_exec1, e->rsv_exec1_sig)) return rc;
        ex = e->rsv_exec1;
      } else {
        if (int rc = graph(kRsvGroup, e->rsv_exec, e->rsv_exec_sig)) return rc;
        ex = e->rsv_exec;
      }
      const int64_t per = count == 1 ? 1 : kRsvGroup;
      hipError_t ge = hipSuccess;
      for (int64_t c = 0; ge == hipSuccess && c < count; c += per) ge = hipGraphLaunch(ex, e->stream);
      if (ge == hipSuccess) ge = hipStreamSynchronize(e->stream);
      if (ge != hipSuccess) return fail(KG_E_DEVICE, "exact pass graph: %s", hipGetErrorString(ge));
    }
  } else if (count > 0) {
    HIP_TRY(hipMemsetAsync(e->out_keys.p + first, 0, count * 8, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
  }
  if (stats) {
    std::memset(stats, 0, sizeof(*stats));
    stats->device_batches = (count + kRsvGroup - 1) / kRsvGroup;
    stats->node_evaluations = count * n;
    stats->seconds = now_s() - t0;
  }
  return 0;
}

#define KG_XF_SWITCH(xf, CALL)    \
  switch (xf) {                   \
    case 0: CALL(0); break;       \
    case 1: CALL(1); break;       \
    case 2: CALL(2); break;       \
    case 3: CALL(3); break;       \
    case 4: CALL(4); break;       \
    case 5: CALL(5); break;       \
    case 6: CALL(6); break;       \
    default: CALL(7); break;      \
  }

// Batched exact rounds (xr_dev.h): rounds of kXrPods pods, kXrGraphRounds rounds per hipGraph launch; the host
// launches about as many rounds as the pods left need at the recent consumption rate, then checks the cursor.
constexpr int kXrGraphRounds = 4;
constexpr int64_t kXrMin = 8;  // schedule calls of fewer pods run one pod per pass
int run_xr(kg_engine* e, int64_t first, int64_t count, kg_stats* stats, double t0) {
  if (int rc = sync_static(e)) return rc;
  const int64_t n = e->n_nodes, end = first + count;
  const int nt = (int)((n + kTile - 1) / kTile);
  const int64_t stride = e->capacity;
  const RsvExt X = rsv_ext(e);
  const unsigned long long init[8] = {0, 0, 0, (unsigned long long)first, (unsigned long long)end, 0, 0, 0};
  HIP_TRY(hipMemcpyAsync(e->rsv_ws.p, init, sizeof(init), hipMemcpyHostToDevice, e->stream));
  // (r5) several ranks: this rank's range of tiles (an empty range keeps one tile past the table: every node masked)
  const int R = e->n_ranks, tpr = (nt + R - 1) / R, tile_base = e->rank * tpr;
  const int ntl = std::max(1, std::min(tpr, nt - tile_base));
  const int64_t lo = std::min<int64_t>(n, (int64_t)tile_base * kTile), hi = std::min<int64_t>(n, (int64_t)(tile_base + ntl) * kTile);
  const unsigned eval_blocks = (unsigned)(((ntl + kEvalWaves - 1) / kEvalWaves) * (kXrPods / kXrPpw));
  const unsigned xr_eval_blocks = (unsigned)ntl * (kXrPods / kXrEvalPpw);
  const int vbits = e->P.score_bits + 1;
  const int bitmap_words = (int)((n + 31) / 32);
  const int xf = (X.ns ? XF_NUMA : 0) | (X.ds ? XF_DS : 0) | (X.defp ? XF_DEF : 0);
  const size_t lds = xr_resolve_lds_bytes(xf, X.nq, X.paux != nullptr, bitmap_words);
  if (lds > 160 * 1024) return fail(KG_E_UNSUPPORTED, "exact rounds: %zu B of LDS for %lld nodes", lds, (long long)n);
  const int32_t* poison = reinterpret_cast<const int32_t*>(e->rsv_ws.p + 7);  // stays 0
  uint64_t* val = e->xr_val.p;
  uint32_t* val2 = e->def_score ? e->xr_val2.p : nullptr;
  uint32_t* affk = e->numa_on ? e->xr_aff.p : nullptr;
  const size_t norm_words = (size_t)kXrPods * kXrNorm, rec_words = (size_t)kXrPods * kCandStride;
  if (R > 1) {
    if (int rc = e->xr_norm_all.ensure(norm_words * R)) return rc;
    if (int rc = e->xr_rec_all.ensure(rec_words * R)) return rc;
  }
  auto issue_round = [&]() -> int {
    size_t t = prof_begin(e, e->stream);
#define KG_XR_EVAL(XF)                                                                                        \
  xr_eval<XF><<<xr_eval_blocks, kTile, 0, e->stream>>>(e->T, e->rsv_d.p, e->rsv_nd.p, e->pods.p, e->rpods.p, n, ntl, \
                                                       tile_base, stride, e->P, e->RP, X, val, val2, affk,          \
                                                       e->xr_part.p, e->rsv_ws.p)
    KG_XF_SWITCH(xf, KG_XR_EVAL);
#undef KG_XR_EVAL
    prof_end(e, KG_PROF_RSV_EVAL, t, e->stream);
    t = prof_begin(e, e->stream);
    if (R > 1) {  // the shard's statistics → every rank's → the global maxima and holder counts
      uint64_t* mine = e->xr_norm_all.p + norm_words * e->rank;
      xr_norm<<<kXrPods, 256, 0, e->stream>>>(e->xr_part.p, ntl, mine, e->rsv_ws.p);
      if (int rc = rank_allgather(e, e->xr_norm_all.p, norm_words, 0, e->stream)) return rc;
      xr_norm_combine<<<1, kXrPods * kXrNorm, 0, e->stream>>>(e->xr_norm_all.p, R, e->xr_norm_d.p, e->rsv_ws.p);
    } else {
      xr_norm<<<kXrPods, 256, 0, e->stream>>>(e->xr_part.p, ntl, e->xr_norm_d.p, e->rsv_ws.p);
    }
    xr_select<<<eval_blocks, kWave * kEvalWaves, 0, e->stream>>>(val, val2, n, ntl, tile_base, stride, vbits, e->RP, X,
                                                               e->xr_norm_d.p, e->xr_lists.p, e->rsv_ws.p);
    uint64_t* rec = R > 1 ? e->xr_rec_all.p + rec_words * e->rank : e->xr_cand.p;
    merge_round<false><<<kXrPods, kMergeThreads, 0, e->stream>>>(e->T, e->P, e->xr_lists.p, (int64_t)ntl * kR, kR, ntl,
                                                                 kR, kXrPods, poison, rec);
    if (R > 1) {  // every rank's record → the global record; the other shards' candidates evaluated here
      if (int rc = rank_allgather(e, e->xr_rec_all.p, rec_words, 0, e->stream)) return rc;
      merge_round<true><<<kXrPods, kMergeThreads, 0, e->stream>>>(e->T, e->P, e->xr_rec_all.p, kCandStride, rec_words,
                                                                  R, kC, kXrPods, poison, e->xr_cand.p);
#define KG_XR_FILL(XF)                                                                                              \
  xr_fill<XF><<<kXrPods * kXrPods, kWave, 0, e->stream>>>(e->T, e->rsv_d.p, e->rsv_nd.p, e->pods.p, e->rpods.p, n, lo, \
                                                          hi, stride, e->P, e->RP, X, e->xr_cand.p, val, val2, affk,  \
                                                          e->rsv_ws.p)
      KG_XF_SWITCH(xf, KG_XR_FILL);
#undef KG_XR_FILL
    }
    prof_end(e, KG_PROF_RSV_SELECT, t, e->stream);
    t = prof_begin(e, e->stream);
#define KG_XR_RESOLVE(XF)                                                                                      \
  xr_resolve<XF><<<1, kWave, lds, e->stream>>>(e->T, e->rsv_d.p, e->rsv_nd.p, e->pods.p, e->rpods.p, stride, e->P, \
                                               e->RP, X, val, val2, affk, e->xr_norm_d.p, e->xr_cand.p,          \
                                               bitmap_words, e->out_keys.p, e->out_rslot.p, e->rsv_ws.p)
    KG_XF_SWITCH(xf, KG_XR_RESOLVE);
#undef KG_XR_RESOLVE
    prof_end(e, KG_PROF_RSV_APPLY, t, e->stream);
    return 0;
  };
  static const bool no_graph = std::getenv("KG_RSV_NO_GRAPH") && std::getenv("KG_RSV_NO_GRAPH")[0] == '1';
  if (!no_graph && !e->prof_on && R == 1) {  // the instantiated graph of kXrGraphRounds rounds, keyed on its launch arguments
    std::vector<unsigned char> sig;
    auto put = [&](const void* q, size_t len) {
      const unsigned char* b = static_cast<const unsigned char*>(q);
      sig.insert(sig.end(), b, b + len);
    };
    put(&e->T, sizeof(e->T));
    const void* ptrs[] = {e->rsv_d.p, e->rsv_nd.p, e->pods.p, e->rpods.p, val, val2, affk, e->xr_part.p,
                          e->xr_norm_d.p, e->xr_lists.p, e->xr_cand.p, e->out_keys.p, e->out_rslot.p, e->rsv_ws.p};
    put(ptrs, sizeof(ptrs));
    put(&n, sizeof(n));
    put(&e->P, sizeof(e->P));
    put(&e->RP, sizeof(e->RP));
    put(&X, sizeof(X));
    if (!e->xr_exec || sig != e->xr_exec_sig) {
      if (e->xr_exec) (void)hipGraphExecDestroy(e->xr_exec);
      e->xr_exec = nullptr;
      hipGraph_t gr = nullptr;
      HIP_TRY(hipStreamBeginCapture(e->stream, hipStreamCaptureModeThreadLocal));
      for (int r = 0; r < kXrGraphRounds; ++r) (void)issue_round();
      const hipError_t ce = hipStreamEndCapture(e->stream, &gr);
      if (ce != hipSuccess) return fail(KG_E_DEVICE, "hipStreamEndCapture: %s", hipGetErrorString(ce));
      const hipError_t ie = hipGraphInstantiate(&e->xr_exec, gr, nullptr, nullptr, 0);
      (void)hipGraphDestroy(gr);
      if (ie != hipSuccess) {
        e->xr_exec = nullptr;
        return fail(KG_E_DEVICE, "exact rounds graph: %s", hipGetErrorString(ie));
      }
      e->xr_exec_sig = sig;
    }
  }
  int64_t cursor = first, launched = 0;
  unsigned long long ws[8];
  while (cursor < end) {
    // rounds for the pods left at the recent rate (at least one graph), then one check of the cursor
    const double per = std::max(1.0, e->xr_avg);
    int64_t rounds = (int64_t)std::ceil((double)(end - cursor) / per);
    rounds = std::max<int64_t>(1, std::min<int64_t>(rounds, kMaxBatchRounds));
    if (e->xr_exec && !e->prof_on && R == 1) {
      const int64_t graphs = (rounds + kXrGraphRounds - 1) / kXrGraphRounds;
      for (int64_t g = 0; g < graphs; ++g) {
        const hipError_t ge = hipGraphLaunch(e->xr_exec, e->stream);
        if (ge != hipSuccess) return fail(KG_E_DEVICE, "exact rounds graph: %s", hipGetErrorString(ge));
      }
      rounds = graphs * kXrGraphRounds;
    } else {
      for (int64_t r = 0; r < rounds; ++r)  // (several ranks: every rank issues the same rounds, so the collectives pair)
        if (int rc = issue_round()) return rc;
      HIP_TRY(hipGetLastError());
    }
    launched += rounds;
    HIP_TRY(hipMemcpyAsync(ws, e->rsv_ws.p, sizeof(ws), hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    if (e->prof_on)
      if (int rc = prof_collect(e)) return rc;
    const int64_t c = (int64_t)ws[3];
    if (c <= cursor) return fail(KG_E_DEVICE, "exact rounds made no progress at pod %lld", (long long)cursor);
    cursor = c;
    if (ws[5] > 0) e->xr_avg = 0.5 * e->xr_avg + 0.5 * ((double)ws[6] / (double)ws[5]);
  }
  if (stats) {
    std::memset(stats, 0, sizeof(*stats));
    stats->device_batches = (int64_t)ws[5];
    stats->node_evaluations = (int64_t)ws[5] * kXrPods * n;
    stats->seconds = now_s() - t0;
  }
  (void)launched;
  return 0;
}

int decode_node_rsv(const kg_node_reservations& r, RsvNode& d, int32_t& ns, RsvGpu* g, bool ds_on, RsvCpu* c,
                    bool numa_on) {
  std::memset(&d, 0, sizeof(d));
  std::memset(g, 0, sizeof(RsvGpu) * kRsvSlots);
  std::memset(c, 0, sizeof(RsvCpu) * kRsvSlots);
  if (r.n < 0 || r.n > KG_MAX_RSV_SLOTS) return fail(KG_E_INVALID, "reservation slot count %lld", (long long)r.n);
  if (r.predicate_count < 0 || r.predicate_count > 64)
    return fail(KG_E_INVALID, "reservation predicate_count %lld outside [0, 64]", (long long)r.predicate_count);
  ns = (int32_t)r.n;
  for (int s = 0; s < ns; ++s) {
    if (r.allocatable_cpu[s] < 0 || r.allocatable_mem[s] < 0 || r.allocatable_cpu[s] > (int64_t(1) << 40) ||
        r.allocatable_mem[s] > (int64_t(1) << 46))
      return fail(KG_E_UNSUPPORTED, "reservation slot %d: allocatable cpu / memory outside [0, 2^40] / [0, 2^46]", s);
    if (r.allocated_cpu[s] < 0 || r.allocated_mem[s] < 0 || r.allocated_cpu[s] > (int64_t(1) << 40) ||
        r.allocated_mem[s] > (int64_t(1) << 46) || r.assigned[s] < 0 || r.assigned[s] > INT32_MAX / 2)
      return fail(KG_E_INVALID, "reservation slot %d: allocated / assigned out of range", s);
    if (r.order[s] < 0 || r.order[s] >= INT32_MAX) return fail(KG_E_UNSUPPORTED, "reservation slot %d: order outside [0, 2^31-1)", s);
    if (r.owner[s] < 0 || r.owner[s] >= KG_MAX_OWNER_GROUPS)
      return fail(KG_E_UNSUPPORTED, "reservation slot %d: owner group outside [0, %d)", s, KG_MAX_OWNER_GROUPS);
    if (r.policy[s] < KG_RSV_POLICY_DEFAULT || r.policy[s] > KG_RSV_POLICY_RESTRICTED) return fail(KG_E_INVALID, "reservation policy");
    d.alloc_cpu[s] = r.allocatable_cpu[s];
    d.alloc_mem[s] = r.allocatable_mem[s];
    d.allocd_cpu[s] = r.allocated_cpu[s];
    d.allocd_mem[s] = r.allocated_mem[s];
    d.owner[s] = (int32_t)r.owner[s];
    d.assigned[s] = (int32_t)r.assigned[s];
    d.order[s] = (int32_t)r.order[s];
    d.meta[s] = (r.available[s] ? RS_AVAIL : 0u) | (r.allocate_once[s] ? RS_ONCE : 0u) |
                (r.unschedulable[s] ? RS_UNSCHED : 0u) | ((uint32_t)r.policy[s] << 4);
    // (ABI 15) the cpuset the reservation holds and its assigned pods' (NodeNUMAResource only reads them)
    uint64_t any = 0;
    for (int w = 0; w < kCpuWords; ++w) any |= r.cpus[s][w];
    if (any && numa_on) {
      for (int w = 0; w < kCpuWords; ++w) {
        c[s].r[w] = r.cpus[s][w];
        c[s].u[w] = r.cpus_assigned[s][w];
      }
      d.meta[s] |= RS_CPUS;
    }
    // (ABI 13) the GPUs the reservation holds (DeviceShare only reads them)
    if (r.gpu_minors[s] < 0 || r.gpu_minors[s] >= (int64_t(1) << kMinors))
      return fail(KG_E_INVALID, "reservation slot %d: gpu_minors outside [0, 2^%d)", s, kMinors);
    if (r.gpu_minors[s] == 0 || !ds_on) continue;
    RsvGpu& G = g[s];
    G.minors = (uint32_t)r.gpu_minors[s];
    for (int m = 0; m < kMinors; ++m)
      for (int q = 0; q < 3; ++q) {
        const int64_t lim = q == 1 ? (int64_t(1) << 46) : (int64_t(1) << 30);
        const int64_t A = r.gpu_alloc[s][m][q], a = r.gpu_allocated[s][m][q];
        if (A < 0 || a < 0 || A > lim || a > lim)
          return fail(KG_E_UNSUPPORTED, "reservation slot %d minor %d: gpu allocatable / allocated outside [0, %s]", s,
                      m, q == 1 ? "2^46" : "2^30");
      }
    for (int m = 0; m < kMinors; ++m) {
      G.acore[m] = (int32_t)r.gpu_alloc[s][m][0];
      G.amem[m] = r.gpu_alloc[s][m][1];
      G.aratio[m] = (int32_t)r.gpu_alloc[s][m][2];
      G.dcore[m] = (int32_t)r.gpu_allocated[s][m][0];
      G.dmem[m] = r.gpu_allocated[s][m][1];
      G.dratio[m] = (int32_t)r.gpu_allocated[s][m][2];
    }
    d.meta[s] |= RS_GPU;
  }
  return 0;
}

// 1 + the highest predicate id a pod's reservation affinity uses (0: none)
int64_t rsv_pred_top(const RsvPod& d, const RsvSel& c) {
  if (!(d.flags & RP_SEL)) return 0;
  uint64_t used = c.sel;
  for (uint32_t t = 0; t < c.nterms; ++t) used |= c.terms[t];
  return used ? 64 - __builtin_clzll(used) : 0;
}

// the Reservation view of one pod: owner groups, the required-affinity flag and (ABI 12) its selector / terms (RP_SEL:
// the caller points aux at where it stores `c`), the reserve pod's node and allocate policy
int decode_rsv_pod(const kg_pod& p, RsvPod& d, RsvSel& c, int64_t k) {
  std::memset(&d, 0, sizeof(d));
  std::memset(&c, 0, sizeof(c));
  if (p.n_reservation_terms < 0 || p.n_reservation_terms > KG_MAX_AFF_TERMS)
    return fail(KG_E_UNSUPPORTED, "pod %lld: more than %d reservation affinity terms (the pod stays on the Go path)",
                (long long)k, KG_MAX_AFF_TERMS);
  d.owner_mask = (uint64_t)p.reservation_owner_mask;
  d.flags = ((p.reservation_flags & KG_POD_RSV_AFFINITY) ? RP_AFFINITY : 0u) |
            ((p.flags & KG_POD_RESERVE) ? RP_RESERVE : 0u) | ((p.reservation_flags & KG_POD_RSV_OPERATING) ? RP_OPERATING : 0u);
  d.aux = -1;
  if (p.flags & KG_POD_RESERVE) {
    if (p.reserve_allocate_policy < KG_RSV_POLICY_DEFAULT || p.reserve_allocate_policy > KG_RSV_POLICY_RESTRICTED)
      return fail(KG_E_INVALID, "pod %lld: reserve_allocate_policy %lld", (long long)k, (long long)p.reserve_allocate_policy);
    if (p.reserve_node < 0 || p.reserve_node > INT32_MAX)
      return fail(KG_E_INVALID, "pod %lld: reserve_node %lld", (long long)k, (long long)p.reserve_node);
    d.aux = (int32_t)p.reserve_node - 1;
    d.flags |= (uint32_t)p.reserve_allocate_policy << RP_POLICY_SHIFT;
  } else {
    d.flags |= (uint32_t)KG_RSV_POLICY_ALIGNED << RP_POLICY_SHIFT;  // operating mode checks as Aligned
    c.nterms = (uint32_t)p.n_reservation_terms;
    c.sel = p.reservation_selector;
    for (uint32_t t = 0; t < c.nterms; ++t) c.terms[t] = p.reservation_terms[t];
    // a reserve pod matches no reservation, so its selectors are never read
    if ((d.flags & RP_AFFINITY) && (c.sel != 0 || c.nterms != 0)) d.flags |= RP_SEL;
  }
  return 0;
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------------------
extern "C" {

int kg_abi_version(void) { return KG_ABI_VERSION; }

int64_t kg_abi_struct_size(int which) {
  switch (which) {
    case 0: return sizeof(kg_config);
    case 1: return sizeof(kg_node);
    case 2: return sizeof(kg_node_metric);
    case 3: return sizeof(kg_pod);
    case 4: return sizeof(kg_stats);
    case 5: return sizeof(kg_node_numa);
    case 6: return sizeof(kg_node_device);
    case 7: return sizeof(kg_quota);
    case 8: return sizeof(kg_node_reservations);
    case 9: return sizeof(kg_pod_metric);
    case 10: return sizeof(kg_node_predicates);
  }
  return -1;
}
const char* kg_last_error(void) { return g_err.c_str(); }

void kg_config_default(kg_config* c) {
  std::memset(c, 0, sizeof(*c));
  c->abi_version = KG_ABI_VERSION;
  // v1beta2.SetDefaults_LoadAwareSchedulingArgs (pkg/scheduler/apis/config/v1beta2/defaults.go:76-99, 30-48)
  c->la_filter_expired_node_metrics = 1;
  c->la_node_metric_expiration_seconds = 180;
  c->la_resource_weights[KG_RES_CPU] = 1;
  c->la_resource_weights[KG_RES_MEMORY] = 1;
  c->la_usage_thresholds[KG_RES_CPU] = 65;
  c->la_usage_thresholds[KG_RES_MEMORY] = 95;
  c->la_estimated_scaling_factors[KG_RES_CPU] = 85;
  c->la_estimated_scaling_factors[KG_RES_MEMORY] = 70;
  // upstream NodeResourcesFit default scoring strategy: LeastAllocated, cpu:1 memory:1
  c->fit_resource_weights[KG_RES_CPU] = 1;
  c->fit_resource_weights[KG_RES_MEMORY] = 1;
  c->fit_filter = c->fit_score = c->la_filter = c->la_score = 1;
  c->weight_fit = 1;
  c->weight_loadaware = 1;
  // v1beta2.SetDefaults_NodeNUMAResourceArgs (defaults.go:101-137): FullPCPUs, LeastAllocated cpu:1 memory:1 for
  // both the node and the NUMA scoring strategies; the plugin is off unless the profile enables it
  c->weight_numa = 1;
  c->numa_default_cpu_bind_policy = KG_BIND_FULL_PCPUS;
  c->numa_scoring_strategy = KG_STRATEGY_LEAST_ALLOCATED;
  c->numa_scoring_weights[0] = c->numa_scoring_weights[1] = 1;
  c->numa_numa_scoring_strategy = KG_STRATEGY_LEAST_ALLOCATED;
  c->numa_numa_scoring_weights[0] = c->numa_numa_scoring_weights[1] = 1;
  c->batch_pods = 32;
  c->pods_per_wave = 8;
  c->device_id = -1;
  // (ABI 12) upstream v1beta2 defaults: PodTopologySpread weight 2, InterPodAffinity weight 1, HardPodAffinityWeight 1
  c->weight_spread = 2;
  c->weight_interpod = 1;
  c->hard_pod_affinity_weight = 1;
}

int kg_debug_rccl_selftest(int device_id, int64_t n) {
  if (n < 1 || n > (1 << 24)) return fail(KG_E_INVALID, "n in [1, 2^24]");
  HIP_TRY(hipSetDevice(device_id));
  ncclUniqueId id;
  NCCL_TRY(ncclGetUniqueId(&id));
  ncclComm_t c = nullptr, c2 = nullptr;
  if (ncclCommInitRank(&c, 1, id, 0) != ncclSuccess) return fail(KG_E_COLLECTIVE, "ncclCommInitRank");
  int rc = 0;
  hipStream_t st = nullptr;
  uint64_t *in = nullptr, *out = nullptr;
  std::vector<uint64_t> h(n), g(n);
  for (int64_t i = 0; i < n; ++i) h[i] = 0x9E3779B97F4A7C15ull * (uint64_t)(i + 1);
  if (ncclCommSplit(c, 0, 0, &c2, nullptr) != ncclSuccess) rc = fail(KG_E_COLLECTIVE, "ncclCommSplit");
  if (!rc && (hipStreamCreate(&st) != hipSuccess || hipMalloc(&in, n * 8) != hipSuccess ||
              hipMalloc(&out, n * 8) != hipSuccess))
    rc = fail(KG_E_DEVICE, "stream / buffers");
  if (!rc && (hipMemcpy(in, h.data(), n * 8, hipMemcpyHostToDevice) != hipSuccess ||
              hipMemset(out, 0, n * 8) != hipSuccess))
    rc = fail(KG_E_DEVICE, "upload");
  if (!rc && ncclAllGather(in, out, (size_t)n, ncclUint64, c2, st) != ncclSuccess)
    rc = fail(KG_E_COLLECTIVE, "ncclAllGather");
  if (!rc && (hipStreamSynchronize(st) != hipSuccess || hipMemcpy(g.data(), out, n * 8, hipMemcpyDeviceToHost) != hipSuccess))
    rc = fail(KG_E_DEVICE, "download");
  if (!rc && g != h) rc = fail(KG_E_COLLECTIVE, "ncclAllGather returned different words");
  if (out) (void)hipFree(out);
  if (in) (void)hipFree(in);
  if (st) (void)hipStreamDestroy(st);
  if (c2) ncclCommDestroy(c2);
  ncclCommDestroy(c);
  return rc;
}

int kg_nccl_unique_id(void* out128) {
  if (!out128) return fail(KG_E_INVALID, "out is NULL");
  ncclUniqueId id;
  NCCL_TRY(ncclGetUniqueId(&id));
  static_assert(sizeof(id) == 128, "ncclUniqueId size");
  std::memcpy(out128, &id, sizeof(id));
  return 0;
}

// (r6) auto multi-rank mode: the smallest tables worth sharding (DESIGN.md §6 model)
constexpr int64_t kShardMinNodes = 262144;      // round profiles: one GPU's wide pass > exchange + second merge
constexpr int64_t kShardMinNodesExact = 32768;  // batched exact rounds of NodeNUMAResource / DeviceShare profiles

static int engine_create(const kg_config* cfg, int64_t capacity_nodes, int rank, int n_ranks, const void* nccl_id,
                         kg_loopback* lb, kg_engine** out, kg_exchange_fn xfn = nullptr, void* xuser = nullptr) {
  if (!out) return fail(KG_E_INVALID, "out is NULL");
  *out = nullptr;
  if (int rc = validate_config(cfg)) return rc;
  if (capacity_nodes <= 0 || capacity_nodes > kMaxNodes) return fail(KG_E_INVALID, "capacity_nodes out of range");
  if (n_ranks < 1 || rank < 0 || rank >= n_ranks) return fail(KG_E_INVALID, "rank/n_ranks");
  if (n_ranks > 1 && !nccl_id && !lb && !xfn) return fail(KG_E_INVALID, "nccl_unique_id required for n_ranks>1");
  if (lb) {
    std::lock_guard<std::mutex> lk(lb->mu);
    if (lb->n != n_ranks) return fail(KG_E_INVALID, "loopback group of %d ranks, engine n_ranks %d", lb->n, n_ranks);
    if (lb->ranks[rank]) return fail(KG_E_INVALID, "loopback rank %d already has an engine", rank);
  }
  kg_engine* e = new kg_engine();
  e->cfg = *cfg;
  if (e->cfg.batch_pods == 0) e->cfg.batch_pods = 32;
  e->rank = rank;
  e->n_ranks = n_ranks;
  const int64_t cap = ((capacity_nodes + kTile - 1) / kTile) * kTile;
  e->capacity = cap;
  auto bail = [&](int rc) {
    kg_engine_destroy(e);
    return rc;
  };
  if (cfg->device_id >= 0) {
    if (hipSetDevice((int)cfg->device_id) != hipSuccess) return bail(fail(KG_E_DEVICE, "hipSetDevice(%lld)", (long long)cfg->device_id));
  }
  if (hipGetDevice(&e->device) != hipSuccess) return bail(fail(KG_E_DEVICE, "no HIP device"));
  if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) return bail(fail(KG_E_DEVICE, "hipStreamCreate"));
  {  // round streams at the device's highest priority (the serial resolve chain runs on them)
    int lo = 0, hi = 0;
    if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) return bail(fail(KG_E_DEVICE, "hipDeviceGetStreamPriorityRange"));
    for (int k = 0; k < kMaxDepth; ++k) {
      if (hipStreamCreateWithPriority(&e->rs[k], hipStreamNonBlocking, hi) != hipSuccess)
        return bail(fail(KG_E_DEVICE, "hipStreamCreateWithPriority"));
      if (hipEventCreateWithFlags(&e->ev_res[k], hipEventDisableTiming) != hipSuccess)
        return bail(fail(KG_E_DEVICE, "hipEventCreate"));
    }
  }
  // 12 int64 columns + inv_mem[2] (f64) + the kAux resources' Allocatable / Requested
  if (int rc = e->cols64.ensure((14 + 2 * kAux) * cap)) return bail(rc);
  if (int rc = e->cols32.ensure(5 * cap)) return bail(rc);   // alloc_pods, num_pods, flags, inv_cpu[2] (f32)
  if (hipMemsetAsync(e->cols64.p, 0, (14 + 2 * kAux) * cap * 8, e->stream) != hipSuccess || hipMemsetAsync(e->cols32.p, 0, 5 * cap * 4, e->stream) != hipSuccess)
    return bail(fail(KG_E_DEVICE, "hipMemset"));
  int64_t* c64 = e->cols64.p;
  e->T.alloc_cpu = c64 + 0 * cap;
  e->T.alloc_mem = c64 + 1 * cap;
  e->T.req_cpu = c64 + 2 * cap;
  e->T.req_mem = c64 + 3 * cap;
  e->T.nz_cpu = c64 + 4 * cap;
  e->T.nz_mem = c64 + 5 * cap;
  e->T.la_alloc_cpu = c64 + 6 * cap;
  e->T.la_alloc_mem = c64 + 7 * cap;
  e->T.la_used_cpu = c64 + 8 * cap;
  e->T.la_used_mem = c64 + 9 * cap;
  e->T.la_pused_cpu = c64 + 10 * cap;
  e->T.la_pused_mem = c64 + 11 * cap;
  e->T.alloc_pods = e->cols32.p + 0 * cap;
  e->T.num_pods = e->cols32.p + 1 * cap;
  e->T.flags = (uint32_t*)(e->cols32.p + 2 * cap);
  e->T.inv_cpu = (float*)(e->cols32.p + 3 * cap);
  e->T.inv_mem = (double*)(e->cols64.p + 12 * cap);
  e->T.aux = e->cols64.p + 14 * cap;
  e->T.cap = cap;
  if (int rc = e->cursor.ensure(16)) return bail(rc);
  if (hipMemsetAsync(e->cursor.p, 0, 16 * 8, e->stream) != hipSuccess) return bail(fail(KG_E_DEVICE, "hipMemset"));
  if (int rc = e->modlists.ensure(kMaxDepth * kModListStride)) return bail(rc);
  if (hipMemsetAsync(e->modlists.p, 0, kMaxDepth * kModListStride * 4, e->stream) != hipSuccess) return bail(fail(KG_E_DEVICE, "hipMemset"));
  if (int rc = e->tickets.ensure(kMaxDepth * kMaxB)) return bail(rc);
  if (hipMemsetAsync(e->tickets.p, 0, kMaxDepth * kMaxB * 4, e->stream) != hipSuccess) return bail(fail(KG_E_DEVICE, "hipMemset"));
  e->nodes.assign(cap, kg_node{});
  e->metrics.assign(cap, kg_node_metric{});
  e->folded_usage.assign(2 * cap, 0);
  e->folded_prod.assign(2 * cap, 0);
  e->assigned.assign(cap, {});
  e->pmetrics.assign(cap, {});
  e->now_of.assign(cap, 0);
  // EvalParams
  const kg_config& c = e->cfg;
  e->P.fit_w_cpu = c.fit_resource_weights[KG_RES_CPU];
  e->P.fit_w_mem = c.fit_resource_weights[KG_RES_MEMORY];
  e->P.la_w_cpu = c.la_resource_weights[KG_RES_CPU];
  e->P.la_w_mem = c.la_resource_weights[KG_RES_MEMORY];
  e->P.la_wsum = std::max<int64_t>(1, e->P.la_w_cpu + e->P.la_w_mem);
  e->P.weight_fit = c.weight_fit;
  e->P.weight_la = c.weight_loadaware;
  e->P.fit_filter = (int)(c.fit_filter != 0);
  e->P.fit_score = (int)(c.fit_score != 0);
  e->P.la_filter = (int)(c.la_filter != 0);
  e->P.la_score = (int)(c.la_score != 0);
  e->numa_on = c.numa_filter || c.numa_score;
  e->ds_on = c.ds_filter || c.ds_score;
  e->rsv_on = c.reservation_filter || c.reservation_score;
  e->grp_on = c.spread_filter || c.spread_score || c.interpod_filter || c.interpod_score;
  // (the group plugins read the pods' nodeSelector / required node affinity: the predicate tables come with them)
  e->def_on = c.taint_filter || c.taint_score || c.affinity_filter || c.affinity_score || c.balanced_score ||
              c.image_score || e->grp_on;
  e->def_score = c.taint_score || c.affinity_score;
  e->exact_on = e->rsv_on || (e->numa_on && e->ds_on) || e->def_on;
  // (r6) Several ranks: node-sharded evaluation with a per-round exchange, or every rank a replica of one GPU (its own
  // full table, the same FIFO resolve, no exchange).  The replicated single-wave resolver bounds the period at any
  // rank count, and sharding adds the all-gather and a second merge to the critical cycle (DESIGN.md §6, r5 numbers),
  // so it pays only where one GPU's wide pass is long: auto shards the round profiles from kShardMinNodes nodes and
  // the batched exact rounds of NodeNUMAResource / DeviceShare profiles from kShardMinNodesExact.  Either way every
  // rank holds the same placements.
  if (c.multi_rank_mode < KG_MULTI_RANK_AUTO || c.multi_rank_mode > KG_MULTI_RANK_REPLICA)
    return bail(fail(KG_E_INVALID, "multi_rank_mode %lld", (long long)c.multi_rank_mode));
  if (n_ranks > 1) {
    const bool heavy_exact = e->exact_on && !e->grp_on && (e->numa_on || e->ds_on);
    const bool shard = c.multi_rank_mode == KG_MULTI_RANK_SHARD ||
                       (c.multi_rank_mode == KG_MULTI_RANK_AUTO &&
                        capacity_nodes >= (e->exact_on ? (heavy_exact ? kShardMinNodesExact : INT64_MAX) : kShardMinNodes));
    if (!shard) {  // a replica: the engine of one GPU (no collective, no exchange)
      e->replica_ranks = n_ranks;
      e->rank = rank = 0;
      e->n_ranks = n_ranks = 1;
      lb = nullptr;
      xfn = nullptr;
    }
  }
  e->DF = DefParams{(int32_t)(c.taint_filter != 0), (int32_t)(c.taint_score != 0), (int32_t)c.weight_taint,
                    (int32_t)(c.affinity_filter != 0), (int32_t)(c.affinity_score != 0), (int32_t)c.weight_affinity,
                    (int32_t)(c.balanced_score != 0), (int32_t)c.weight_balanced,
                    (int32_t)(c.balanced_resources & 1), (int32_t)((c.balanced_resources >> 1) & 1),
                    (int32_t)(c.image_score != 0), (int32_t)c.weight_image};
  if (e->def_on) {
    if (int rc = e->npred.ensure(cap)) return bail(rc);
    if (hipMemsetAsync(e->npred.p, 0, cap * sizeof(NodePred), e->stream) != hipSuccess) return bail(fail(KG_E_DEVICE, "hipMemset"));
    e->np_taint_top.assign(cap, 0);
    e->np_pred_cnt.assign(cap, 0);
    e->np_img_cnt.assign(cap, 0);
    if (e->def_score)
      if (int rc = e->rsv_val2.ensure(cap)) return bail(rc);
  }
  e->GP = GroupParams{(int32_t)(c.spread_filter != 0), (int32_t)(c.spread_score != 0), (int32_t)c.weight_spread,
                      (int32_t)(c.interpod_filter != 0), (int32_t)(c.interpod_score != 0), (int32_t)c.weight_interpod,
                      (int32_t)c.hard_pod_affinity_weight, 0};
  if (e->grp_on) {
    if (int rc = e->grp_d.ensure((size_t)kGroupArrays * kGroups * cap)) return bail(rc);
    if (int rc = e->logw.ensure(cap + 1)) return bail(rc);
    if (int rc = e->gval.ensure(cap)) return bail(rc);
    if (int rc = e->gz.ensure((size_t)2 * kZoneSumWords)) return bail(rc);
    if (int rc = e->gzm.ensure(2)) return bail(rc);
    std::vector<double> lw((size_t)cap + 1);
    for (int64_t f = 0; f <= cap; ++f) lw[f] = go_log((double)(f + 2));  // TopologyNormalizingWeight (Go's Log)
    if (hipMemsetAsync(e->grp_d.p, 0, (size_t)kGroupArrays * kGroups * cap * 4, e->stream) != hipSuccess ||
        hipMemcpyAsync(e->logw.p, lw.data(), lw.size() * 8, hipMemcpyHostToDevice, e->stream) != hipSuccess ||
        hipStreamSynchronize(e->stream) != hipSuccess)
      return bail(fail(KG_E_DEVICE, "group tables"));
  }
  e->RP.filter = (int32_t)(c.reservation_filter != 0);
  e->RP.score = (int32_t)(c.reservation_score != 0);
  e->RP.weight = (int32_t)c.weight_reservation;
  {  // the exact pass's tables: its profiles, and single-pod calls of every profile (schedule_staged_impl)
    if (e->numa_on)
      if (int rc = e->numa_aff.ensure(cap)) return bail(rc);
    if (int rc = e->rsv_d.ensure(cap)) return bail(rc);
    if (int rc = e->rsv_nd.ensure(cap)) return bail(rc);
    if (int rc = e->rsv_pd.ensure((size_t)kRsvSlots * cap)) return bail(rc);
    if (int rc = e->rsv_val.ensure(cap)) return bail(rc);
    if (int rc = e->rsv_ws.ensure(8)) return bail(rc);
    if (int rc = e->rsv_part.ensure(15 * ((cap + kRsvThreads - 1) / kRsvThreads) + 4)) return bail(rc);
    if (hipMemsetAsync(e->rsv_nd.p, 0, cap * 4, e->stream) != hipSuccess || hipMemsetAsync(e->rsv_ws.p, 0, 64, e->stream) != hipSuccess ||
        hipMemsetAsync(e->rsv_pd.p, 0, (size_t)kRsvSlots * cap * 8, e->stream) != hipSuccess)
      return bail(fail(KG_E_DEVICE, "hipMemset"));
  }
  {
    const char* xr = std::getenv("KG_EXACT_ROUNDS");
    e->xr_on = !(xr && xr[0] == '0');
  }
  if (e->exact_on && e->xr_on) {  // batched exact rounds
    const size_t nt = (size_t)((cap + kTile - 1) / kTile);
    if (int rc = e->xr_val.ensure((size_t)kXrPods * cap)) return bail(rc);
    if (e->def_score)
      if (int rc = e->xr_val2.ensure((size_t)kXrPods * cap)) return bail(rc);
    if (e->numa_on)
      if (int rc = e->xr_aff.ensure((size_t)kXrPods * cap)) return bail(rc);
    if (int rc = e->xr_part.ensure((size_t)kXrPods * nt * kXrNorm)) return bail(rc);
    if (int rc = e->xr_norm_d.ensure((size_t)kXrPods * kXrNorm)) return bail(rc);
    if (int rc = e->xr_lists.ensure((size_t)kXrPods * nt * kR)) return bail(rc);
    if (int rc = e->xr_cand.ensure((size_t)kXrPods * kCandStride)) return bail(rc);
    if (hipMemsetAsync(e->xr_lists.p, 0, (size_t)kXrPods * nt * kR * 8, e->stream) != hipSuccess)
      return bail(fail(KG_E_DEVICE, "hipMemset"));
    hipError_t fe = hipSuccess;
#define KG_XR_ATTR(XF) \
  fe = hipFuncSetAttribute((const void*)xr_resolve<XF>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024)
    for (int xf = 0; xf < 8 && fe == hipSuccess; ++xf) KG_XF_SWITCH(xf, KG_XR_ATTR);
#undef KG_XR_ATTR
    if (fe != hipSuccess) return bail(fail(KG_E_DEVICE, "hipFuncSetAttribute(xr_resolve LDS)"));
  }
  const int64_t max_total = 100 * ((c.fit_score ? c.weight_fit : 0) + (c.la_score ? c.weight_loadaware : 0) +
                                   (c.numa_score ? c.weight_numa : 0) + (c.ds_score ? c.weight_deviceshare : 0) +
                                   (c.reservation_score ? c.weight_reservation : 0) +
                                   (c.taint_score ? c.weight_taint : 0) + (c.affinity_score ? c.weight_affinity : 0) +
                                   (c.balanced_score ? c.weight_balanced : 0) + (c.image_score ? c.weight_image : 0) +
                                   (c.spread_score ? c.weight_spread : 0) + (c.interpod_score ? c.weight_interpod : 0));
  e->P.score_bits = (int32_t)bits_for(max_total);
  // NodeResourcesFit + LoadAwareScheduling: assume only lowers a node's key; NodeNUMAResource does not
  e->P.monotone = (e->numa_on || e->ds_on || e->rsv_on) ? 0 : 1;  // DeviceShare: normalization couples every node's key
  e->DP.filter = (int32_t)(c.ds_filter != 0);
  e->DP.score = (int32_t)(c.ds_score != 0);
  e->DP.weight = (int32_t)c.weight_deviceshare;
  e->DP.w_core = (int32_t)c.ds_scoring_weights[0];
  e->DP.w_mem = (int32_t)c.ds_scoring_weights[1];
  e->DP.w_ratio = (int32_t)c.ds_scoring_weights[2];
  e->DP.most = (int32_t)(c.ds_scoring_strategy == KG_STRATEGY_MOST_ALLOCATED);
  e->DP.w_x[KG_XTYPE_RDMA] = (int32_t)c.ds_scoring_weights_x[KG_XTYPE_RDMA];
  e->DP.w_x[KG_XTYPE_FPGA] = (int32_t)c.ds_scoring_weights_x[KG_XTYPE_FPGA];
  if (e->ds_on) {
    if (int rc = e->dsx_d.ensure(cap)) return bail(rc);
    if (hipMemsetAsync(e->dsx_d.p, 0, cap * sizeof(DsXNode), e->stream) != hipSuccess)
      return bail(fail(KG_E_DEVICE, "hipMemset"));
    if (int rc = e->ds_d.ensure(cap)) return bail(rc);
    e->ds_host.assign(cap, DsNode{});
    for (auto& d : e->ds_host) d.first = -1;
    if (hipMemcpyAsync(e->ds_d.p, e->ds_host.data(), cap * sizeof(DsNode), hipMemcpyHostToDevice, e->stream) != hipSuccess)
      return bail(fail(KG_E_DEVICE, "hipMemcpy"));
    const int lds = (int)(kMaxNodes / 8 + ((size_t)32 * (kCandStride + kPodWords + kDsPodWords + kDsNodeWords + kQuotaRes) +
                                           (size_t)kWave * kDsNodeWords) * 8 + KG_MAX_QUOTAS * sizeof(QuotaRow) +
                          32 * sizeof(Row) + (size_t)kWave * (sizeof(DsNode) + sizeof(Row)));
    const int lds_cap = (int)std::min<size_t>((size_t)lds, 160 * 1024);  // prepare_rounds checks the real need
    if (hipFuncSetAttribute((const void*)resolve_round_ds, hipFuncAttributeMaxDynamicSharedMemorySize, lds_cap) != hipSuccess)
      return bail(fail(KG_E_DEVICE, "hipFuncSetAttribute(resolve_round_ds LDS)"));
  }
  e->NP.filter = (int32_t)(c.numa_filter != 0);
  e->NP.score = (int32_t)(c.numa_score != 0);
  e->NP.weight = (int32_t)c.weight_numa;
  e->NP.node_strategy = (int32_t)c.numa_scoring_strategy;
  e->NP.numa_strategy = (int32_t)c.numa_numa_scoring_strategy;
  e->NP.w_cpu = (int32_t)c.numa_scoring_weights[0];
  e->NP.w_mem = (int32_t)c.numa_scoring_weights[1];
  e->NP.nw_cpu = (int32_t)c.numa_numa_scoring_weights[0];
  e->NP.nw_mem = (int32_t)c.numa_numa_scoring_weights[1];
  // GetDefaultNUMAAllocateStrategy (util.go:26-32): MostAllocated iff the NUMA scoring strategy is
  e->NP.default_alloc_strategy = c.numa_numa_scoring_strategy == KG_STRATEGY_MOST_ALLOCATED ? 1 : 0;
  if (e->numa_on) {
    if (int rc = e->numa_s.ensure(cap)) return bail(rc);
    if (int rc = e->numa_m.ensure(cap)) return bail(rc);
    if (hipMemsetAsync(e->numa_s.p, 0, cap * sizeof(NumaStatic), e->stream) != hipSuccess ||
        hipMemsetAsync(e->numa_m.p, 0, cap * sizeof(NumaMut), e->stream) != hipSuccess)
      return bail(fail(KG_E_DEVICE, "hipMemset"));
    const int lds = (int)(kMaxNodes / 8 + ((size_t)kMaxB * (kCandStride + kPodWords + kNumaPodWords) +
                                           (size_t)kWave * (kNumaStaticWords + kNumaMutWords)) * 8);
    if (hipFuncSetAttribute((const void*)resolve_round_numa, hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess ||
        hipFuncSetAttribute((const void*)resolve_round_numa2, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)std::min<size_t>(lds + numa2_extra_lds_bytes() + numa2_pre_lds_bytes(kMaxB), kMaxLds)) !=
            hipSuccess)
      return bail(fail(KG_E_DEVICE, "hipFuncSetAttribute(resolve_round_numa LDS)"));
  }
  e->P.inv_la_wsum = 1.0f / (float)e->P.la_wsum;
  e->P.fit_wsum32 = (int32_t)(e->P.fit_w_cpu + e->P.fit_w_mem);
  e->P.la_prod_score = (int32_t)(c.la_score_according_prod_usage != 0);
  {
    const float wc = (float)e->P.fit_w_cpu, wm = (float)e->P.fit_w_mem;
    e->P.inv_fit_ws[0] = 0.0f;
    e->P.inv_fit_ws[1] = wc > 0 ? 1.0f / wc : 0.0f;
    e->P.inv_fit_ws[2] = wm > 0 ? 1.0f / wm : 0.0f;
    e->P.inv_fit_ws[3] = wc + wm > 0 ? 1.0f / (wc + wm) : 0.0f;
  }
#ifdef KG_DEV_PF  // (r5) an iteration build refuses other profiles here, as a product build refuses what it lacks
  if (profile_bits(e->P) != KG_DEV_PF)
    return bail(fail(KG_E_UNSUPPORTED, "iteration build (KG_DEV_PF=%d): profile %d is not compiled in", KG_DEV_PF,
                     profile_bits(e->P)));
#endif
  {
    const int lds = (int)kMaxLds;
    hipError_t fe = hipSuccess;
#define KG_ATTR(X)                                                                                           \
  fe = hipFuncSetAttribute((const void*)resolve_round<X, false>, hipFuncAttributeMaxDynamicSharedMemorySize, lds); \
  if (fe == hipSuccess)                                                                                      \
    fe = hipFuncSetAttribute((const void*)resolve_round<X, true>, hipFuncAttributeMaxDynamicSharedMemorySize, lds); \
  if (fe == hipSuccess)                                                                                      \
    fe = hipFuncSetAttribute((const void*)resolve_mw<X, false>, hipFuncAttributeMaxDynamicSharedMemorySize, lds); \
  if (fe == hipSuccess)                                                                                      \
    fe = hipFuncSetAttribute((const void*)resolve_mw<X, true>, hipFuncAttributeMaxDynamicSharedMemorySize, lds)
    KG_PF_SWITCH(profile_bits(e->P), KG_ATTR)
#undef KG_ATTR
    if (fe != hipSuccess) return bail(fail(KG_E_DEVICE, "hipFuncSetAttribute(resolve_round LDS)"));
  }
  if (lb) {
    if (hipEventCreateWithFlags(&e->lb_ready, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&e->lb_done, hipEventDisableTiming) != hipSuccess)
      return bail(fail(KG_E_DEVICE, "hipEventCreate"));
    std::lock_guard<std::mutex> lk(lb->mu);
    e->lb = lb;
    lb->ranks[rank] = e;
    lb->ready[rank] = e->lb_ready;
    lb->done[rank] = e->lb_done;
  } else if (xfn) {
    e->xfn = xfn;
    e->xuser = xuser;
  } else if (n_ranks > 1) {
    ncclUniqueId id;
    std::memcpy(&id, nccl_id, sizeof(id));
    if (ncclCommInitRank(&e->comm, n_ranks, id, rank) != ncclSuccess) return bail(fail(KG_E_COLLECTIVE, "ncclCommInitRank"));
    // one communicator per round stream: collectives of one communicator never run concurrently
    e->comms[0] = e->comm;
    for (int k = 1; k < kMaxDepth; ++k)
      if (ncclCommSplit(e->comm, 0, rank, &e->comms[k], nullptr) != ncclSuccess)
        return bail(fail(KG_E_COLLECTIVE, "ncclCommSplit"));
  }
  // Every initialisation above is ordered on e->stream and complete before the first ingest call.  (r4) They were
  // null-stream hipMemset calls: the engine's streams are non-blocking, so nothing ordered the first ingest deltas
  // (apply_deltas on e->stream) after the table's zero fill, and on some boxes the fill landed after the NodeMetric
  // deltas — the node usage vanished from la_used (GPUTEST_r03, test_schedule_parity_round_shapes[16-4]).
  if (hipStreamSynchronize(e->stream) != hipSuccess) return bail(fail(KG_E_DEVICE, "engine initialisation"));
  *out = e;
  return 0;
}

int kg_engine_ranks(const kg_engine* e, int64_t* shard_ranks, int64_t* replica_ranks) {
  if (!e) return fail(KG_E_INVALID, "engine is NULL");
  if (shard_ranks) *shard_ranks = e->n_ranks;
  if (replica_ranks) *replica_ranks = e->replica_ranks;
  return 0;
}

int kg_engine_create(const kg_config* cfg, int64_t capacity_nodes, int rank, int n_ranks, const void* nccl_id,
                     kg_engine** out) {
  return engine_create(cfg, capacity_nodes, rank, n_ranks, nccl_id, nullptr, out);
}

int kg_loopback_create(int n_ranks, kg_loopback** out) {
  if (!out || n_ranks < 1 || n_ranks > 64) return fail(KG_E_INVALID, "n_ranks in [1, 64]");
  kg_loopback* lb = new kg_loopback();
  lb->n = n_ranks;
  lb->ranks.assign(n_ranks, nullptr);
  lb->buf.assign(n_ranks, nullptr);
  lb->ready.assign(n_ranks, nullptr);
  lb->done.assign(n_ranks, nullptr);
  *out = lb;
  return 0;
}

void kg_loopback_destroy(kg_loopback* lb) { delete lb; }

int kg_engine_create_hosted(const kg_config* cfg, int64_t capacity_nodes, int rank, int n_ranks,
                            kg_exchange_fn exchange, void* user, kg_engine** out) {
  if (!exchange) return fail(KG_E_INVALID, "exchange function is NULL");
  return engine_create(cfg, capacity_nodes, rank, n_ranks, nullptr, nullptr, out, exchange, user);
}

int kg_engine_create_loopback(const kg_config* cfg, int64_t capacity_nodes, int rank, int n_ranks, kg_loopback* lb,
                              kg_engine** out) {
  if (!lb) return fail(KG_E_INVALID, "loopback group is NULL");
  return engine_create(cfg, capacity_nodes, rank, n_ranks, nullptr, lb, out);
}

void kg_engine_destroy(kg_engine* e) {
  if (!e) return;
  if (e->lb) {
    std::lock_guard<std::mutex> lk(e->lb->mu);
    e->lb->ranks[e->rank] = nullptr;
    e->lb->ready[e->rank] = e->lb->done[e->rank] = nullptr;
  }
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  for (int k = 0; k < kMaxDepth; ++k)
    if (e->rs[k]) (void)hipStreamSynchronize(e->rs[k]);
  if (e->lb_ready) (void)hipEventDestroy(e->lb_ready);
  if (e->lb_done) (void)hipEventDestroy(e->lb_done);
  for (int k = 1; k < kMaxDepth; ++k)
    if (e->comms[k]) ncclCommDestroy(e->comms[k]);
  if (e->comm) ncclCommDestroy(e->comm);
  for (hipEvent_t ev : e->prof_pool) (void)hipEventDestroy(ev);
  e->cols64.release();
  e->paux.release();
  e->paux1.release();
  e->cols32.release();
  e->pods.release();
  e->lists.release();
  e->gathered.release();
  e->cand.release();
  e->out_keys.release();
  e->cursor.release();
  e->modlists.release();
  e->tickets.release();
  for (int k = 0; k < kMaxDepth; ++k) {
    if (e->ev_res[k]) (void)hipEventDestroy(e->ev_res[k]);
    if (e->rs[k]) (void)hipStreamDestroy(e->rs[k]);
  }
  e->deltas.release();
  e->numa_s.release();
  e->numa_m.release();
  e->npods.release();
  e->out_cpus.release();
  e->out_nrec.release();
  e->ds_d.release();
  e->dsx_d.release();
  e->quotas.release();
  e->qdev.release();
  e->dpods.release();
  e->out_minors.release();
  e->dsmax.release();
  e->dsnorm.release();
  e->dsnorm_all.release();
  e->dsval.release();
  e->rsv_d.release();
  e->rsv_g.release();
  e->rsv_nd.release();
  e->rsv_pd.release();
  e->rsel.release();
  e->rpods.release();
  e->out_rslot.release();
  e->rsv_val.release();
  if (e->rsv_exec) (void)hipGraphExecDestroy(e->rsv_exec);
  e->rsv_exec = nullptr;
  if (e->rsv_exec1) (void)hipGraphExecDestroy(e->rsv_exec1);
  e->rsv_exec1 = nullptr;
  if (e->xr_exec) (void)hipGraphExecDestroy(e->xr_exec);
  e->xr_exec = nullptr;
  e->xr_val.release();
  e->xr_val2.release();
  e->xr_aff.release();
  e->xr_part.release();
  e->xr_norm_d.release();
  e->xr_lists.release();
  e->xr_cand.release();
  e->xr_norm_all.release();
  e->xr_rec_all.release();
  e->rsv_ws.release();
  e->rsv_part.release();
  e->npred.release();
  e->defpods.release();
  e->rsv_val2.release();
  e->grp_d.release();
  e->gpods.release();
  e->logw.release();
  e->gval.release();
  e->gdelta.release();
  e->gdelta_ns.release();
  e->gz.release();
  e->gzm.release();
  e->scratch64.release();
  e->scratch32.release();
  e->uidx.release();
  if (e->stream) (void)hipStreamDestroy(e->stream);
  delete e;
}

int64_t kg_engine_num_nodes(const kg_engine* e) { return e ? e->n_nodes : 0; }

int kg_nodes_upsert(kg_engine* e, const kg_node* nodes, const int32_t* idx, int64_t n) {
  if (!e || (n > 0 && (!nodes || !idx))) return fail(KG_E_INVALID, "null argument");
  for (int64_t k = 0; k < n; ++k) {
    const int64_t i = idx[k];
    if (i < 0 || i >= e->capacity) return fail(KG_E_INVALID, "node index %lld outside capacity", (long long)i);
    for (int r = 0; r < KG_RES_MAX; ++r)
      if (nodes[k].allocatable[r] < 0 || nodes[k].allocatable[r] > (int64_t(1) << 56))
        return fail(KG_E_INVALID, "allocatable out of range");
  }
  for (int64_t k = 0; k < n; ++k) {
    const int64_t i = idx[k];
    e->nodes[i] = nodes[k];
    e->n_nodes = std::max<int64_t>(e->n_nodes, i + 1);
  }
  e->static_dirty = true;
  e->np_dirty = true;
  return 0;
}

int kg_nodes_delete(kg_engine* e, const int32_t* idx, int64_t n) {
  if (!e || (n > 0 && !idx)) return fail(KG_E_INVALID, "null argument");
  for (int64_t k = 0; k < n; ++k) {
    if (idx[k] < 0 || idx[k] >= e->capacity) return fail(KG_E_INVALID, "node index");
    e->nodes[idx[k]].flags &= ~(int64_t)KG_NODE_VALID;
  }
  e->static_dirty = true;
  e->np_dirty = true;
  return 0;
}

static int flush_placements(kg_engine* e);

int kg_node_pods_metric_set(kg_engine* e, int32_t node_idx, const kg_pod_metric* m, int64_t n) {
  if (!e || (n > 0 && !m)) return fail(KG_E_INVALID, "null argument");
  if (node_idx < 0 || node_idx >= e->capacity) return fail(KG_E_INVALID, "node index");
  if (int rc = flush_placements(e)) return rc;
  auto& v = e->pmetrics[node_idx];
  const bool was = !v.empty();
  v.clear();
  for (int64_t k = 0; k < n; ++k)
    v.push_back(kg_engine::PodMetricRec{m[k].uid, {m[k].usage[0], m[k].usage[1]}, m[k].usage_present & 3,
                                        m[k].prod ? 1 : 0});
  e->pm_nodes += (int64_t)(!v.empty()) - (int64_t)was;
  std::vector<RowDelta> d;
  la_refold(e, node_idx, d);
  return push_deltas(e, d);
}

int kg_node_metrics_update(kg_engine* e, const kg_node_metric* m, const int32_t* idx, int64_t n, int64_t now) {
  if (!e || (n > 0 && (!m || !idx))) return fail(KG_E_INVALID, "null argument");
  for (int64_t k = 0; k < n; ++k) {
    if (idx[k] < 0 || idx[k] >= e->capacity) return fail(KG_E_INVALID, "node index");
  }
  if (e->pm_nodes > 0)
    if (int rc = flush_placements(e)) return rc;
  std::vector<RowDelta> d;
  d.reserve(n);
  for (int64_t k = 0; k < n; ++k) {
    const int64_t i = idx[k];
    e->metrics[i] = m[k];
    e->now_of[i] = now;
    e->clock_metrics = std::max(e->clock_metrics, now);
    la_refold(e, i, d);
  }
  e->static_dirty = true;
  return push_deltas(e, d);
}

static int pods_delta(kg_engine* e, const kg_pod* pods, const int32_t* node_idx, int64_t n, int sign) {
  if (!e || (n > 0 && (!pods || !node_idx))) return fail(KG_E_INVALID, "null argument");
  // (r5) every pod is decoded and validated — node index, requests, group fields — before any host or device
  // state changes, so a refused call leaves the engine as it was and may be retried
  std::vector<RowDelta> d(n);
  std::vector<DevPod> dp((size_t)n);
  for (int64_t k = 0; k < n; ++k) {
    const int64_t i = node_idx[k];
    if (i < 0 || i >= e->capacity) return fail(KG_E_INVALID, "node index %lld", (long long)i);
    if (int rc = decode_pod(e, pods[k], dp[k])) return rc;
  }
  std::vector<GroupPod> hg;
  std::vector<int32_t> hn;
  bool ipa_zone = false;
  if (e->grp_on && n > 0) {
    hg.resize((size_t)n);
    hn.resize((size_t)(2 * n));
    for (int64_t k = 0; k < n; ++k) {
      if (int rc = decode_group_pod(pods[k], hg[k], k)) return rc;
      ipa_zone |= (hg[k].aff_terms_z | hg[k].anti_z | hg[k].pref_zone) != 0;
      hn[k] = (int32_t)node_idx[k];
      hn[n + k] = sign;
    }
  }
  if (sign < 0)  // a delete may name a pod this engine placed
    if (int rc = flush_placements(e)) return rc;
  for (int64_t k = 0; k < n; ++k) {
    const int64_t i = node_idx[k];
    const DevPod& p = dp[k];
    RowDelta& x = d[k];
    x.idx = i;
    x.d[0] = sign * p.req_cpu;
    x.d[1] = sign * p.req_mem;
    x.d[2] = sign * p.nz_cpu;
    x.d[3] = sign * p.nz_mem;
    x.d[4] = sign;
    const int64_t la = (pods[k].flags & KG_POD_RESERVE) ? 0 : sign;  // reserve pods: not in the assign cache
    x.d[5] = la * p.est_cpu;
    x.d[6] = la * p.est_mem;
    x.d[7] = (p.flags & P_PROD) ? la * p.est_cpu : 0;
    x.d[8] = (p.flags & P_PROD) ? la * p.est_mem : 0;
    for (int r = 0; r < kAux; ++r) x.aux[r] = sign * pods[k].requests[kAuxFirst + r];
    if (x.aux[0] != 0) e->eph_any = e->eph_dirty = true;
    if (la) {  // the podAssignCache mirror (reserve pods are not in the assign cache)
      const int64_t est[2] = {p.est_cpu, p.est_mem};
      if (sign > 0)
        mirror_assign(e, i, kg_engine::AssignedPod{pods[k].uid, pods[k].assign_time_unix_nano, {est[0], est[1]},
                                                   (p.flags & P_PROD) ? 1 : 0});
      else
        mirror_unassign(e, i, pods[k].uid, est);
    }
  }
  if (e->grp_on && n > 0) {  // the nodes' pod-group counters (NodeInfo.AddPod / RemovePod of the pods' labels / terms)
    if (ipa_zone) e->GP.ipa_zone = 1;  // sticky: zone channels on
    if (int rc = e->gdelta.ensure(n)) return rc;
    if (int rc = e->gdelta_ns.ensure(2 * n)) return rc;
    HIP_TRY(hipMemcpyAsync(e->gdelta.p, hg.data(), n * sizeof(GroupPod), hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipMemcpyAsync(e->gdelta_ns.p, hn.data(), 2 * n * 4, hipMemcpyHostToDevice, e->stream));
    group_deltas<<<(unsigned)((n + 255) / 256), 256, 0, e->stream>>>(GroupTable{e->grp_d.p, e->capacity}, e->gdelta.p,
                                                                      e->gdelta_ns.p, e->gdelta_ns.p + n, n, e->GP.hard_w);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(e->stream));
  }
  if (e->pm_nodes > 0) {  // the PodsMetric terms of the touched nodes
    std::vector<char> seen((size_t)e->capacity, 0);
    for (int64_t k = 0; k < n; ++k) {
      const int64_t i = node_idx[k];
      if (!seen[i] && !e->pmetrics[i].empty()) la_refold(e, i, d);
      seen[i] = 1;
    }
  }
  return push_deltas(e, d);
}

int kg_pods_add(kg_engine* e, const kg_pod* pods, const int32_t* node_idx, int64_t n) {
  return pods_delta(e, pods, node_idx, n, +1);
}
int kg_pods_remove(kg_engine* e, const kg_pod* pods, const int32_t* node_idx, int64_t n) {
  return pods_delta(e, pods, node_idx, n, -1);
}

int kg_pods_unreserve(kg_engine* e, int64_t first, int64_t count, const uint8_t* mask) {
  if (!e) return fail(KG_E_INVALID, "engine is NULL");
  if (first < 0 || count < 0 || first + count > e->n_staged) return fail(KG_E_INVALID, "staged range");
  std::vector<int64_t> idx;
  for (int64_t k = 0; k < count; ++k)
    if (!mask || mask[k]) idx.push_back(first + k);
  if (idx.empty()) return 0;
  if (int rc = flush_placements(e)) return rc;
  {  // podAssignCache.unAssign of the placed ones, then the PodsMetric terms of their nodes
    std::vector<uint64_t> keys((size_t)count);
    HIP_TRY(hipMemcpy(keys.data(), e->out_keys.p + first, count * 8, hipMemcpyDeviceToHost));
    std::vector<RowDelta> d;
    for (int64_t j : idx) {
      const uint64_t key = keys[j - first];
      if (!key) continue;
      const int64_t i = (int64_t)(0xFFFFFFFFu - (uint32_t)key);
      mirror_unassign(e, i, e->staged_info[j].uid, e->staged_info[j].est);
      if (!e->pmetrics[i].empty()) la_refold(e, i, d);
    }
    if (int rc = push_deltas(e, d)) return rc;
  }
  if (int rc = e->uidx.ensure(idx.size())) return rc;
  HIP_TRY(hipMemcpyAsync(e->uidx.p, idx.data(), idx.size() * 8, hipMemcpyHostToDevice, e->stream));
  unreserve_pods<<<1, 1, 0, e->stream>>>(e->T, e->pods.p, e->uidx.p, (int64_t)idx.size(), e->out_keys.p,
                                        e->numa_on ? e->numa_m.p : nullptr, e->out_cpus.p, e->out_nrec.p,
                                        e->ds_on ? e->ds_d.p : nullptr, e->dpods.p, e->out_minors.p,
                                        e->rsv_on ? e->rsv_d.p : nullptr, e->out_rslot.p, e->quotas.p, e->nq,
                                        (e->ds_on || e->rsv_on) ? e->qdev.p : nullptr, e->paux.p,
                                        GroupTable{e->grp_d.p, e->capacity}, e->grp_on ? e->gpods.p : nullptr,
                                        e->GP.hard_w, e->rsv_on && e->ds_on && e->rgpu_nodes > 0 ? e->rsv_g.p : nullptr,
                                        e->rsv_on && e->numa_on && e->rcpu_nodes > 0 ? e->rsv_c.p : nullptr,
                                        e->ds_on ? e->dsx_d.p : nullptr);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(e->stream));
  e->eph_dirty |= e->eph_any;  // a release may end an ephemeral-storage overcommit
  return 0;
}

int kg_engine_set_clock(kg_engine* e, int64_t now_unix_nano) {
  if (!e) return fail(KG_E_INVALID, "engine is NULL");
  e->clock_mode = now_unix_nano > 0 ? 1 : now_unix_nano == 0 ? 2 : 0;
  e->clock_fixed = now_unix_nano > 0 ? now_unix_nano : 0;
  return 0;
}

int kg_pods_stage(kg_engine* e, const kg_pod* pods, int64_t n) {
  if (!e || (n > 0 && !pods)) return fail(KG_E_INVALID, "null argument");
  for (int64_t k = 0; k < n; ++k) {
    if (pods[k].quota_id < 0 || pods[k].quota_id > e->nq)
      return fail(KG_E_INVALID, "pod %lld: quota_id %lld outside the quota table (%d quotas)", (long long)k,
                  (long long)pods[k].quota_id, e->nq);
  }
  std::vector<DevPod> h(std::max<int64_t>(n, 1));
  bool aux_q = false;
  for (int64_t k = 0; k < n; ++k) {
    if (int rc = decode_pod(e, pods[k], h[k])) return rc;
    aux_q |= (h[k].flags & P_AUX) != 0;
  }
  if (int rc = flush_placements(e)) return rc;  // before the staged queue is replaced
  e->aux_q = aux_q;
  e->staged_info.resize((size_t)n);
  for (int64_t k = 0; k < n; ++k)
    e->staged_info[k] = kg_engine::AssignedPod{pods[k].uid, 0, {h[k].est_cpu, h[k].est_mem}, (h[k].flags & P_PROD) ? 1 : 0};
  if (int rc = e->pods.ensure(n + kMaxB)) return rc;
  if (int rc = e->out_keys.ensure(n + kMaxB)) return rc;
  if (n > 0) HIP_TRY(hipMemcpyAsync(e->pods.p, h.data(), n * sizeof(DevPod), hipMemcpyHostToDevice, e->stream));
  {  // the kAux requests (NodeResourcesFit Filter of ephemeral-storage / scalar resources)
    std::vector<int64_t> ha((size_t)std::max<int64_t>(n, 1) * kAux, 0);
    for (int64_t k = 0; k < n; ++k)
      for (int r = 0; r < kAux; ++r) ha[(size_t)k * kAux + r] = pods[k].requests[kAuxFirst + r];
    if (int rc = e->paux.ensure((size_t)(n + kMaxB) * kAux)) return rc;
    if (n > 0) HIP_TRY(hipMemcpyAsync(e->paux.p, ha.data(), (size_t)n * kAux * 8, hipMemcpyHostToDevice, e->stream));
  }
  if (e->ds_on || e->rsv_on) {  // the pods' device requests as ElasticQuota dims (cpu, memory, 6 device resources)
    std::vector<int64_t> hq((size_t)std::max<int64_t>(n, 1) * kQuotaRes, 0);
    for (int64_t k = 0; k < n; ++k)
      for (int r = 0; r < KG_QUOTA_RES - 2; ++r) hq[(size_t)k * kQuotaRes + r] = pods[k].device_requests[r];
    if (int rc = e->qdev.ensure((size_t)(n + kMaxB) * kQuotaRes)) return rc;
    if (n > 0) HIP_TRY(hipMemcpyAsync(e->qdev.p, hq.data(), (size_t)n * kQuotaRes * 8, hipMemcpyHostToDevice, e->stream));
  }
  HIP_TRY(hipMemsetAsync(e->out_keys.p, 0, (n + kMaxB) * 8, e->stream));
  std::vector<NumaPod> hn;
  if (e->numa_on) {
    hn.resize(std::max<int64_t>(n, 1));
    for (int64_t k = 0; k < n; ++k)
      if (int rc = decode_numa_pod(e->cfg, pods[k], hn[k])) return rc;
    if (int rc = e->npods.ensure(n + kMaxB)) return rc;
    if (int rc = e->out_cpus.ensure((n + kMaxB) * kCpuWords)) return rc;
    if (n > 0) HIP_TRY(hipMemcpyAsync(e->npods.p, hn.data(), n * sizeof(NumaPod), hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipMemsetAsync(e->out_cpus.p, 0, (n + kMaxB) * kCpuWords * 8, e->stream));
    if (int rc = e->out_nrec.ensure((n + kMaxB) * kNumaRecWords)) return rc;
    HIP_TRY(hipMemsetAsync(e->out_nrec.p, 0, (n + kMaxB) * kNumaRecWords * 8, e->stream));
  }
  std::vector<DsPod> hd;
  e->dsx_q = false;
  if (e->ds_on) {
    hd.resize(std::max<int64_t>(n, 1));
    for (int64_t k = 0; k < n; ++k) {
      if (int rc = decode_ds_pod(pods[k], hd[k])) return rc;
      e->dsx_q |= (hd[k].xq[0] | hd[k].xq[1]) != 0;  // (ABI 17) RDMA / FPGA pods take the per-pod pass
    }
    if (int rc = e->dpods.ensure(n + kMaxB)) return rc;
    if (int rc = e->out_minors.ensure(n + kMaxB)) return rc;
    if (n > 0) HIP_TRY(hipMemcpyAsync(e->dpods.p, hd.data(), n * sizeof(DsPod), hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipMemsetAsync(e->out_minors.p, 0, (n + kMaxB) * 4, e->stream));
  } else {
    for (int64_t k = 0; k < n; ++k)
      for (int r = 0; r < KG_DEV_RES_MAX; ++r)
        if (pods[k].device_requests[r] != 0 && e->cfg.fit_filter)
          return fail(KG_E_UNSUPPORTED, "pod %lld requests devices; the profile has no DeviceShare (NodeResourcesFit on "
                      "device resources is not accelerated)", (long long)k);
  }
  if (e->def_on) {  // TaintToleration / NodeAffinity view of the pods
    std::vector<DefPod> hf(std::max<int64_t>(n, 1));
    for (int64_t k = 0; k < n; ++k)
      if (int rc = decode_def_pod(pods[k], hf[k], k)) return rc;
    int64_t tmin = 64, ptop = 0, itop = 0;  // what the queue was compiled against (ABI 11)
    for (int64_t k = 0; k < n; ++k) {
      const kg_pod& q = pods[k];
      if (q.flags & KG_POD_TAINT_TABLE) {
        if (q.taint_count < 0 || q.taint_count > 64) return fail(KG_E_INVALID, "pod %lld: taint_count", (long long)k);
        tmin = std::min<int64_t>(tmin, q.taint_count);
      }
      uint64_t used = q.node_selector;
      for (int t = 0; t < KG_MAX_AFF_TERMS; ++t) {
        if (t < q.n_required_terms) used |= q.required_terms[t];
        if (t < q.n_preferred_terms) used |= q.preferred_terms[t];
      }
      ptop = std::max<int64_t>(ptop, used ? 64 - __builtin_clzll(used) : 0);
      for (int c = 0; c < KG_MAX_CONTAINERS && c < q.n_containers; ++c)
        itop = std::max<int64_t>(itop, q.container_image_bit[c] + 1);
    }
    e->sq_taint_min = tmin;
    e->sq_pred_top = ptop;
    e->sq_img_top = itop;
    if (int rc = e->defpods.ensure(n + kMaxB)) return rc;
    if (n > 0) HIP_TRY(hipMemcpyAsync(e->defpods.p, hf.data(), n * sizeof(DefPod), hipMemcpyHostToDevice, e->stream));
  }
  if (e->grp_on) {  // PodTopologySpread / InterPodAffinity view of the pods
    std::vector<GroupPod> hg(std::max<int64_t>(n, 1));
    for (int64_t k = 0; k < n; ++k) {
      if (int rc = decode_group_pod(pods[k], hg[k], k)) return rc;
      if (hg[k].aff_terms_z | hg[k].anti_z | hg[k].pref_zone) e->GP.ipa_zone = 1;  // sticky: zone channels on
    }
    if (int rc = e->gpods.ensure(n + kMaxB)) return rc;
    if (n > 0) HIP_TRY(hipMemcpyAsync(e->gpods.p, hg.data(), n * sizeof(GroupPod), hipMemcpyHostToDevice, e->stream));
  }
  {  // exact-pass records (the Reservation view of every pod; single-pod calls of any profile use the pass)
    std::vector<RsvPod> hr(std::max<int64_t>(n, 1));
    std::vector<RsvSel> hs(std::max<int64_t>(n, 1));
    int64_t rtop = 0;
    bool ext = false;
    for (int64_t k = 0; k < n; ++k) {
      if (int rc = decode_rsv_pod(pods[k], hr[k], hs[k], k)) return rc;
      if (hr[k].flags & RP_SEL) hr[k].aux = (int32_t)k;
      ext |= (hr[k].flags & (RP_RESERVE | RP_OPERATING | RP_SEL)) != 0;
      rtop = std::max<int64_t>(rtop, rsv_pred_top(hr[k], hs[k]));
      // (r5) reserve pods in NodeNUMAResource / DeviceShare profiles: matched to no reservation and never nominated,
      // they take both plugins' plain paths (nodenumaresource/plugin.go:515, deviceshare/reservation.go:301, :342)
    }
    e->sq_rsv_top = rtop;
    e->rsv_ext_q = ext;
    if (int rc = e->rpods.ensure(n + kMaxB)) return rc;
    if (int rc = e->out_rslot.ensure(n + kMaxB)) return rc;
    if (n > 0) HIP_TRY(hipMemcpyAsync(e->rpods.p, hr.data(), n * sizeof(RsvPod), hipMemcpyHostToDevice, e->stream));
    if (int rc = e->rsel.ensure(n + kMaxB)) return rc;
    if (n > 0) HIP_TRY(hipMemcpyAsync(e->rsel.p, hs.data(), n * sizeof(RsvSel), hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipMemsetAsync(e->out_rslot.p, 0xff, (n + kMaxB) * 4, e->stream));
  }
  HIP_TRY(hipStreamSynchronize(e->stream));
  e->n_staged = n;
  return 0;
}

static int schedule_staged_impl(kg_engine* e, int64_t first, int64_t count, kg_stats* stats);
// the placed pods enter the podAssignCache mirror (LoadAware Reserve → assign, timestamp = the engine clock; a pod
// placed under the default clock, the newest NodeMetric update, is taken as assigned just after it)
// Reserve → podAssignCache.assign (load_aware.go:260-263) of the pods a schedule call placed.  The mirror only
// feeds the PodsMetric terms, so the placed ranges are recorded and read back lazily: right away when some node
// reports PodsMetric, otherwise before the next call that reads or rewrites the mirror or the staged queue.
static int flush_placements(kg_engine* e) {
  std::vector<uint64_t> keys;
  for (const auto& r : e->pending_place) {
    keys.resize((size_t)r.count);
    HIP_TRY(hipMemcpy(keys.data(), e->out_keys.p + r.first, r.count * 8, hipMemcpyDeviceToHost));
    for (int64_t k = 0; k < r.count; ++k) {
      if (!keys[k]) continue;
      kg_engine::AssignedPod a = e->staged_info[r.first + k];
      a.time = r.time;
      mirror_assign(e, (int64_t)(0xFFFFFFFFu - (uint32_t)keys[k]), a);
    }
  }
  e->pending_place.clear();
  return 0;
}
int kg_pods_schedule_staged(kg_engine* e, int64_t first, int64_t count, kg_stats* stats) {
  if (int rc = schedule_staged_impl(e, first, count, stats)) return rc;
  if (count == 0) return 0;
  // the assign time: after this call's clock (clock mode 0 keeps the newest metric time, so +1 ns = after it)
  e->pending_place.push_back({first, count, e->clock_now + (e->clock_mode == 0 ? 1 : 0)});
  return e->pm_nodes > 0 ? flush_placements(e) : 0;
}
// (ABI 11) the caller's taint / predicate / image tables only grow; rows compiled before an id existed leave it
// undecided, so a schedule call is refused when the staged queue and the valid node rows disagree on what was compiled
static int check_predicate_tables(kg_engine* e) {
  if (!e->def_on) return 0;
  if (e->np_dirty) {
    int64_t tt = 0, pc = 64, ic = 64;
    for (int64_t i = 0; i < e->n_nodes; ++i) {
      if (!(e->nodes[i].flags & KG_NODE_VALID)) continue;
      tt = std::max<int64_t>(tt, e->np_taint_top[i]);
      pc = std::min<int64_t>(pc, e->np_pred_cnt[i]);
      ic = std::min<int64_t>(ic, e->np_img_cnt[i]);
    }
    e->np_taint_top_max = tt, e->np_pred_cnt_min = pc, e->np_img_cnt_min = ic;
    e->np_dirty = false;
  }
  if (e->np_taint_top_max > e->sq_taint_min)
    return fail(KG_E_INVALID, "TaintToleration: a node row carries taint %lld but a staged pod's tolerations were compiled "
                "against %lld taints: re-stage the pods", (long long)e->np_taint_top_max - 1, (long long)e->sq_taint_min);
  if (e->sq_pred_top > e->np_pred_cnt_min)
    return fail(KG_E_INVALID, "NodeAffinity: the staged pods use predicate %lld but a node row was compiled against %lld "
                "predicates: re-send the node rows", (long long)e->sq_pred_top - 1, (long long)e->np_pred_cnt_min);
  if (e->sq_img_top > e->np_img_cnt_min)
    return fail(KG_E_INVALID, "ImageLocality: the staged pods use image %lld but a node row was compiled against %lld "
                "images: re-send the node rows", (long long)e->sq_img_top - 1, (long long)e->np_img_cnt_min);
  return 0;
}

// one pod (the preemption dry run's) against the node rows' tables, as check_predicate_tables does for a staged queue
static int check_pod_tables(kg_engine* e, const kg_pod& q) {
  const int64_t st = e->sq_taint_min, sp = e->sq_pred_top, si = e->sq_img_top;
  int64_t tmin = 64, ptop = 0, itop = 0;
  if (q.flags & KG_POD_TAINT_TABLE) {
    if (q.taint_count < 0 || q.taint_count > 64) return fail(KG_E_INVALID, "pod: taint_count");
    tmin = q.taint_count;
  }
  uint64_t used = q.node_selector;
  for (int t = 0; t < KG_MAX_AFF_TERMS; ++t) {
    if (t < q.n_required_terms) used |= q.required_terms[t];
    if (t < q.n_preferred_terms) used |= q.preferred_terms[t];
  }
  ptop = used ? 64 - __builtin_clzll(used) : 0;
  for (int c = 0; c < KG_MAX_CONTAINERS && c < q.n_containers; ++c) itop = std::max<int64_t>(itop, q.container_image_bit[c] + 1);
  e->sq_taint_min = tmin, e->sq_pred_top = ptop, e->sq_img_top = itop;
  const int rc = check_predicate_tables(e);
  e->sq_taint_min = st, e->sq_pred_top = sp, e->sq_img_top = si;
  return rc;
}

// (ABI 12) the same rule for the reservation slots' fakeNode predicates (kg_node_reservations.predicate_count)
static int check_rsv_predicates(kg_engine* e, int64_t top) {
  if (top == 0) return 0;
  if (e->rsv_pdirty) {
    int64_t pc = 64;
    for (int64_t i = 0; i < std::min<int64_t>(e->n_nodes, (int64_t)e->rsv_pcnt.size()); ++i)
      pc = std::min<int64_t>(pc, e->rsv_pcnt[i]);
    e->rsv_pcnt_min = pc;
    e->rsv_pdirty = false;
  }
  if (top > e->rsv_pcnt_min)
    return fail(KG_E_INVALID, "Reservation affinity: a pod uses predicate %lld but reservation slots were compiled "
                "against %lld predicates: re-send the reservations", (long long)top - 1, (long long)e->rsv_pcnt_min);
  return 0;
}

static int schedule_staged_impl(kg_engine* e, int64_t first, int64_t count, kg_stats* stats) {
  if (!e) return fail(KG_E_INVALID, "engine is NULL");
  if (first < 0 || count < 0 || first + count > e->n_staged) return fail(KG_E_INVALID, "staged range");
  if (count > 0)
    if (int rc = check_predicate_tables(e)) return rc;
  if (count > 0)
    if (int rc = check_rsv_predicates(e, e->sq_rsv_top)) return rc;
  const double t0 = now_s();
  // the exact per-pod pass: its profiles, and calls of at most kExactSmall pods of any profile (the drop-in's per-pod
  // scheduleOne): one pass costs less than a round's eval + merge + resolve when a round would hold one pod
  // (PodTopologySpread / InterPodAffinity profiles: one pod per pass — the batched rounds' stop rules do not cover
  // their cluster-wide minimum / count and min-max normalisation)
  // (ABI 13) GPU-holding reservations: the per-pod pass (the batched rounds keep no DeviceShare restore)
  // (ABI 15) reservations holding cpusets: the per-pod pass too (the batched rounds compile the preferred-cpu path out)
  // (ABI 17) RDMA / FPGA requests: the per-pod pass (the batched rounds and the round engine carry the GPU type only)
  if (e->dsx_q && count > 0) {
    if (e->rsv_on && e->rgpu_nodes > 0)
      return fail(KG_E_UNSUPPORTED, "RDMA / FPGA requests with reservations that hold GPUs keep the Go path");
    if (!e->exact_on && e->n_ranks > 1)
      return fail(KG_E_UNSUPPORTED, "RDMA / FPGA requests on a multi-rank round-engine profile keep the Go path");
  }
  if (e->exact_on && e->xr_on && !e->grp_on && !e->rsv_ext_q && !e->dsx_q && e->rgpu_nodes == 0 &&
      e->rcpu_nodes == 0 && count >= kXrMin && e->n_nodes > 0)
    return run_xr(e, first, count, stats, t0);
  if (e->exact_on || e->dsx_q || (count <= kExactSmall && e->n_ranks == 1)) return run_rsv(e, first, count, stats, t0);
  RoundGeom g;
  if (int rc = prepare_rounds(e, g)) return rc;
  const int64_t end = first + count;
  const int64_t init[16] = {first};
  int64_t host_stats[16] = {first};
  HIP_TRY(hipMemcpyAsync(e->cursor.p, init, 16 * 8, hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  int64_t cur = first;
  while (cur < end) {
    // a round that stops early poisons the rest of its batch; the next batch restarts from the device cursor
    // (DeviceShare rounds read the cursor themselves: an early stop only shortens that round).  The batch launches
    // at most rounds_ahead rounds: halved towards the rounds that ran before a stop when rounds stop early (small
    // clusters), doubled back when a batch completes, so a stop wastes few poisoned launches.
    const int64_t n_rounds = std::min<int64_t>({(end - cur + g.B - 1) / g.B, kMaxBatchRounds, e->rounds_ahead});
    const int64_t ran0 = host_stats[1];
    if (int rc = e->ds_on ? run_batch_ds(e, g, end, n_rounds) : run_batch(e, g, cur, end, n_rounds)) return rc;
    HIP_TRY(hipMemcpy(host_stats, e->cursor.p, 16 * 8, hipMemcpyDeviceToHost));
    if (host_stats[5]) return fail(KG_E_DEVICE, "resolver chain wait timed out (round sequence %lld)", (long long)host_stats[4]);
    const bool stopped = host_stats[0] < std::min<int64_t>(end, cur + n_rounds * g.B);
    const int64_t ran = host_stats[1] - ran0;
    if (!e->ds_on)  // DeviceShare rounds are cursor-driven: a stop never poisons the rest of the batch
      e->rounds_ahead = stopped ? std::max<int64_t>(2, std::min<int64_t>(e->rounds_ahead, 2 * ran))
                                : std::min<int64_t>(kMaxBatchRounds, 2 * e->rounds_ahead);
    cur = host_stats[0];
  }
  if (stats) {
    std::memset(stats, 0, sizeof(*stats));
    stats->device_batches = host_stats[1];
    stats->reserved[0] = (double)host_stats[6];  // diagnostics: slow-path pods, speculation steps (resolve_round)
    stats->reserved[1] = (double)host_stats[7];
    stats->reserved[2] = (double)host_stats[8] * 1e-8;  // resolvers' active time (s_memrealtime, 100 MHz): after the
                                                         // chain wait to the publish, summed over the call's rounds
    stats->node_evaluations = count * g.N;
    stats->seconds = now_s() - t0;
  }
  return 0;
}

int kg_results_fetch(kg_engine* e, int64_t first, int64_t count, int32_t* out_node, int64_t* out_score) {
  if (!e) return fail(KG_E_INVALID, "engine is NULL");
  if (first < 0 || count < 0 || first + count > e->n_staged) return fail(KG_E_INVALID, "staged range");
  std::vector<uint64_t> keys(std::max<int64_t>(count, 1));
  if (count > 0) {
    HIP_TRY(hipMemcpyAsync(keys.data(), e->out_keys.p + first, count * 8, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
  }
  for (int64_t i = 0; i < count; ++i) {
    const uint64_t k = keys[i];
    if (out_node) out_node[i] = k ? (int32_t)(0xFFFFFFFFu - (uint32_t)k) : -1;
    if (out_score) out_score[i] = k ? (int64_t)(k >> 32) : 0;
  }
  return 0;
}

int kg_pods_schedule(kg_engine* e, const kg_pod* pods, int64_t n, int32_t* out_node, int64_t* out_score,
                     kg_stats* stats) {
  const double t0 = now_s();
  if (int rc = kg_pods_stage(e, pods, n)) return rc;
  if (int rc = kg_pods_schedule_staged(e, 0, n, stats)) return rc;
  if (int rc = kg_results_fetch(e, 0, n, out_node, out_score)) return rc;
  if (stats) {
    stats->seconds = now_s() - t0;
    for (int64_t i = 0; i < n; ++i) (out_node && out_node[i] >= 0) ? ++stats->pods_scheduled : ++stats->pods_unschedulable;
  }
  return 0;
}

int kg_pods_evaluate(kg_engine* e, const kg_pod* pod, int32_t* out_reject, int64_t* out_fit, int64_t* out_la) {
  if (!e || !pod) return fail(KG_E_INVALID, "null argument");
  if (int rc = sync_static(e)) return rc;
  DevPod d;
  if (int rc = decode_pod(e, *pod, d)) return rc;
  const int64_t n = e->n_nodes;
  if (n == 0) return 0;
  if (int rc = e->scratch64.ensure(2 * n + kPodWords)) return rc;
  if (int rc = e->scratch32.ensure(n)) return rc;
  DevPod* dp = reinterpret_cast<DevPod*>(e->scratch64.p + 2 * n);  // the kPodWords spare int64s
  HIP_TRY(hipMemcpyAsync(dp, &d, sizeof(d), hipMemcpyHostToDevice, e->stream));
  if (int rc = e->paux1.ensure(kAux)) return rc;
  HIP_TRY(hipMemcpyAsync(e->paux1.p, &pod->requests[kAuxFirst], kAux * 8, hipMemcpyHostToDevice, e->stream));
  evaluate_pod<<<(unsigned)((n + 255) / 256), 256, 0, e->stream>>>(e->T, dp, n, e->P, e->scratch32.p, e->scratch64.p,
                                                                   e->scratch64.p + n, e->paux1.p);
  HIP_TRY(hipGetLastError());
  std::vector<int32_t> rej(n);
  std::vector<int64_t> fs(n), ls(n);
  HIP_TRY(hipMemcpyAsync(rej.data(), e->scratch32.p, n * 4, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipMemcpyAsync(fs.data(), e->scratch64.p, n * 8, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipMemcpyAsync(ls.data(), e->scratch64.p + n, n * 8, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  // reject bits are only reported for enabled Filter plugins (eval_node checks P.*_filter)
  if (out_reject) std::memcpy(out_reject, rej.data(), n * 4);
  if (out_fit) std::memcpy(out_fit, fs.data(), n * 8);
  if (out_la) std::memcpy(out_la, ls.data(), n * 8);
  return 0;
}

int kg_nodes_read_state(kg_engine* e, int64_t* req_cpu, int64_t* req_mem, int64_t* nz_cpu, int64_t* nz_mem,
                        int64_t* num_pods, int64_t* la_est_cpu, int64_t* la_est_mem, int64_t* la_pcpu,
                        int64_t* la_pmem) {
  if (!e) return fail(KG_E_INVALID, "engine is NULL");
  const int64_t n = e->n_nodes;
  if (n == 0) return 0;
  auto get64 = [&](int64_t* dst, const int64_t* src) -> int {
    if (dst) HIP_TRY(hipMemcpyAsync(dst, src, n * 8, hipMemcpyDeviceToHost, e->stream));
    return 0;
  };
  if (int rc = get64(req_cpu, e->T.req_cpu)) return rc;
  if (int rc = get64(req_mem, e->T.req_mem)) return rc;
  if (int rc = get64(nz_cpu, e->T.nz_cpu)) return rc;
  if (int rc = get64(nz_mem, e->T.nz_mem)) return rc;
  if (int rc = get64(la_est_cpu, e->T.la_used_cpu)) return rc;
  if (int rc = get64(la_est_mem, e->T.la_used_mem)) return rc;
  if (int rc = get64(la_pcpu, e->T.la_pused_cpu)) return rc;
  if (int rc = get64(la_pmem, e->T.la_pused_mem)) return rc;
  std::vector<int32_t> np(n);
  HIP_TRY(hipMemcpyAsync(np.data(), e->T.num_pods, n * 4, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  if (num_pods)
    for (int64_t i = 0; i < n; ++i) num_pods[i] = np[i];
  // la_used folds NodeUsage in; report Σ estimates only
  for (int64_t i = 0; i < n; ++i) {
    if (la_est_cpu) la_est_cpu[i] -= e->folded_usage[2 * i];
    if (la_est_mem) la_est_mem[i] -= e->folded_usage[2 * i + 1];
    if (la_pcpu) la_pcpu[i] -= e->folded_prod[2 * i];
    if (la_pmem) la_pmem[i] -= e->folded_prod[2 * i + 1];
  }
  return 0;
}

int kg_nodes_numa_upsert(kg_engine* e, const kg_node_numa* numa, const int32_t* idx, int64_t n) {
  if (!e || (n > 0 && (!numa || !idx))) return fail(KG_E_INVALID, "null argument");
  if (!e->numa_on) return fail(KG_E_INVALID, "the profile does not enable NodeNUMAResource");
  if (n == 0) return 0;
  std::vector<NumaStatic> hs(n);
  std::vector<NumaMut> hm(n);
  for (int64_t k = 0; k < n; ++k) {
    if (idx[k] < 0 || idx[k] >= e->capacity) return fail(KG_E_INVALID, "node index %d outside capacity", idx[k]);
    if (int rc = decode_node_numa(numa[k], hs[k], hm[k])) return rc;
  }
  DevBuf<uint8_t> b;
  const size_t bytes = n * (sizeof(NumaStatic) + sizeof(NumaMut) + 4);
  if (int rc = b.ensure(bytes)) return rc;
  NumaStatic* ds = reinterpret_cast<NumaStatic*>(b.p);
  NumaMut* dm = reinterpret_cast<NumaMut*>(b.p + n * sizeof(NumaStatic));
  int32_t* di = reinterpret_cast<int32_t*>(b.p + n * (sizeof(NumaStatic) + sizeof(NumaMut)));
  HIP_TRY(hipMemcpyAsync(ds, hs.data(), n * sizeof(NumaStatic), hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipMemcpyAsync(dm, hm.data(), n * sizeof(NumaMut), hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipMemcpyAsync(di, idx, n * 4, hipMemcpyHostToDevice, e->stream));
  scatter_numa<<<(unsigned)((n + 255) / 256), 256, 0, e->stream>>>(numa_table(e), ds, dm, di, n);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(e->stream));
  b.release();
  return 0;
}

int kg_nodes_read_numa(kg_engine* e, uint64_t* allocated_cpus, int64_t* numa_alloc_cpu, int64_t* numa_alloc_mem) {
  if (!e) return fail(KG_E_INVALID, "engine is NULL");
  if (!e->numa_on) return fail(KG_E_INVALID, "the profile does not enable NodeNUMAResource");
  const int64_t n = e->n_nodes;
  if (n == 0) return 0;
  std::vector<NumaMut> hm(n);
  HIP_TRY(hipMemcpyAsync(hm.data(), e->numa_m.p, n * sizeof(NumaMut), hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  for (int64_t i = 0; i < n; ++i)
    for (int k = 0; k < 4; ++k) {
      if (allocated_cpus) allocated_cpus[i * 4 + k] = hm[i].allocated[k];
      if (numa_alloc_cpu) numa_alloc_cpu[i * 4 + k] = hm[i].alloc_cpu[k];
      if (numa_alloc_mem) numa_alloc_mem[i * 4 + k] = hm[i].alloc_mem[k];
    }
  return 0;
}

int kg_results_fetch_cpusets(kg_engine* e, int64_t first, int64_t count, uint64_t* out_cpusets) {
  if (!e || (count > 0 && !out_cpusets)) return fail(KG_E_INVALID, "null argument");
  if (first < 0 || count < 0 || first + count > e->n_staged) return fail(KG_E_INVALID, "staged range");
  if (!e->numa_on) {
    std::memset(out_cpusets, 0, (size_t)count * kCpuWords * 8);
    return 0;
  }
  if (count > 0) {
    HIP_TRY(hipMemcpyAsync(out_cpusets, e->out_cpus.p + first * kCpuWords, count * kCpuWords * 8, hipMemcpyDeviceToHost,
                           e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
  }
  return 0;
}

int kg_pods_evaluate_numa(kg_engine* e, const kg_pod* pod, int32_t* out_pass, int64_t* out_score,
                          int64_t* out_affinity) {
  if (!e || !pod) return fail(KG_E_INVALID, "null argument");
  if (!e->numa_on) return fail(KG_E_INVALID, "the profile does not enable NodeNUMAResource");
  if (int rc = sync_static(e)) return rc;
  DevPod d;
  NumaPod np;
  if (int rc = decode_pod(e, *pod, d)) return rc;
  if (int rc = decode_numa_pod(e->cfg, *pod, np)) return rc;
  const int64_t n = e->n_nodes;
  if (n == 0) return 0;
  if (int rc = e->scratch64.ensure(2 * n + kPodWords + kNumaPodWords)) return rc;
  if (int rc = e->scratch32.ensure(n)) return rc;
  DevPod* dp = reinterpret_cast<DevPod*>(e->scratch64.p + 2 * n);
  NumaPod* dn = reinterpret_cast<NumaPod*>(e->scratch64.p + 2 * n + kPodWords);
  HIP_TRY(hipMemcpyAsync(dp, &d, sizeof(d), hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipMemcpyAsync(dn, &np, sizeof(np), hipMemcpyHostToDevice, e->stream));
  evaluate_pod_numa<<<(unsigned)((n + 255) / 256), 256, 0, e->stream>>>(e->T, numa_table(e), dp, dn, n, e->NP,
                                                                        e->scratch32.p, e->scratch64.p,
                                                                        e->scratch64.p + n);
  HIP_TRY(hipGetLastError());
  std::vector<int32_t> ps(n);
  std::vector<int64_t> sc(n), af(n);
  HIP_TRY(hipMemcpyAsync(ps.data(), e->scratch32.p, n * 4, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipMemcpyAsync(sc.data(), e->scratch64.p, n * 8, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipMemcpyAsync(af.data(), e->scratch64.p + n, n * 8, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  if (out_pass) std::memcpy(out_pass, ps.data(), n * 4);
  if (out_score) std::memcpy(out_score, sc.data(), n * 8);
  if (out_affinity) std::memcpy(out_affinity, af.data(), n * 8);
  return 0;
}

int kg_nodes_device_upsert(kg_engine* e, const kg_node_device* dev, const int32_t* idx, int64_t n) {
  if (!e || (n > 0 && (!dev || !idx))) return fail(KG_E_INVALID, "null argument");
  if (!e->ds_on) return fail(KG_E_INVALID, "the profile does not enable DeviceShare");
  if (n == 0) return 0;
  std::vector<DsNode> h(n);
  std::vector<DsXNode> hx(n);
  for (int64_t k = 0; k < n; ++k) {
    if (idx[k] < 0 || idx[k] >= e->capacity) return fail(KG_E_INVALID, "node index %d outside capacity", idx[k]);
    if (int rc = decode_node_device(dev[k], h[k], hx[k])) return rc;
  }
  DevBuf<uint8_t> b;
  if (int rc = b.ensure(n * (sizeof(DsNode) + sizeof(DsXNode) + 4))) return rc;
  DsNode* dd = reinterpret_cast<DsNode*>(b.p);
  DsXNode* dx = reinterpret_cast<DsXNode*>(b.p + n * sizeof(DsNode));
  int32_t* di = reinterpret_cast<int32_t*>(b.p + n * (sizeof(DsNode) + sizeof(DsXNode)));
  HIP_TRY(hipMemcpyAsync(dd, h.data(), n * sizeof(DsNode), hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipMemcpyAsync(dx, hx.data(), n * sizeof(DsXNode), hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipMemcpyAsync(di, idx, n * 4, hipMemcpyHostToDevice, e->stream));
  scatter_ds<<<(unsigned)((n + 255) / 256), 256, 0, e->stream>>>(DsTable{e->ds_d.p}, dd, di, n);
  HIP_TRY(hipGetLastError());
  scatter_dsx<<<(unsigned)((n + 255) / 256), 256, 0, e->stream>>>(e->dsx_d.p, dx, di, n);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(e->stream));
  b.release();
  return 0;
}

int kg_nodes_read_device(kg_engine* e, int64_t* used_core, int64_t* used_memory, int64_t* used_ratio) {
  if (!e) return fail(KG_E_INVALID, "engine is NULL");
  if (!e->ds_on) return fail(KG_E_INVALID, "the profile does not enable DeviceShare");
  const int64_t n = e->n_nodes;
  if (n == 0) return 0;
  std::vector<DsNode> h(n);
  HIP_TRY(hipMemcpyAsync(h.data(), e->ds_d.p, n * sizeof(DsNode), hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  for (int64_t i = 0; i < n; ++i)
    for (int m = 0; m < KG_MAX_MINORS; ++m) {
      if (used_core) used_core[i * KG_MAX_MINORS + m] = h[i].ucore[m];
      if (used_memory) used_memory[i * KG_MAX_MINORS + m] = h[i].umem[m];
      if (used_ratio) used_ratio[i * KG_MAX_MINORS + m] = h[i].uratio[m];
    }
  return 0;
}

int kg_results_fetch_devices(kg_engine* e, int64_t first, int64_t count, int32_t* out_minor_mask) {
  if (!e || (count > 0 && !out_minor_mask)) return fail(KG_E_INVALID, "null argument");
  if (first < 0 || count < 0 || first + count > e->n_staged) return fail(KG_E_INVALID, "staged range");
  if (!e->ds_on) {
    std::memset(out_minor_mask, 0, (size_t)count * 4);
    return 0;
  }
  if (count > 0) {
    HIP_TRY(hipMemcpyAsync(out_minor_mask, e->out_minors.p + first, count * 4, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    for (int64_t k = 0; k < count; ++k) out_minor_mask[k] &= 0xFF;  // the GPU byte of the packed record
  }
  return 0;
}

int kg_results_fetch_devices_x(kg_engine* e, int64_t first, int64_t count, int32_t* out) {
  if (!e || (count > 0 && !out)) return fail(KG_E_INVALID, "null argument");
  if (first < 0 || count < 0 || first + count > e->n_staged) return fail(KG_E_INVALID, "staged range");
  if (!e->ds_on) {
    std::memset(out, 0, (size_t)count * kXTypes * 4);
    return 0;
  }
  if (count > 0) {
    std::vector<int32_t> h((size_t)count);
    HIP_TRY(hipMemcpyAsync(h.data(), e->out_minors.p + first, count * 4, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    for (int64_t k = 0; k < count; ++k)
      for (int t = 0; t < kXTypes; ++t) out[k * kXTypes + t] = ((uint32_t)h[k] >> (8 * (t + 1))) & 0xFFu;
  }
  return 0;
}

int kg_nodes_read_device_x(kg_engine* e, int64_t* x_used) {
  if (!e || !x_used) return fail(KG_E_INVALID, "null argument");
  if (!e->ds_on) return fail(KG_E_INVALID, "the profile does not enable DeviceShare");
  const int64_t n = e->n_nodes;
  if (n == 0) return 0;
  std::vector<DsXNode> h(n);
  HIP_TRY(hipMemcpyAsync(h.data(), e->dsx_d.p, n * sizeof(DsXNode), hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  for (int64_t i = 0; i < n; ++i)
    for (int t = 0; t < kXTypes; ++t)
      for (int m = 0; m < KG_MAX_MINORS; ++m) x_used[(i * kXTypes + t) * KG_MAX_MINORS + m] = h[i].u[t][m];
  return 0;
}

int kg_pods_evaluate_device(kg_engine* e, const kg_pod* pod, int32_t* out_pass, int64_t* out_score) {
  if (!e || !pod) return fail(KG_E_INVALID, "null argument");
  if (!e->ds_on) return fail(KG_E_INVALID, "the profile does not enable DeviceShare");
  DsPod dp;
  if (int rc = decode_ds_pod(*pod, dp)) return rc;
  const int64_t n = e->n_nodes;
  if (n == 0) return 0;
  if (int rc = e->scratch64.ensure(n + kDsPodWords)) return rc;
  if (int rc = e->scratch32.ensure(n)) return rc;
  DsPod* d = reinterpret_cast<DsPod*>(e->scratch64.p + n);
  HIP_TRY(hipMemcpyAsync(d, &dp, sizeof(dp), hipMemcpyHostToDevice, e->stream));
  evaluate_pod_ds<<<(unsigned)((n + 255) / 256), 256, 0, e->stream>>>(DsTable{e->ds_d.p}, d, n, e->DP, e->scratch32.p,
                                                                      e->scratch64.p, e->dsx_d.p);
  HIP_TRY(hipGetLastError());
  std::vector<int32_t> ps(n);
  std::vector<int64_t> sc(n);
  HIP_TRY(hipMemcpyAsync(ps.data(), e->scratch32.p, n * 4, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipMemcpyAsync(sc.data(), e->scratch64.p, n * 8, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  if (out_pass) std::memcpy(out_pass, ps.data(), n * 4);
  if (out_score) std::memcpy(out_score, sc.data(), n * 8);
  return 0;
}

int kg_quotas_set(kg_engine* e, const kg_quota* quotas, int64_t n) {
  if (!e || (n > 0 && !quotas)) return fail(KG_E_INVALID, "null argument");
  if (n < 0 || n > KG_MAX_QUOTAS) return fail(KG_E_UNSUPPORTED, "%lld quotas > %d", (long long)n, KG_MAX_QUOTAS);
  static_assert(sizeof(kg_quota) == sizeof(QuotaRow), "kg_quota is the device row");
  for (int64_t k = 0; k < n; ++k) {
    const kg_quota& q = quotas[k];
    for (int r = 0; r < KG_QUOTA_RES; ++r)
      if (q.used[r] < 0 || q.non_preemptible_used[r] < 0 || q.used_limit[r] < -1 || q.min[r] < -1 ||
          q.used[r] > (1ll << 60) || q.used_limit[r] > (1ll << 60) || q.min[r] > (1ll << 60) ||
          q.non_preemptible_used[r] > (1ll << 60))
        return fail(KG_E_INVALID, "quota %lld: quantity out of range", (long long)k);
  }
  if (int rc = e->quotas.ensure(KG_MAX_QUOTAS)) return rc;
  if (n > 0) {
    HIP_TRY(hipMemcpyAsync(e->quotas.p, quotas, n * sizeof(QuotaRow), hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
  }
  e->nq = (int)n;
  return 0;
}

int kg_quotas_read(kg_engine* e, kg_quota* out, int64_t n) {
  if (!e || (n > 0 && !out)) return fail(KG_E_INVALID, "null argument");
  if (n != e->nq) return fail(KG_E_INVALID, "the quota table holds %d quotas", e->nq);
  if (n == 0) return 0;
  HIP_TRY(hipMemcpyAsync(out, e->quotas.p, n * sizeof(QuotaRow), hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return 0;
}

// Reservation profile: which 0 = rsv_eval, 1 = rsv_select, replayed on the first staged pod (neither kernel
// changes node state; the cursor words are reset afterwards).  Algorithmic bytes of rsv_eval per launch: SURVEY
// §8d's 76 B of Fit + LoadAware columns per node, the 4-B slot count and the 8-B packed value written, plus the
// 192-B slot record of every node that has reservations; rsv_select reads the 8-B packed value per node.
static int bench_rsv(kg_engine* e, int which, int iters, double* avg_ms, double* algo_bytes) {
  if (iters <= 0 || which < 0 || which > 1) return fail(KG_E_INVALID, "bad argument");
  if (e->n_staged <= 0) return fail(KG_E_INVALID, "stage a pod queue first");
  if (int rc = sync_static(e)) return rc;
  const int64_t n = e->n_nodes;
  if (n <= 0) return fail(KG_E_INVALID, "no nodes");
  std::vector<int32_t> hn(n);
  HIP_TRY(hipMemcpy(hn.data(), e->rsv_nd.p, n * 4, hipMemcpyDeviceToHost));
  int64_t with_slots = 0;
  for (int64_t i = 0; i < n; ++i) with_slots += hn[i] > 0;
  const unsigned blocks = (unsigned)((n + kRsvThreads - 1) / kRsvThreads);
  const unsigned long long zero[4] = {0, 0, 0, 0};
  HIP_TRY(hipMemcpyAsync(e->rsv_ws.p, zero, 32, hipMemcpyHostToDevice, e->stream));
  RsvExt X = rsv_ext(e);
  if (!e->dsx_q) X.dsx = nullptr;  // the variant run_rsv launches
  const int rf = rsv_eval_flags(X);
  auto launch = [&]() {
    if (which == 0)
      rsv_eval_kernel(rf)<<<blocks, kRsvThreads, 0, e->stream>>>(
          e->T, e->rsv_d.p, e->rsv_nd.p, e->pods.p, e->rpods.p, e->n_staged, n, 0, e->P, e->RP, X, e->rsv_val.p,
          e->rsv_part.p, e->out_keys.p, e->out_rslot.p, e->rsv_ws.p);
    else
      rsv_select<<<blocks, kRsvThreads, 0, e->stream>>>(e->rsv_val.p, e->pods.p, e->n_staged, n, 0, e->RP, X, e->rsv_part.p,
                                                         e->rsv_ws.p);
  };
  if (which == 1)  // rsv_select needs the packed values and partials of a real pass
    rsv_eval_kernel(rf)<<<blocks, kRsvThreads, 0, e->stream>>>(
        e->T, e->rsv_d.p, e->rsv_nd.p, e->pods.p, e->rpods.p, e->n_staged, n, 0, e->P, e->RP, X, e->rsv_val.p,
        e->rsv_part.p, e->out_keys.p, e->out_rslot.p, e->rsv_ws.p);
  launch();  // warm
  hipEvent_t a, b;
  HIP_TRY(hipEventCreate(&a));
  HIP_TRY(hipEventCreate(&b));
  HIP_TRY(hipEventRecord(a, e->stream));
  for (int k = 0; k < iters; ++k) launch();
  HIP_TRY(hipEventRecord(b, e->stream));
  HIP_TRY(hipEventSynchronize(b));
  float ms = 0;
  HIP_TRY(hipEventElapsedTime(&ms, a, b));
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  HIP_TRY(hipMemcpyAsync(e->rsv_ws.p, zero, 32, hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  if (avg_ms) *avg_ms = ms / iters;
  // rsv_eval: the Fit/LoadAware columns, rsv_n and the packed value per node, the slot rows of nodes holding
  // reservations and — for a device pod in a DeviceShare profile — the 272-B GPU row of every node
  bool dev_pod = false;
  if (e->ds_on) {
    DsPod d0;
    HIP_TRY(hipMemcpy(&d0, e->dpods.p, sizeof(DsPod), hipMemcpyDeviceToHost));
    dev_pod = !d0.skip;
  }
  // NodeNUMAResource: the NumaStatic + NodeAllocation rows and the stored affinity of every node
  if (algo_bytes)
    *algo_bytes = which == 0 ? (double)n * (76 + 4 + 8) + (double)with_slots * sizeof(RsvNode) +
                                   (dev_pod ? (double)n * sizeof(DsNode) : 0.0) +
                                   (e->numa_on ? (double)n * (sizeof(NumaStatic) + sizeof(NumaMut) + 4) : 0.0)
                             : (double)n * 8;
  return 0;
}

int kg_bench_kernel(kg_engine* e, int which, int iters, double* avg_ms, double* algo_bytes) {
  if (e && e->exact_on) return bench_rsv(e, which, iters, avg_ms, algo_bytes);
  if (!e || iters <= 0 || which < 0 || which > (e && e->ds_on ? 4 : 2)) return fail(KG_E_INVALID, "bad argument");
  if (e->n_staged <= 0) return fail(KG_E_INVALID, "stage a pod queue first");
  RoundGeom g;
  if (int rc = prepare_rounds(e, g)) return rc;
  const int64_t end = std::min<int64_t>(e->n_staged, g.B);
  // snapshot the mutable columns: the resolver writes rows back, replays must start from the same state
  const size_t bytes64 = (size_t)e->capacity * 8;
  DevBuf<int64_t> save;
  if (int rc = save.ensure((9 + (e->numa_on ? sizeof(NumaMut) / 8 : 0) + (e->ds_on ? sizeof(DsNode) / 8 : 0)) *
                           e->capacity))
    return rc;
  int64_t* mut64[8] = {e->T.req_cpu, e->T.req_mem, e->T.nz_cpu, e->T.nz_mem,
                       e->T.la_used_cpu, e->T.la_used_mem, e->T.la_pused_cpu, e->T.la_pused_mem};
  auto snapshot = [&](bool restore) -> int {
    for (int k = 0; k < 8; ++k) {
      int64_t* a = save.p + k * e->capacity;
      HIP_TRY(hipMemcpyAsync(restore ? mut64[k] : a, restore ? a : mut64[k], bytes64, hipMemcpyDeviceToDevice, e->stream));
    }
    int32_t* a = (int32_t*)(save.p + 8 * e->capacity);
    HIP_TRY(hipMemcpyAsync(restore ? e->T.num_pods : a, restore ? a : e->T.num_pods, e->capacity * 4,
                           hipMemcpyDeviceToDevice, e->stream));
    if (e->numa_on) {
      NumaMut* m = reinterpret_cast<NumaMut*>(save.p + 9 * e->capacity);
      HIP_TRY(hipMemcpyAsync(restore ? e->numa_m.p : m, restore ? m : e->numa_m.p, e->capacity * sizeof(NumaMut),
                             hipMemcpyDeviceToDevice, e->stream));
    }
    if (e->ds_on) {
      DsNode* m = reinterpret_cast<DsNode*>(save.p + 9 * e->capacity);
      HIP_TRY(hipMemcpyAsync(restore ? e->ds_d.p : m, restore ? m : e->ds_d.p, e->capacity * sizeof(DsNode),
                             hipMemcpyDeviceToDevice, e->stream));
    }
    return 0;
  };
  static const int64_t zero4[6] = {0, 0, 0, 0, 0, 0};
  const int nb = (int)end;
  if (int rc = snapshot(false)) return rc;
  HIP_TRY(hipMemcpyAsync(e->cursor.p, zero4, 48, hipMemcpyHostToDevice, e->stream));
  // one real round: valid lists and candidates to replay on
  if (int rc = e->ds_on ? launch_round_ds(e, g, end, e->stream) : run_batch(e, g, 0, end, 1)) return rc;
  HIP_TRY(hipGetLastError());
  if (int rc = snapshot(true)) return rc;
  hipEvent_t a, b;
  HIP_TRY(hipEventCreate(&a));
  HIP_TRY(hipEventCreate(&b));
  float total_ms = 0.f;
  for (int it = 0; it < iters; ++it) {
    HIP_TRY(hipMemcpyAsync(e->cursor.p, zero4, 48, hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipEventRecord(a, e->stream));
    if (e->ds_on) {
      if (int rc = launch_round_ds(e, g, end, e->stream, which)) return rc;
    }
    else if (which == 0) launch_eval(e, g, 0, nb, 0, e->stream);
    else if (which == 1) launch_merge_local(e, g, nb, 0, e->stream);
    else launch_resolve(e, g, 0, nb, 0, 0, 1, 0, e->stream);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(b, e->stream));
    HIP_TRY(hipEventSynchronize(b));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, a, b));
    total_ms += ms;
    if (which == 2)
      if (int rc = snapshot(true)) return rc;
  }
  HIP_TRY(hipStreamSynchronize(e->stream));
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  save.release();
  const double nbd = (double)end;
  if (avg_ms) *avg_ms = total_ms / iters;
  if (algo_bytes) {
    // eval: SURVEY §8(d) per-evaluation bytes (Fit 56 B + LoadAware 20 B = 76 B per node) × pods × nodes,
    //       + the candidate lists written;  merge: lists read + records written;  resolve: records + pods read.
    // NUMA profiles add the node's NumaStatic + NumaMut (232 B) to every evaluation
    const double per_node = kAlgoBytesPerNode + (e->numa_on ? (double)(sizeof(NumaStatic) + sizeof(NumaMut)) : 0.0) +
                            (e->ds_on ? (double)sizeof(DsNode) : 0.0);
    if (which == 3) *algo_bytes = nbd * (double)g.n_local * (per_node + 4.0) + nbd * g.nt_local * 8.0;  // + dsval
    else if (which == 0 && e->ds_on)  // eval_round_ds reads the packed values ds_max_round left, writes the lists
      *algo_bytes = nbd * (double)g.n_local * 4.0 + nbd * g.nt_local * kR * 8.0;
    else if (which == 4) *algo_bytes = nbd * g.nt_local * 8.0 + nbd * 8.0;
    else if (which == 0) *algo_bytes = nbd * (double)g.n_local * per_node + nbd * g.nt_local * kR * 8.0 + nbd * 96.0;
    else if (which == 1) *algo_bytes = nbd * g.nt_local * kR * 8.0 + nbd * kCandStride * 8.0;
    else *algo_bytes = nbd * kCandStride * 8.0 + nbd * 96.0;
  }
  return 0;
}

int kg_profile_enable(kg_engine* e, int on) {
  if (!e) return fail(KG_E_INVALID, "engine is NULL");
  e->prof_on = on != 0;
  for (int k = 0; k < KG_PROF_KINDS; ++k) e->prof_ms[k] = 0.0, e->prof_n[k] = 0;
  e->prof_recs.clear();
  e->prof_used = 0;
  return 0;
}

int kg_profile_read(kg_engine* e, double* ms_total, int64_t* launches) {
  if (!e) return fail(KG_E_INVALID, "engine is NULL");
  for (int k = 0; k < KG_PROF_KINDS; ++k) {
    if (ms_total) ms_total[k] = e->prof_ms[k];
    if (launches) launches[k] = e->prof_n[k];
  }
  return 0;
}

int kg_debug_eval_paths(kg_engine* e, int64_t* mismatches) {
  if (!e || !mismatches) return fail(KG_E_INVALID, "bad argument");
  if (int rc = sync_static(e)) return rc;
  if (e->n_staged <= 0) return fail(KG_E_INVALID, "stage a pod queue first");
  DevBuf<int64_t> b;
  if (int rc = b.ensure(1)) return rc;
  HIP_TRY(hipMemsetAsync(b.p, 0, 8, e->stream));
  const int64_t n = e->n_nodes;
  if (n > 0)
    debug_eval_paths<<<(unsigned)((n + 255) / 256), 256, 0, e->stream>>>(e->T, e->pods.p, e->n_staged, n, e->P,
                                                                         (unsigned long long*)b.p);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(mismatches, b.p, 8, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  b.release();
  return 0;
}

int kg_debug_stamps(kg_engine* e, uint64_t* out) {
#ifdef KG_STAMPS
  if (!e || !out) return fail(KG_E_INVALID, "bad argument");
  HIP_TRY(hipStreamSynchronize(e->stream));
  HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(kg::g_stamps), sizeof(kg::g_stamps), 0, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpyFromSymbol(out + 4 * 32 * 2, HIP_SYMBOL(kg::g_pod_diag), sizeof(kg::g_pod_diag), 0,
                              hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpyFromSymbol(out + 4 * 32 * 2 + 64 * 6, HIP_SYMBOL(kg::g_merge_count), sizeof(kg::g_merge_count), 0,
                              hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpyFromSymbol(out + 4 * 32 * 2 + 64 * 6 + 2, HIP_SYMBOL(kg::g_lane_diag), sizeof(kg::g_lane_diag), 0,
                              hipMemcpyDeviceToHost));
  return 0;
#else
  (void)e;
  (void)out;
  return fail(KG_E_UNSUPPORTED, "not a -DKG_STAMPS diagnostic build");
#endif
}

int kg_debug_numa_merge(kg_engine* e, const int64_t* cases, int64_t n, int64_t* out) {
  if (!e || (n > 0 && (!cases || !out))) return fail(KG_E_INVALID, "null argument");
  if (n <= 0) return 0;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t* c = cases + (size_t)i * KG_DBG_MERGE_WORDS;
    if (c[0] < 0 || c[0] > 3 || c[1] < 1 || c[1] > kNumaMax || c[2] < 1 || c[2] > 2)
      return fail(KG_E_INVALID, "merge case %lld: policy / NUMA count / list count", (long long)i);
  }
  DevBuf<int64_t> din, dout;
  if (int rc = din.ensure((size_t)n * KG_DBG_MERGE_WORDS)) return rc;
  if (int rc = dout.ensure((size_t)n * 8)) return rc;
  HIP_TRY(hipMemcpy(din.p, cases, (size_t)n * KG_DBG_MERGE_WORDS * 8, hipMemcpyHostToDevice));
  debug_numa_merge<<<(unsigned)((n + 63) / 64), 64, 0, e->stream>>>(din.p, n, dout.p);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(e->stream));
  HIP_TRY(hipMemcpy(out, dout.p, (size_t)n * 8 * 8, hipMemcpyDeviceToHost));
  return 0;
}

int kg_debug_least_requested(kg_engine* e, const int64_t* req, const int64_t* cap, int64_t* out, int64_t n) {
  if (!e || n < 0 || (n > 0 && (!req || !cap || !out))) return fail(KG_E_INVALID, "bad argument");
  if (n == 0) return 0;
  DevBuf<int64_t> b;
  if (int rc = b.ensure(3 * n)) return rc;
  HIP_TRY(hipMemcpyAsync(b.p, req, n * 8, hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipMemcpyAsync(b.p + n, cap, n * 8, hipMemcpyHostToDevice, e->stream));
  debug_least_requested<<<(unsigned)((n + 255) / 256), 256, 0, e->stream>>>(b.p, b.p + n, b.p + 2 * n, n);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(out, b.p + 2 * n, n * 8, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  b.release();
  return 0;
}

int kg_debug_fast_lrs(kg_engine* e, const int64_t* req, const int64_t* cap, int64_t* out_cpu, int64_t* out_mem,
                      int64_t n) {
  if (!e || n < 0 || (n > 0 && (!req || !cap || !out_cpu || !out_mem))) return fail(KG_E_INVALID, "bad argument");
  if (n == 0) return 0;
  DevBuf<int64_t> b;
  if (int rc = b.ensure(4 * n)) return rc;
  HIP_TRY(hipMemcpyAsync(b.p, req, n * 8, hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipMemcpyAsync(b.p + n, cap, n * 8, hipMemcpyHostToDevice, e->stream));
  debug_fast_lrs<<<(unsigned)((n + 255) / 256), 256, 0, e->stream>>>(b.p, b.p + n, b.p + 2 * n, b.p + 3 * n, n);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(out_cpu, b.p + 2 * n, n * 8, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipMemcpyAsync(out_mem, b.p + 3 * n, n * 8, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  b.release();
  return 0;
}

int kg_nodes_predicates_upsert(kg_engine* e, const kg_node_predicates* p, const int32_t* idx, int64_t n) {
  if (!e || (n > 0 && (!p || !idx))) return fail(KG_E_INVALID, "null argument");
  if (!e->def_on) return fail(KG_E_INVALID, "the profile enables none of TaintToleration / NodeAffinity / BalancedAllocation");
  if (n == 0) return 0;
  for (int64_t k = 0; k < n; ++k)
    if (idx[k] < 0 || idx[k] >= e->capacity) return fail(KG_E_INVALID, "node index %d outside capacity", idx[k]);
  std::vector<NodePred> h((size_t)n);
  for (int64_t k = 0; k < n; ++k) {
    if (p[k].predicate_count < 0 || p[k].predicate_count > 64 || p[k].image_count < 0 || p[k].image_count > 64)
      return fail(KG_E_INVALID, "node row %lld: predicate_count / image_count outside [0, 64]", (long long)k);
    if (p[k].zone < 0 || p[k].zone > KG_MAX_ZONES)
      return fail(KG_E_INVALID, "node predicates row %lld: zone %lld outside [0, %d]", (long long)k, (long long)p[k].zone,
                  KG_MAX_ZONES);
    h[k] = NodePred{p[k].predicates, p[k].taints_hard, p[k].taints_soft, p[k].images, (int32_t)p[k].zone, 0};
    const uint64_t t = p[k].taints_hard | p[k].taints_soft;
    const int i = idx[k];
    e->np_taint_top[i] = (int16_t)(t ? 64 - __builtin_clzll(t) : 0);
    e->np_pred_cnt[i] = (int16_t)p[k].predicate_count;
    e->np_img_cnt[i] = (int16_t)p[k].image_count;
  }
  e->np_dirty = true;
  DevBuf<uint8_t> b;
  if (int rc = b.ensure(n * (sizeof(NodePred) + 4))) return rc;
  NodePred* dp = reinterpret_cast<NodePred*>(b.p);
  int32_t* di = reinterpret_cast<int32_t*>(b.p + n * sizeof(NodePred));
  HIP_TRY(hipMemcpyAsync(dp, h.data(), n * sizeof(NodePred), hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipMemcpyAsync(di, idx, n * 4, hipMemcpyHostToDevice, e->stream));
  scatter_rows<NodePred><<<(unsigned)((n + 255) / 256), 256, 0, e->stream>>>(e->npred.p, dp, di, n);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(e->stream));
  b.release();
  return 0;
}

int kg_nodes_reservation_upsert(kg_engine* e, const kg_node_reservations* r, const int32_t* idx, int64_t n) {
  if (!e || (n > 0 && (!r || !idx))) return fail(KG_E_INVALID, "null argument");
  if (!e->rsv_on) return fail(KG_E_INVALID, "the profile does not enable Reservation");
  if (n == 0) return 0;
  std::vector<RsvNode> h(n);
  std::vector<int32_t> hn(n);
  std::vector<RsvGpu> hg((size_t)n * kRsvSlots);
  std::vector<RsvCpu> hc((size_t)n * kRsvSlots);
  bool any_gpu = false, any_cpu = false;
  for (int64_t k = 0; k < n; ++k) {
    if (idx[k] < 0 || idx[k] >= e->capacity) return fail(KG_E_INVALID, "node index %d outside capacity", idx[k]);
    if (int rc = decode_node_rsv(r[k], h[k], hn[k], hg.data() + (size_t)k * kRsvSlots, e->ds_on,
                                 hc.data() + (size_t)k * kRsvSlots, e->numa_on))
      return rc;
    for (int s = 0; s < hn[k]; ++s) {
      any_gpu |= (h[k].meta[s] & RS_GPU) != 0;
      any_cpu |= (h[k].meta[s] & RS_CPUS) != 0;
    }
  }
  // (ABI 15) the cpusets: allocated (zeroed) at the first cpu-holding slot, then scattered with every upsert
  if (any_cpu && !e->rsv_c.p) {
    if (int rc = e->rsv_c.ensure((size_t)kRsvSlots * e->capacity)) return rc;
    HIP_TRY(hipMemsetAsync(e->rsv_c.p, 0, sizeof(RsvCpu) * kRsvSlots * (size_t)e->capacity, e->stream));
  }
  if ((int64_t)e->rsv_cnode.size() < e->capacity) e->rsv_cnode.assign(e->capacity, 0);
  for (int64_t k = 0; k < n; ++k) {
    bool c = false;
    for (int s = 0; s < hn[k]; ++s) c |= (h[k].meta[s] & RS_CPUS) != 0;
    e->rcpu_nodes += (int64_t)c - (int64_t)e->rsv_cnode[idx[k]];
    e->rsv_cnode[idx[k]] = c ? 1 : 0;
  }
  // (ABI 13) the GPU holdings: allocated (zeroed) at the first GPU-holding slot, then scattered with every upsert
  if (any_gpu && !e->rsv_g.p) {
    if (int rc = e->rsv_g.ensure((size_t)kRsvSlots * e->capacity)) return rc;
    HIP_TRY(hipMemsetAsync(e->rsv_g.p, 0, sizeof(RsvGpu) * kRsvSlots * (size_t)e->capacity, e->stream));
  }
  if ((int64_t)e->rsv_gnode.size() < e->capacity) e->rsv_gnode.assign(e->capacity, 0);
  for (int64_t k = 0; k < n; ++k) {
    bool g = false;
    for (int s = 0; s < hn[k]; ++s) g |= (h[k].meta[s] & RS_GPU) != 0;
    e->rgpu_nodes += (int64_t)g - (int64_t)e->rsv_gnode[idx[k]];
    e->rsv_gnode[idx[k]] = g ? 1 : 0;
  }
  if ((int64_t)e->rsv_pcnt.size() < e->capacity) e->rsv_pcnt.assign(e->capacity, 64);
  for (int64_t k = 0; k < n; ++k) e->rsv_pcnt[idx[k]] = (int16_t)(r[k].n > 0 ? r[k].predicate_count : 64);
  e->rsv_pdirty = true;
  std::vector<uint64_t> hp((size_t)n * kRsvSlots);
  for (int64_t k = 0; k < n; ++k)
    for (int s = 0; s < kRsvSlots; ++s) hp[(size_t)k * kRsvSlots + s] = s < r[k].n ? r[k].predicates[s] : 0;
  DevBuf<uint8_t> b;
  const size_t pb = (size_t)n * kRsvSlots * 8;
  if (int rc = b.ensure(pb + n * (sizeof(RsvNode) + 8))) return rc;
  uint64_t* dp = reinterpret_cast<uint64_t*>(b.p);
  RsvNode* dd = reinterpret_cast<RsvNode*>(b.p + pb);
  int32_t* dn = reinterpret_cast<int32_t*>(b.p + pb + n * sizeof(RsvNode));
  int32_t* di = dn + n;
  HIP_TRY(hipMemcpyAsync(dp, hp.data(), pb, hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipMemcpyAsync(dd, h.data(), n * sizeof(RsvNode), hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipMemcpyAsync(dn, hn.data(), n * 4, hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipMemcpyAsync(di, idx, n * 4, hipMemcpyHostToDevice, e->stream));
  scatter_rsv<<<(unsigned)((n + 255) / 256), 256, 0, e->stream>>>(e->rsv_d.p, e->rsv_nd.p, e->rsv_pd.p, dd, dn, dp, di,
                                                                  n);
  HIP_TRY(hipGetLastError());
  DevBuf<RsvGpuNode> bg;
  if (e->rsv_g.p) {
    if (int rc = bg.ensure(n)) return rc;
    HIP_TRY(hipMemcpyAsync(bg.p, hg.data(), n * sizeof(RsvGpuNode), hipMemcpyHostToDevice, e->stream));
    scatter_rows<RsvGpuNode><<<(unsigned)((n + 255) / 256), 256, 0, e->stream>>>(
        reinterpret_cast<RsvGpuNode*>(e->rsv_g.p), bg.p, di, n);
    HIP_TRY(hipGetLastError());
  }
  DevBuf<RsvCpuNode> bc;
  if (e->rsv_c.p) {
    if (int rc = bc.ensure(n)) return rc;
    HIP_TRY(hipMemcpyAsync(bc.p, hc.data(), n * sizeof(RsvCpuNode), hipMemcpyHostToDevice, e->stream));
    scatter_rows<RsvCpuNode><<<(unsigned)((n + 255) / 256), 256, 0, e->stream>>>(
        reinterpret_cast<RsvCpuNode*>(e->rsv_c.p), bc.p, di, n);
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(hipStreamSynchronize(e->stream));
  b.release();
  bg.release();
  bc.release();
  return 0;
}

int kg_nodes_read_reservation_cpus(kg_engine* e, uint64_t* cpus_assigned) {
  if (!e || !cpus_assigned) return fail(KG_E_INVALID, "null argument");
  if (!e->rsv_on) return fail(KG_E_INVALID, "the profile does not enable Reservation");
  const int64_t n = e->n_nodes;
  const size_t per = (size_t)KG_MAX_RSV_SLOTS * kCpuWords;
  std::memset(cpus_assigned, 0, (size_t)n * per * 8);
  if (n == 0 || !e->rsv_c.p) return 0;
  std::vector<RsvCpu> h((size_t)n * kRsvSlots);
  HIP_TRY(hipMemcpyAsync(h.data(), e->rsv_c.p, h.size() * sizeof(RsvCpu), hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  for (int64_t i = 0; i < n; ++i)
    for (int s = 0; s < kRsvSlots; ++s)
      for (int w = 0; w < kCpuWords; ++w) cpus_assigned[(size_t)i * per + (size_t)s * kCpuWords + w] = h[(size_t)i * kRsvSlots + s].u[w];
  return 0;
}

int kg_nodes_read_reservation_gpus(kg_engine* e, int64_t* gpu_allocated) {
  if (!e || !gpu_allocated) return fail(KG_E_INVALID, "null argument");
  if (!e->rsv_on) return fail(KG_E_INVALID, "the profile does not enable Reservation");
  const int64_t n = e->n_nodes;
  const size_t per = (size_t)KG_MAX_RSV_SLOTS * KG_MAX_MINORS * 3;
  std::memset(gpu_allocated, 0, (size_t)n * per * 8);
  if (n == 0 || !e->rsv_g.p) return 0;
  std::vector<RsvGpu> h((size_t)n * kRsvSlots);
  HIP_TRY(hipMemcpyAsync(h.data(), e->rsv_g.p, h.size() * sizeof(RsvGpu), hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  for (int64_t i = 0; i < n; ++i)
    for (int s = 0; s < kRsvSlots; ++s)
      for (int m = 0; m < kMinors; ++m) {
        const RsvGpu& g = h[(size_t)i * kRsvSlots + s];
        int64_t* o = gpu_allocated + (size_t)i * per + ((size_t)s * KG_MAX_MINORS + m) * 3;
        o[0] = g.dcore[m];
        o[1] = g.dmem[m];
        o[2] = g.dratio[m];
      }
  return 0;
}

int kg_nodes_read_reservations(kg_engine* e, int64_t* allocated_cpu, int64_t* allocated_mem, int64_t* assigned) {
  if (!e) return fail(KG_E_INVALID, "engine is NULL");
  if (!e->rsv_on) return fail(KG_E_INVALID, "the profile does not enable Reservation");
  const int64_t n = e->n_nodes;
  if (n == 0) return 0;
  std::vector<RsvNode> h(n);
  std::vector<int32_t> hn(n);
  HIP_TRY(hipMemcpyAsync(h.data(), e->rsv_d.p, n * sizeof(RsvNode), hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipMemcpyAsync(hn.data(), e->rsv_nd.p, n * 4, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  for (int64_t i = 0; i < n; ++i)
    for (int s = 0; s < KG_MAX_RSV_SLOTS; ++s) {
      const bool on = s < hn[i];
      if (allocated_cpu) allocated_cpu[i * KG_MAX_RSV_SLOTS + s] = on ? h[i].allocd_cpu[s] : 0;
      if (allocated_mem) allocated_mem[i * KG_MAX_RSV_SLOTS + s] = on ? h[i].allocd_mem[s] : 0;
      if (assigned) assigned[i * KG_MAX_RSV_SLOTS + s] = on ? h[i].assigned[s] : 0;
    }
  return 0;
}

int kg_nodes_read_pod_groups(kg_engine* e, int32_t* match_count, int32_t* anti_count, int32_t* sym_weight,
                             int32_t* anti_zone, int32_t* sym_zone) {
  if (!e) return fail(KG_E_INVALID, "engine is NULL");
  if (!e->grp_on) return fail(KG_E_INVALID, "the profile enables neither PodTopologySpread nor InterPodAffinity");
  const int64_t n = e->n_nodes, cap = e->capacity;
  if (n == 0) return 0;
  std::vector<int32_t> h((size_t)kGroupArrays * kGroups * cap);
  HIP_TRY(hipMemcpyAsync(h.data(), e->grp_d.p, h.size() * 4, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  int32_t* outs[kGroupArrays] = {match_count, anti_count, sym_weight, anti_zone, sym_zone};
  for (int a = 0; a < kGroupArrays; ++a)
    if (outs[a])
      for (int64_t i = 0; i < n; ++i)
        for (int k = 0; k < kGroups; ++k) outs[a][i * kGroups + k] = h[((size_t)a * kGroups + k) * cap + i];
  return 0;
}

int kg_pods_evaluate_reservation(kg_engine* e, const kg_pod* pod, int64_t* out) {
  if (!e || !pod || !out) return fail(KG_E_INVALID, "null argument");
  if (!e->exact_on) return fail(KG_E_INVALID, "the profile does not run the exact pass (Reservation or NUMA + DeviceShare)");
  if (e->grp_on)
    return fail(KG_E_UNSUPPORTED, "kg_pods_evaluate_reservation: PodTopologySpread / InterPodAffinity need the pass's "
                "cluster-wide reductions (use kg_pods_schedule)");
  if (int rc = sync_static(e)) return rc;
  DevPod d;
  if (int rc = decode_pod(e, *pod, d)) return rc;
  RsvPod rp;
  RsvSel rs;
  if (int rc = decode_rsv_pod(*pod, rp, rs, 0)) return rc;
  if (int rc = check_rsv_predicates(e, rsv_pred_top(rp, rs))) return rc;
  if (rp.flags & RP_SEL) rp.aux = 0;  // the scratch copy below
  DsPod dsp{};
  dsp.skip = 1;
  if (e->ds_on)
    if (int rc = decode_ds_pod(*pod, dsp)) return rc;
  NumaPod np{};
  if (e->numa_on)
    if (int rc = decode_numa_pod(e->cfg, *pod, np)) return rc;
  const int64_t n = e->n_nodes;
  if (n == 0) return 0;
  const int64_t words = (int64_t)KG_RSV_EVAL_WORDS * n;
  const int64_t pw = kPodWords + (int64_t)(sizeof(RsvPod) / 8) + kDsPodWords + kNumaPodWords;
  if (int rc = e->scratch64.ensure(words + pw + sizeof(RsvSel) / 8)) return rc;
  RsvSel* gs = reinterpret_cast<RsvSel*>(e->scratch64.p + words + pw);
  DevPod* gp = reinterpret_cast<DevPod*>(e->scratch64.p + words);
  RsvPod* gr = reinterpret_cast<RsvPod*>(e->scratch64.p + words + kPodWords);
  DsPod* gd = reinterpret_cast<DsPod*>(e->scratch64.p + words + kPodWords + sizeof(RsvPod) / 8);
  NumaPod* gn = reinterpret_cast<NumaPod*>(e->scratch64.p + words + kPodWords + sizeof(RsvPod) / 8 + kDsPodWords);
  HIP_TRY(hipMemcpyAsync(gp, &d, sizeof(d), hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipMemcpyAsync(gr, &rp, sizeof(rp), hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipMemcpyAsync(gd, &dsp, sizeof(dsp), hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipMemcpyAsync(gn, &np, sizeof(np), hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipMemcpyAsync(gs, &rs, sizeof(rs), hipMemcpyHostToDevice, e->stream));
  RsvExt X = rsv_ext(e);
  X.rsv_sel = gs;
  X.aff = nullptr;  // no pass affinity store: this is not a scheduling pass
  evaluate_pod_rsv<<<(unsigned)((n + 255) / 256), 256, 0, e->stream>>>(e->T, e->rsv_d.p, e->rsv_nd.p, gp, gr,
                                                                       e->ds_on ? gd : nullptr,
                                                                       e->numa_on ? gn : nullptr, n, e->P, e->RP, X,
                                                                       e->scratch64.p);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(out, e->scratch64.p, words * 8, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return 0;
}

// the pod and its victims of one dry-run call, decoded and checked (the shared front half of the two entry points).
// (r6) NodeNUMAResource, DeviceShare and TaintToleration / NodeAffinity run in the dry run too (PreExt); refused:
// PodTopologySpread / InterPodAffinity (their PreFilterExtensions move cluster-wide counters) and DeviceShare with
// reservations that hold GPUs (preemptibleInRRs of devices).
static int preempt_prepare(kg_engine* e, const kg_pod* pod, const kg_pod* victims, const int32_t* victim_slot,
                           const int32_t* victim_minors, int64_t n_victims, DevPod& d, RsvPod& rp, RsvSel& rs,
                           int64_t (&rq)[kAux], std::vector<Victim>& hv, PreExt& X) {
  if (e->grp_on)
    return fail(KG_E_UNSUPPORTED, "preemption dry run: PodTopologySpread / InterPodAffinity keep the Go path (their "
                "AddPod / RemovePod move cluster-wide counters)");
  if (e->ds_on && e->rsv_on && e->rgpu_nodes > 0)
    return fail(KG_E_UNSUPPORTED, "preemption dry run: DeviceShare with reservations that hold GPUs keeps the Go path "
                "(preemptibleInRRs of devices)");
  if (int rc = sync_static(e)) return rc;
  if (int rc = decode_pod(e, *pod, d)) return rc;
  for (int q = 0; q < kAux; ++q) rq[q] = pod->requests[kAuxFirst + q];
  if (int rc = decode_rsv_pod(*pod, rp, rs, 0)) return rc;
  if (int rc = check_rsv_predicates(e, rsv_pred_top(rp, rs))) return rc;
  if (rp.flags & RP_SEL) rp.aux = 0;
  if (rp.flags & (RP_RESERVE | RP_OPERATING))
    return fail(KG_E_UNSUPPORTED, "preemption dry run for a reserve pod / reservation operating mode keeps the Go path");
  X = PreExt{};
  X.dp.skip = 1;
  if (e->numa_on) {
    if (int rc = decode_numa_pod(e->cfg, *pod, X.np)) return rc;
    X.ns = e->numa_s.p, X.nm = e->numa_m.p, X.NP = e->NP;
  }
  if (e->ds_on) {
    if (int rc = decode_ds_pod(*pod, X.dp)) return rc;
    X.ds = e->ds_d.p, X.dsx = e->dsx_d.p, X.DP = e->DP;
  } else {
    for (int r = 0; r < KG_DEV_RES_MAX; ++r)
      if (pod->device_requests[r] != 0 && e->cfg.fit_filter)
        return fail(KG_E_UNSUPPORTED, "the pod requests devices; the profile has no DeviceShare");
  }
  if (e->def_on) {
    if (int rc = decode_def_pod(*pod, X.df, 0)) return rc;
    if (int rc = check_pod_tables(e, *pod)) return rc;
    X.pred = e->npred.p, X.DF = e->DF;
  }
  hv.resize((size_t)std::max<int64_t>(n_victims, 1));
  for (int64_t k = 0; k < n_victims; ++k) {
    DevPod v;
    if (int rc = decode_pod(e, victims[k], v)) return rc;
    const int32_t s = victim_slot ? victim_slot[k] : -1;
    if (s < -1 || s >= KG_MAX_RSV_SLOTS) return fail(KG_E_INVALID, "victim %lld: reservation slot %d", (long long)k, s);
    const int32_t m = victim_minors ? victim_minors[k] : 0;
    if (m < 0 || m >= (1 << (8 * (1 + kXTypes)))) return fail(KG_E_INVALID, "victim %lld: minors 0x%x", (long long)k, m);
    bool nz = false;
    for (int q = 0; q < KG_RES_MAX; ++q) nz |= victims[k].requests[q] != 0;
    // (r5) RemovePod returns before counting a reserve pod (reservation/plugin.go:286): the framework still
    // removes it from the NodeInfo copy, but it never becomes preemptible
    const bool reserve = (victims[k].flags & KG_POD_RESERVE) != 0;
    if (reserve) nz = false;
    Victim w{};
    w.req_cpu = v.req_cpu, w.req_mem = v.req_mem, w.nz_cpu = v.nz_cpu, w.nz_mem = v.nz_mem;
    w.slot = s, w.nonzero = nz ? 1 : 0, w.reserve = reserve ? 1 : 0;
    for (int q = 0; q < kAux; ++q) w.aux[q] = victims[k].requests[kAuxFirst + q];
    w.dp.skip = 1;
    if (e->ds_on && m != 0) {
      if (int rc = decode_ds_pod(victims[k], w.dp)) return rc;
      if (w.dp.skip || w.dp.error)
        return fail(KG_E_INVALID, "victim %lld holds minors 0x%x but requests no valid GPU share", (long long)k, m);
      w.dminors = m;
    }
    hv[k] = w;
  }
  return 0;
}

int kg_pods_filter_preemption(kg_engine* e, const kg_pod* pod, int32_t node_idx, const kg_pod* victims,
                              const int32_t* victim_slot, const int32_t* victim_minors, int64_t n_victims,
                              int32_t* out_reject) {
  if (!e || !pod || !out_reject || n_victims < 0 || (n_victims > 0 && !victims)) return fail(KG_E_INVALID, "null argument");
  if (node_idx < 0 || node_idx >= e->n_nodes) return fail(KG_E_INVALID, "node index %d outside [0, %lld)", node_idx,
                                                           (long long)e->n_nodes);
  DevPod d;
  RsvPod rp;
  RsvSel rs;
  int64_t rq[kAux];
  std::vector<Victim> hv;
  PreExt X;
  if (int rc = preempt_prepare(e, pod, victims, victim_slot, victim_minors, n_victims, d, rp, rs, rq, hv, X)) return rc;
  const size_t vw = (hv.size() * sizeof(Victim) + 7) / 8;
  if (int rc = e->scratch64.ensure(kPodWords + kAux + vw + 1 + sizeof(RsvSel) / 8)) return rc;
  DevPod* gp = reinterpret_cast<DevPod*>(e->scratch64.p);
  int64_t* ga = reinterpret_cast<int64_t*>(e->scratch64.p + kPodWords);
  Victim* gv = reinterpret_cast<Victim*>(e->scratch64.p + kPodWords + kAux);
  int32_t* go = reinterpret_cast<int32_t*>(e->scratch64.p + kPodWords + kAux + vw);
  RsvSel* gs = reinterpret_cast<RsvSel*>(e->scratch64.p + kPodWords + kAux + vw + 1);
  HIP_TRY(hipMemcpyAsync(gp, &d, sizeof(d), hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipMemcpyAsync(ga, rq, sizeof(rq), hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipMemcpyAsync(gs, &rs, sizeof(rs), hipMemcpyHostToDevice, e->stream));
  if (n_victims > 0) HIP_TRY(hipMemcpyAsync(gv, hv.data(), (size_t)n_victims * sizeof(Victim), hipMemcpyHostToDevice, e->stream));
  filter_pod_preempt<<<1, kWave, 0, e->stream>>>(e->T, e->rsv_d.p, e->rsv_nd.p, e->rsv_pd.p, gs, node_idx, gp, ga, rp,
                                                 e->P, e->RP, e->rsv_on ? 1 : 0, gv, n_victims, go, X);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(out_reject, go, 4, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return 0;
}

int kg_pods_select_victims(kg_engine* e, const kg_pod* pod, int64_t n_candidates, const int32_t* node_idx,
                           const int64_t* victim_offsets, const kg_pod* victims, const int32_t* victim_slot,
                           const int32_t* victim_minors, const uint8_t* pdb_violating, int32_t* out_reject, uint8_t* out_victim,
                           int32_t* out_violating) {
  if (!e || !pod || n_candidates < 0 || (n_candidates > 0 && (!node_idx || !victim_offsets || !out_reject ||
                                                              !out_violating)))
    return fail(KG_E_INVALID, "null argument");
  if (n_candidates == 0) return 0;
  if (victim_offsets[0] != 0) return fail(KG_E_INVALID, "victim_offsets[0] must be 0");
  for (int64_t c = 0; c < n_candidates; ++c) {
    if (node_idx[c] < 0 || node_idx[c] >= e->n_nodes)
      return fail(KG_E_INVALID, "candidate %lld: node index %d outside [0, %lld)", (long long)c, node_idx[c],
                  (long long)e->n_nodes);
    if (victim_offsets[c + 1] < victim_offsets[c])
      return fail(KG_E_INVALID, "victim_offsets decrease at candidate %lld", (long long)c);
  }
  const int64_t nv = victim_offsets[n_candidates];
  if (nv > 0 && (!victims || !out_victim)) return fail(KG_E_INVALID, "null argument");
  DevPod d;
  RsvPod rp;
  RsvSel rs;
  int64_t rq[kAux];
  std::vector<Victim> hv;
  PreExt X;
  if (int rc = preempt_prepare(e, pod, victims, victim_slot, victim_minors, nv, d, rp, rs, rq, hv, X)) return rc;
  // one device buffer: pod, pod aux, RsvSel, victims, offsets, nodes, violating flags, then the outputs
  auto words = [](size_t bytes) { return (bytes + 7) / 8; };
  const size_t w_pod = kPodWords, w_aux = kAux, w_sel = words(sizeof(RsvSel)), w_vic = words(hv.size() * sizeof(Victim));
  const size_t w_off = (size_t)n_candidates + 1, w_nodes = words((size_t)n_candidates * 4),
               w_viol = words((size_t)std::max<int64_t>(nv, 1)), w_rej = words((size_t)n_candidates * 4),
               w_out = words((size_t)std::max<int64_t>(nv, 1)), w_nvio = words((size_t)n_candidates * 4);
  size_t o = 0;
  const size_t o_pod = o; o += w_pod;
  const size_t o_aux = o; o += w_aux;
  const size_t o_sel = o; o += w_sel;
  const size_t o_vic = o; o += w_vic;
  const size_t o_off = o; o += w_off;
  const size_t o_nodes = o; o += w_nodes;
  const size_t o_viol = o; o += w_viol;
  const size_t o_rej = o; o += w_rej;
  const size_t o_out = o; o += w_out;
  const size_t o_nvio = o; o += w_nvio;
  if (int rc = e->scratch64.ensure(o)) return rc;
  int64_t* b = e->scratch64.p;
  HIP_TRY(hipMemcpyAsync(b + o_pod, &d, sizeof(d), hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipMemcpyAsync(b + o_aux, rq, sizeof(rq), hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipMemcpyAsync(b + o_sel, &rs, sizeof(rs), hipMemcpyHostToDevice, e->stream));
  if (nv > 0) HIP_TRY(hipMemcpyAsync(b + o_vic, hv.data(), (size_t)nv * sizeof(Victim), hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipMemcpyAsync(b + o_off, victim_offsets, w_off * 8, hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipMemcpyAsync(b + o_nodes, node_idx, (size_t)n_candidates * 4, hipMemcpyHostToDevice, e->stream));
  const uint8_t* gviol = nullptr;
  if (pdb_violating && nv > 0) {
    HIP_TRY(hipMemcpyAsync(b + o_viol, pdb_violating, (size_t)nv, hipMemcpyHostToDevice, e->stream));
    gviol = reinterpret_cast<const uint8_t*>(b + o_viol);
  }
  const unsigned blocks = (unsigned)((n_candidates + kWave - 1) / kWave);
  select_victims<<<blocks, kWave, 0, e->stream>>>(e->T, e->rsv_d.p, e->rsv_nd.p, e->rsv_pd.p,
                                                  reinterpret_cast<const RsvSel*>(b + o_sel),
                                                  reinterpret_cast<const DevPod*>(b + o_pod),
                                                  reinterpret_cast<const int64_t*>(b + o_aux), rp, e->P, e->RP,
                                                  e->rsv_on ? 1 : 0, n_candidates,
                                                  reinterpret_cast<const int32_t*>(b + o_nodes),
                                                  reinterpret_cast<const int64_t*>(b + o_off),
                                                  reinterpret_cast<const Victim*>(b + o_vic), gviol,
                                                  reinterpret_cast<int32_t*>(b + o_rej),
                                                  reinterpret_cast<uint8_t*>(b + o_out),
                                                  reinterpret_cast<int32_t*>(b + o_nvio), X);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(out_reject, b + o_rej, (size_t)n_candidates * 4, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipMemcpyAsync(out_violating, b + o_nvio, (size_t)n_candidates * 4, hipMemcpyDeviceToHost, e->stream));
  if (nv > 0) HIP_TRY(hipMemcpyAsync(out_victim, b + o_out, (size_t)nv, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return 0;
}

int kg_results_fetch_reservations(kg_engine* e, int64_t first, int64_t count, int32_t* out_slot) {
  if (!e || (count > 0 && !out_slot)) return fail(KG_E_INVALID, "null argument");
  if (first < 0 || count < 0 || first + count > e->n_staged) return fail(KG_E_INVALID, "staged range");
  if (!e->rsv_on) {
    for (int64_t i = 0; i < count; ++i) out_slot[i] = -1;
    return 0;
  }
  if (count > 0) {
    HIP_TRY(hipMemcpyAsync(out_slot, e->out_rslot.p + first, count * 4, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
  }
  return 0;
}

}  // extern "C"
