// Batched exact rounds (SURVEY §8a A15–A24 on the profiles the per-pod exact pass runs: Reservation, the shipped
// NodeNUMAResource + DeviceShare profile, the upstream defaults): kXrPods FIFO pods per round instead of one pod per
// device pass.  Included by engine.hip inside its kernel namespace (uses kTile / kNPT / kR / select_write).
//
// A round over pods [c, c + nb), c = the device cursor ws[3]:
//   xr_eval    every (pod, node) of the round through rsv_eval_node on the round-start state (BeforePreFilter restore,
//              every Filter, the un-normalised totals and raw Scores): val[k][i] (rsv_pack), val2[k][i] (raw
//              TaintToleration / NodeAffinity), aff[k][i] (the NUMA affinity Reserve needs), and per (pod, tile) the
//              PreScore preferred-node key and, per normalised Score, (max + 1, holders);
//   xr_norm    per pod: the round-start maxima and holder counts over all nodes;
//   xr_select  per (pod, tile): the weighted totals with the round-start maxima (rsv_total, as rsv_select) → top-kR;
//   merge      merge_round: per pod the kC best keys + ub (a strict bound on every key left out);
//   xr_resolve one wave replays the pods in order (ElasticQuota PreFilter, winner, Reserve).  Lane l owns the l-th
//              row modified in this round and re-runs pod j on it (the exact current key).  The round-start keys
//              of unmodified rows stay exact while the normalisation of pod j is unchanged, so pod j is resolved
//              iff: no modified row raises a maximum or, having been a holder of it, lowers it when every holder
//              was modified (the holder count says so); the preferred node neither moves nor changes; and the best
//              candidate is ≥ ub.  Otherwise the round stops before pod j and the next round starts there.
// The first pod of a round always resolves (nothing modified yet), so every round makes progress.
// (r5) Several ranks: each rank evaluates its own range of tiles (xr_eval / xr_select over tiles [tile_base,
// tile_base + nt)), the per-pod statistics and the merged records are all-gathered (xr_norm_combine, merge_round<true>),
// and xr_fill evaluates, on this rank's replica of the round-start table, the candidates of the merged records that
// lie in other ranks' shards — the only nodes outside the shard whose round-start values the resolver reads (a
// winner and every modified row is a listed candidate).  The table and the resolver stay replicated.
#pragma once

constexpr int kXrPods = 32;      // pods per round (< kWave: one modified row per resolver lane)
constexpr int kXrPpw = 2;        // pods per select wave (4 x 2 = 8 waves per tile group: enough waves to fill the chip)
constexpr int kXrNorm = 5;       // per-pod statistics: preferred key, raw Reservation, DeviceShare, taint, affinity
// Exact-round features (compile-time: the kernels carry only the plugins the profile enables, so the Fit /
// LoadAware / Reservation-only variants keep their registers, and none spills for code it never runs)
constexpr int XF_NUMA = 1, XF_DS = 2, XF_DEF = 4;
static_assert(kXrPods < kWave, "resolver lanes");

__device__ __forceinline__ bool xr_range(const unsigned long long* __restrict__ ws, int64_t& first, int& nb) {
  first = (int64_t)ws[3];
  const int64_t left = (int64_t)ws[4] - first;
  nb = left < kXrPods ? (int)left : kXrPods;
  return nb > 0;
}

// (max + 1, count) of one statistic over a wave; v = value + 1 (0 = infeasible)
__device__ __forceinline__ uint64_t xr_wave_maxcount(uint32_t m, uint32_t c) {
  const uint32_t wm = wave_max_u32(m);
  const uint32_t wc = wave_sum_u32(m == wm ? c : 0u);
  return ((uint64_t)wm << 32) | wc;
}
__device__ __forceinline__ void xr_acc(uint32_t v, uint32_t& m, uint32_t& c) {
  c = v > m ? 1u : c + (v == m && v != 0 ? 1u : 0u);
  m = v > m ? v : m;
}
__device__ __forceinline__ void xr_tile_coords(int n_pg, int& tile, int& p0) {
  const int wave = threadIdx.x / kWave;
  const uint32_t nwg = gridDim.x, bid = blockIdx.x, xcd = bid % 8u, q = nwg / 8u, r = nwg % 8u;
  const uint32_t wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8u;  // XCD-aware swizzle
  tile = (int)(wgid / (uint32_t)n_pg) * kEvalWaves + wave;
  p0 = (int)(wgid % (uint32_t)n_pg) * kXrPpw;
}

// One block per (256-node tile, group of kXrEvalPpw pods), one node per thread: rsv_eval_node is long and divergent
// (NUMA hints, DeviceShare minors, reservation slots), so the parallelism is in the (pod, node) pairs, not in several
// nodes per lane (a 50k-node round then had < 1 wave per SIMD).  The per-(pod, tile) statistics are combined over the
// block's waves in LDS.
constexpr int kXrEvalPpw = 2;
template <int XF>
__global__ __launch_bounds__(kTile) void xr_eval(DevTable T, const RsvNode* __restrict__ RN,
                                                 const int32_t* __restrict__ rsv_n, const DevPod* __restrict__ pods,
                                                 const RsvPod* __restrict__ rpods, int64_t n, int nt, int tile_base,
                                                 int64_t stride, EvalParams P, RsvParams RP, RsvExt X,
                                                 uint64_t* __restrict__ val, uint32_t* __restrict__ val2,
                                                 uint32_t* __restrict__ affk, uint64_t* __restrict__ part,
                                                 const unsigned long long* __restrict__ ws) {
  __shared__ uint64_t s_st[kTile / kWave][kXrNorm];
  int64_t first;
  int nb;
  if (!xr_range(ws, first, nb)) return;
  constexpr int n_pg = kXrPods / kXrEvalPpw;
  const uint32_t nwg = gridDim.x, bid = blockIdx.x, xcd = bid % 8u, q8 = nwg / 8u, r8 = nwg % 8u;
  const uint32_t wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8u;  // XCD-aware swizzle
  const int tile = (int)(wgid / (uint32_t)n_pg), p0 = (int)(wgid % (uint32_t)n_pg) * kXrEvalPpw;
  if (tile >= nt || p0 >= nb) return;  // block-uniform
  const int tid = threadIdx.x, lane = tid % kWave, wave = tid / kWave;
  const int p1 = p0 + kXrEvalPpw < nb ? p0 + kXrEvalPpw : nb;
  const int64_t i = (int64_t)(tile_base + tile) * kTile + tid;  // nt tiles of this rank's shard
  for (int k = p0; k < p1; ++k) {
    const int64_t j = first + k;
    uint64_t pk = 0;
    uint32_t m[4] = {0, 0, 0, 0};
    if (i < n) {
      const DevPod p = pods[j];
      const RsvPod rp = rpods[j];
      const DsPod* dp = (XF & XF_DS) ? &X.dpods[j] : nullptr;
      const NumaPod* np = (XF & XF_NUMA) ? &X.npods[j] : nullptr;
      const int64_t* aux = (X.paux && (p.flags & P_AUX)) ? X.paux + (size_t)j * kAux : nullptr;
      const DefPod* df = (XF & XF_DEF) ? &X.defp[j] : nullptr;
      RsvExt Xk = X;
      Xk.aff = X.aff ? affk + (size_t)k * stride : nullptr;  // rsv_eval_node stores the NUMA affinity per node
      const RsvOut o = rsv_eval_node<false, false>(T, RN, rsv_n, i, p, rp, P, RP, Xk, dp, np, nullptr, aux, df);
      uint64_t v = 0;
      uint32_t v2 = 0;
      if (o.feas) {
        v = rsv_pack(o);
        v2 = ((uint32_t)o.tcnt << 24) | (uint32_t)o.asum;
        pk = rsv_pref_key(o, (uint32_t)i);
        m[0] = (uint32_t)o.raw + 1u;
        m[1] = (uint32_t)o.dsraw + 1u;
        m[2] = (uint32_t)o.tcnt + 1u;
        m[3] = (uint32_t)o.asum + 1u;
      }
      val[(size_t)k * stride + i] = v;
      if (val2) val2[(size_t)k * stride + i] = v2;
    }
    pk = wave_max_u64_dpp(pk);
    uint64_t s[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) s[q] = xr_wave_maxcount(m[q], m[q] != 0 ? 1u : 0u);
    if (lane == 0) {
      s_st[wave][0] = pk;
#pragma unroll
      for (int q = 0; q < 4; ++q) s_st[wave][1 + q] = s[q];
    }
    __syncthreads();
    if (tid < kXrNorm) {  // thread q combines statistic q over the block's waves
      uint64_t r = 0;
      if (tid == 0) {
        for (int w = 0; w < kTile / kWave; ++w) r = s_st[w][0] > r ? s_st[w][0] : r;
      } else {
        uint32_t M = 0, C = 0;
        for (int w = 0; w < kTile / kWave; ++w) {
          const uint32_t vm = (uint32_t)(s_st[w][tid] >> 32), vc = (uint32_t)s_st[w][tid];
          C = vm > M ? vc : C + (vm == M ? vc : 0u);
          M = vm > M ? vm : M;
        }
        r = ((uint64_t)M << 32) | C;
      }
      part[((size_t)k * nt + tile) * kXrNorm + tid] = r;
    }
    __syncthreads();
  }
}

// one block per pod: norm[k] = {preferred key, (M + 1) << 32 | holders for raw, ds, taint, affinity}
__global__ __launch_bounds__(256) void xr_norm(const uint64_t* __restrict__ part, int nt,
                                               uint64_t* __restrict__ norm, const unsigned long long* __restrict__ ws) {
  __shared__ uint64_t s_v[256 / kWave][kXrNorm];
  int64_t first;
  int nb;
  if (!xr_range(ws, first, nb)) return;
  const int k = blockIdx.x;
  if (k >= nb) return;
  const int tid = threadIdx.x, lane = tid % kWave, wave = tid / kWave;
  uint64_t pk = 0;
  uint32_t m[4] = {0, 0, 0, 0}, c[4] = {0, 0, 0, 0};
  for (int t = tid; t < nt; t += 256) {
    const uint64_t* o = part + ((size_t)k * nt + t) * kXrNorm;
    pk = o[0] > pk ? o[0] : pk;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t vm = (uint32_t)(o[1 + q] >> 32), vc = (uint32_t)o[1 + q];
      c[q] = vm > m[q] ? vc : c[q] + (vm == m[q] ? vc : 0u);
      m[q] = vm > m[q] ? vm : m[q];
    }
  }
  pk = wave_max_u64_dpp(pk);
  uint64_t s[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) s[q] = xr_wave_maxcount(m[q], c[q]);
  if (lane == 0) {
    s_v[wave][0] = pk;
#pragma unroll
    for (int q = 0; q < 4; ++q) s_v[wave][1 + q] = s[q];
  }
  __syncthreads();
  if (tid < kXrNorm) {
    uint64_t r = 0;
    if (tid == 0) {
      for (int w = 0; w < 256 / kWave; ++w) r = s_v[w][0] > r ? s_v[w][0] : r;
    } else {
      uint32_t M = 0, C = 0;
      for (int w = 0; w < 256 / kWave; ++w) {
        const uint32_t vm = (uint32_t)(s_v[w][tid] >> 32), vc = (uint32_t)s_v[w][tid];
        C = vm > M ? vc : C + (vm == M ? vc : 0u);
        M = vm > M ? vm : M;
      }
      r = ((uint64_t)M << 32) | C;
    }
    norm[(size_t)k * kXrNorm + tid] = r;
  }
}

// several ranks: the global statistics per pod from the ranks' all-gathered xr_norm values ([n_ranks][kXrPods][kXrNorm]):
// the preferred key's maximum, and per normalised Score the max of M + 1 with the holders summed over the ranks at it
__global__ __launch_bounds__(kXrPods* kXrNorm) void xr_norm_combine(const uint64_t* __restrict__ all, int n_ranks,
                                                                     uint64_t* __restrict__ norm,
                                                                     const unsigned long long* __restrict__ ws) {
  int64_t first;
  int nb;
  if (!xr_range(ws, first, nb)) return;
  const int t = threadIdx.x, k = t / kXrNorm, q = t % kXrNorm;
  if (k >= nb) return;
  uint64_t r = 0;
  uint32_t M = 0, C = 0;
  for (int rk = 0; rk < n_ranks; ++rk) {
    const uint64_t v = all[((size_t)rk * kXrPods + k) * kXrNorm + q];
    if (q == 0) {
      r = v > r ? v : r;
    } else {
      const uint32_t vm = (uint32_t)(v >> 32), vc = (uint32_t)v;
      C = vm > M ? vc : C + (vm == M ? vc : 0u);
      M = vm > M ? vm : M;
    }
  }
  norm[(size_t)k * kXrNorm + q] = q == 0 ? r : ((uint64_t)M << 32) | C;
}

// several ranks: the round-start values (val, val2, the NUMA affinity) of pod k on every candidate of the merged
// records that lies outside this rank's node range [lo, hi).  Block (k, j) = pod k on the kC entries of pod j's record,
// one per lane; a node listed by several records is evaluated once per record, each time to the same values.
template <int XF>
__global__ __launch_bounds__(kWave) void xr_fill(DevTable T, const RsvNode* __restrict__ RN,
                                                 const int32_t* __restrict__ rsv_n, const DevPod* __restrict__ pods,
                                                 const RsvPod* __restrict__ rpods, int64_t n, int64_t lo, int64_t hi,
                                                 int64_t stride, EvalParams P, RsvParams RP, RsvExt X,
                                                 const uint64_t* __restrict__ cand, uint64_t* __restrict__ val,
                                                 uint32_t* __restrict__ val2, uint32_t* __restrict__ affk,
                                                 const unsigned long long* __restrict__ ws) {
  int64_t first;
  int nb;
  if (!xr_range(ws, first, nb)) return;
  const int k = blockIdx.x / kXrPods, jr = blockIdx.x % kXrPods, lane = threadIdx.x;
  if (k >= nb || jr >= nb) return;
  const uint64_t key = cand[(size_t)jr * kCandStride + lane];
  if (key == 0) return;
  const int64_t i = (int64_t)key_node(key);
  if ((i >= lo && i < hi) || i >= n) return;
  const int64_t j = first + k;
  const DevPod p = pods[j];
  const RsvPod rp = rpods[j];
  const DsPod* dp = (XF & XF_DS) ? &X.dpods[j] : nullptr;
  const NumaPod* np = (XF & XF_NUMA) ? &X.npods[j] : nullptr;
  const int64_t* aux = (X.paux && (p.flags & P_AUX)) ? X.paux + (size_t)j * kAux : nullptr;
  const DefPod* df = (XF & XF_DEF) ? &X.defp[j] : nullptr;
  RsvExt Xk = X;
  Xk.aff = X.aff ? affk + (size_t)k * stride : nullptr;
  const RsvOut o = rsv_eval_node<false, false>(T, RN, rsv_n, i, p, rp, P, RP, Xk, dp, np, nullptr, aux, df);
  val[(size_t)k * stride + i] = o.feas ? rsv_pack(o) : 0;
  if (val2) val2[(size_t)k * stride + i] = o.feas ? (((uint32_t)o.tcnt << 24) | (uint32_t)o.asum) : 0u;
}

struct XrNorms {
  int64_t pref;             // the PreScore preferred node (-1 = none)
  int64_t mx, mds, mt, ma;  // the normalisation maxima rsv_total takes
};
__device__ __forceinline__ XrNorms xr_norms(const uint64_t* __restrict__ nk) {
  auto mval = [](uint64_t e) -> int64_t { return (e >> 32) ? (int64_t)(e >> 32) - 1 : 0; };
  XrNorms r;
  const uint64_t pk = nk[0];
  const int64_t mraw = mval(nk[1]);
  r.pref = pk ? (int64_t)(uint32_t)(~pk) : -1;
  r.mx = pk ? (mraw > 1000 ? mraw : 1000) : mraw;
  r.mds = mval(nk[2]);
  r.mt = mval(nk[3]);
  r.ma = mval(nk[4]);
  return r;
}

__global__ __launch_bounds__(kWave* kEvalWaves) void xr_select(const uint64_t* __restrict__ val,
                                                               const uint32_t* __restrict__ val2, int64_t n, int nt,
                                                               int tile_base, int64_t stride, int vbits, RsvParams RP, RsvExt X,
                                                               const uint64_t* __restrict__ norm,
                                                               uint64_t* __restrict__ lists,
                                                               const unsigned long long* __restrict__ ws) {
  int64_t first;
  int nb;
  if (!xr_range(ws, first, nb)) return;
  int tile, p0;
  xr_tile_coords(kXrPods / kXrPpw, tile, p0);
  if (tile >= nt || p0 >= nb) return;
  const int lane = threadIdx.x % kWave;
  const int p1 = p0 + kXrPpw < nb ? p0 + kXrPpw : nb;
  uint32_t gidx[kNPT];
#pragma unroll
  for (int q = 0; q < kNPT; ++q) gidx[q] = (uint32_t)((int64_t)(tile_base + tile) * kTile + q * kWave + lane);
  for (int k = p0; k < p1; ++k) {
    const XrNorms N = xr_norms(norm + (size_t)k * kXrNorm);
    uint32_t v[kNPT];
#pragma unroll
    for (int q = 0; q < kNPT; ++q) {
      const int64_t i = gidx[q];
      const uint64_t pv = i < n ? val[(size_t)k * stride + i] : 0;
      v[q] = 0;
      if (pv & (1ull << 7)) {
        const uint32_t pv2 = val2 ? val2[(size_t)k * stride + i] : 0u;
        v[q] = (uint32_t)rsv_total(pv, pv2, i == N.pref, N.mx, N.mds, N.mt, N.ma, RP, X) + 1u;
      }
    }
    select_write(v, gidx, vbits, lists + ((size_t)k * nt + tile) * kR, lane);
  }
}

constexpr int kRsvPodWords = (int)(sizeof(RsvPod) / 8), kDefPodWords = (int)((sizeof(DefPod) + 7) / 8);

// LDS bytes of xr_resolve: the records, the pods' staged per-plugin records, the quota rows, the modified bitmap
__host__ __device__ inline size_t xr_resolve_lds_bytes(int XF, int nq, bool aux, int bitmap_words) {
  size_t w = (size_t)kXrPods * (kC + 1) + (size_t)kXrPods * (kPodWords + kRsvPodWords);
  if (XF & XF_DS) w += (size_t)kXrPods * kDsPodWords;
  if (XF & XF_NUMA) w += (size_t)kXrPods * kNumaPodWords;
  if (XF & XF_DEF) w += (size_t)kXrPods * kDefPodWords;
  if (aux) w += (size_t)kXrPods * kAux;
  if (nq > 0) w += (size_t)nq * (sizeof(QuotaRow) / 8) + (size_t)kXrPods * kQuotaRes;
  return w * 8 + (size_t)bitmap_words * 4;
}

// Wave-cooperative Reserve of pod j on its winner row w (every lane calls it with the same w, v, j; `owner` holds row
// w): NodeNUMAResource Reserve on copies (owner lane), then DeviceShare's minor choice with one lane per minor —
// score and fit of minor m on lane m, the (score desc, minor asc) rank from the other lanes, the first `count` fitting
// minors taken (defaultAllocateDevices, device_allocator.go:384-454; sortDeviceResourcesByMinor,
// device_resources.go:187-208) and their deviceUsed updated by their lanes (updateCacheUsed, device_cache.go:124-135) —
// then the commits on the owner lane (NUMA NodeAllocation, NodeInfo + LoadAware assign cache, reservationCache
// assumePod).  The same Reserve as rsv_reserve, with the ~1.5 k-instruction per-minor scoring off the single lane.
template <bool NUMA, bool DS>
__device__ __forceinline__ bool xr_reserve(const DevTable& T, RsvNode* __restrict__ RN, int64_t w, uint64_t v,
                                           const DevPod& p, const RsvExt& X, int64_t j, int owner, int32_t& slot_out,
                                           int diag_j) {
  (void)diag_j;
  const int lane = threadIdx.x;
  slot_out = -1;
  KG_LANE_SUB(diag_j, 0);
  NumaMut nmw;
  CpuSet cpus = cs_zero();
  NumaAlloc rec;
  rec.res = 0;
  if (NUMA && X.ns) {
    // every lane runs the NUMA Reserve on the same row (uniform loads): scalar mask arithmetic (take_cpus)
    const NumaStatic nsw = X.ns[w];
    nmw = X.nm[w];
    const NumaView nv = make_view(&nsw, &nmw, X.NP);
    // X.aff[w] was stored by one lane (the owner's hand-off of pod j's affinity, or rsv_eval_node on a modified row)
    // and is read here by every lane: a workgroup-scope fence orders that store before these loads
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    const uint32_t a = X.aff[w];
    const NumaHint aff{a & 0xFFu, (int)((a >> 8) & 1u), 0, 0};
    const bool ok = numa_reserve(nsw, nmw, nv, X.npods[j], aff, cpus, rec);
    if (!ok) {
      if (lane == 0 && X.out_minors) X.out_minors[j] = 0;
      return false;
    }
  }
  KG_LANE_SUB(diag_j, 1);
  if (DS && X.ds) {
    const DsPod dp = X.dpods[j];
    const DsNode& d = X.ds[w];
    int32_t minors = 0;
    bool failed = false;
    if (!dp.skip && d.has_device) {
      const DsInst in = dp.error ? DsInst{0, 0, 0, 0, 0} : ds_instance(d, dp);
      bool f = false, nz = false;
      int64_t sc = 0;
      if (in.ok && lane < kMinors) sc = ds_minor(d, lane, in, X.DP, f, nz);
      const uint64_t anym = __ballot(nz), fitm = __ballot(f);
      failed = !in.ok || anym == 0 || __popcll(fitm) < in.count;
      if (!failed) {
        int rank = 0;
#pragma unroll
        for (int q = 0; q < kMinors; ++q) {
          const int64_t sq = (int64_t)readlane_u64((uint64_t)sc, q);
          rank += (((fitm >> q) & 1ull) != 0) && (sq > sc || (sq == sc && q < lane)) ? 1 : 0;
        }
        const uint64_t taken = __ballot(f && rank < in.count);
        if ((taken >> lane) & 1ull) {
          DsNode* dw = const_cast<DsNode*>(X.ds) + w;
          dw->ucore[lane] += (int32_t)in.core;
          dw->uratio[lane] += (int32_t)in.ratio;
          dw->umem[lane] += in.mem;
        }
        minors = (int32_t)taken;
      }
    }
    if (lane == 0) X.out_minors[j] = failed ? 0 : minors;
    if (failed) return false;
    __threadfence_block();  // the owner lane re-reads this row's deviceUsed for later pods
  }
  KG_LANE_SUB(diag_j, 2);
  int32_t slot = -1;
  if (lane == owner) {
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
    KG_LANE_SUB(diag_j, 4);
    slot = (int32_t)(v & 7) - 1;
    if (slot >= 0) {  // Allocated += quotav1.Mask(requests, ResourceNames): only the reservation's keys (0 = absent)
      if (RN[w].alloc_cpu[slot] > 0) RN[w].allocd_cpu[slot] += p.req_cpu;
      if (RN[w].alloc_mem[slot] > 0) RN[w].allocd_mem[slot] += p.req_mem;
      RN[w].assigned[slot] += 1;
    }
    KG_LANE_SUB(diag_j, 5);
  }
  slot_out = __builtin_amdgcn_readlane(slot, owner);
  return true;
}

// One wave: the round's FIFO replay (see the header).  Dynamic LDS: the pods' candidate records [nb][kC + 1], the
// round's pods and their per-plugin records (DevPod, RsvPod, DsPod, NumaPod, DefPod, aux requests), the ElasticQuota
// rows (admitted / charged in LDS, written back at the end) and the modified-node bitmap — one bulk load, so the
// per-pod chain touches global memory only for the modified rows and the Reserve.
template <int XF>
__global__ __launch_bounds__(kWave) void xr_resolve(DevTable T, RsvNode* __restrict__ RN,
                                                    const int32_t* __restrict__ rsv_n,
                                                    const DevPod* __restrict__ pods,
                                                    const RsvPod* __restrict__ rpods, int64_t stride,
                                                    EvalParams P, RsvParams RP, RsvExt X,
                                                    const uint64_t* __restrict__ val, const uint32_t* __restrict__ val2,
                                                    const uint32_t* __restrict__ affk,
                                                    const uint64_t* __restrict__ norm,
                                                    const uint64_t* __restrict__ cand, int bitmap_words,
                                                    uint64_t* __restrict__ out_keys, int32_t* __restrict__ out_slot,
                                                    unsigned long long* __restrict__ ws) {
  extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
  constexpr bool kNuma = (XF & XF_NUMA) != 0, kDs = (XF & XF_DS) != 0, kDef = (XF & XF_DEF) != 0;
  int64_t first;
  int nb;
  if (!xr_range(ws, first, nb)) return;
  const int lane = threadIdx.x;
  const int nq = X.nq;
  const bool has_aux = X.paux != nullptr;
  uint64_t* s_cand = smem;                                        // [kXrPods][kC + 1]
  uint64_t* s_podw = s_cand + (size_t)kXrPods * (kC + 1);         // [kXrPods][kPodWords]
  uint64_t* s_rpw = s_podw + (size_t)kXrPods * kPodWords;         // [kXrPods][kRsvPodWords]
  uint64_t* s_next = s_rpw + (size_t)kXrPods * kRsvPodWords;
  uint64_t* s_dpw = s_next;                                        // [kXrPods][kDsPodWords]      (DS)
  if (kDs) s_next += (size_t)kXrPods * kDsPodWords;
  uint64_t* s_npw = s_next;                                        // [kXrPods][kNumaPodWords]    (NUMA)
  if (kNuma) s_next += (size_t)kXrPods * kNumaPodWords;
  uint64_t* s_dfw = s_next;                                        // [kXrPods][kDefPodWords]     (defaults)
  if (kDef) s_next += (size_t)kXrPods * kDefPodWords;
  int64_t* s_aux = reinterpret_cast<int64_t*>(s_next);             // [kXrPods][kAux]             (aux requests)
  if (has_aux) s_next += (size_t)kXrPods * kAux;
  QuotaRow* s_q = reinterpret_cast<QuotaRow*>(s_next);             // [nq]
  int64_t* s_qdev = reinterpret_cast<int64_t*>(s_q + nq);          // [kXrPods][kQuotaRes]
  if (nq > 0) s_next += (size_t)nq * (sizeof(QuotaRow) / 8) + (size_t)kXrPods * kQuotaRes;
  uint32_t* bitmap = reinterpret_cast<uint32_t*>(s_next);
  {  // one bulk load of everything the per-pod chain reads
    for (int w = lane; w < nb * (kC + 1); w += kWave) s_cand[w] = cand[(size_t)(w / (kC + 1)) * kCandStride + w % (kC + 1)];
    auto stage = [&](uint64_t* dst, const void* src, int words) {
      const uint64_t* g = reinterpret_cast<const uint64_t*>(src);
      for (int w = lane; w < nb * words; w += kWave) dst[w] = g[(size_t)first * words + w];
    };
    stage(s_podw, pods, kPodWords);
    stage(s_rpw, rpods, kRsvPodWords);
    if (kDs) stage(s_dpw, X.dpods, kDsPodWords);
    if (kNuma) stage(s_npw, X.npods, kNumaPodWords);
    if (kDef) {  // DefPod (sizeof: 184 B since ABI 10): byte-exact copy of the nb records
      const uint32_t* g = reinterpret_cast<const uint32_t*>(X.defp + first);
      uint32_t* d = reinterpret_cast<uint32_t*>(s_dfw);
      constexpr int kW = (int)(sizeof(DefPod) / 4);
      for (int w = lane; w < nb * kW; w += kWave) d[(w / kW) * (kDefPodWords * 2) + w % kW] = g[w];
    }
    if (has_aux) {
      for (int w = lane; w < nb * kAux; w += kWave) s_aux[w] = X.paux[(size_t)first * kAux + w];
    }
    if (nq > 0) {
      const uint64_t* qw = reinterpret_cast<const uint64_t*>(X.quotas);
      uint64_t* sq = reinterpret_cast<uint64_t*>(s_q);
      for (int w = lane; w < nq * (int)(sizeof(QuotaRow) / 8); w += kWave) sq[w] = qw[w];
      for (int w = lane; w < nb * kQuotaRes; w += kWave) s_qdev[w] = X.qdev[(size_t)first * kQuotaRes + w];
    }
    for (int w = lane; w < bitmap_words; w += kWave) bitmap[w] = 0;
  }
  __syncthreads();
  const DevPod* s_pods = reinterpret_cast<const DevPod*>(s_podw);
  const RsvPod* s_rpods = reinterpret_cast<const RsvPod*>(s_rpw);
  uint32_t midx = 0xFFFFFFFFu;  // the modified row this lane owns
  int nM = 0, consumed = 0;
  const bool dscore = val2 != nullptr;
  for (int j = 0; j < nb; ++j) {
    KG_POD_DIAG(j, (uint32_t)nM);
    const int64_t jj = first + j;
    const DevPod p = s_pods[j];
    // the round-start values of this lane's modified row, issued before the pod's own evaluation
    uint64_t ov = 0;
    uint32_t ov2 = 0;
    if (lane < nM) {
      ov = val[(size_t)j * stride + midx];
      ov2 = dscore ? val2[(size_t)j * stride + midx] : 0u;
    }
    // ElasticQuota PreFilter against every earlier Reserve (lane 0 owns the LDS quota rows)
    int admit = 1;
    QuotaReq qr;
    if (nq > 0 && p.quota >= 0) {
      qr = quota_req(p, s_qdev + (size_t)j * kQuotaRes);
      if (lane == 0) admit = quota_row_admit(s_q[p.quota], qr, (p.flags & P_NONPREEMPT) != 0) ? 1 : 0;
      admit = __builtin_amdgcn_readfirstlane(admit);
    }
    if (!admit) {
      if (lane == 0) {
        out_keys[jj] = 0;
        out_slot[jj] = -1;
        if (X.out_minors) X.out_minors[jj] = 0;
      }
      ++consumed;
      continue;
    }
    // pod j on the modified rows: the exact current values, next to the round-start ones
    const RsvPod rp = s_rpods[j];
    const DsPod* dp = kDs ? reinterpret_cast<const DsPod*>(s_dpw + (size_t)j * kDsPodWords) : nullptr;
    const NumaPod* np = kNuma ? reinterpret_cast<const NumaPod*>(s_npw + (size_t)j * kNumaPodWords) : nullptr;
    const int64_t* aux = (has_aux && (p.flags & P_AUX)) ? s_aux + (size_t)j * kAux : nullptr;
    const DefPod* df = kDef ? reinterpret_cast<const DefPod*>(s_dfw + (size_t)j * kDefPodWords) : nullptr;
    RsvOut cur{false, 0, 0, -1, 0x7fffffff, 0, 0, 0};
    uint64_t cv = 0;
    uint32_t cv2 = 0;
    if (lane < nM) {
      cur = rsv_eval_node<true, false>(T, RN, rsv_n, midx, p, rp, P, RP, X, dp, np, nullptr, aux, df);  // X.aff[midx] = pod j's
      if (cur.feas) cv = rsv_pack(cur), cv2 = ((uint32_t)cur.tcnt << 24) | (uint32_t)cur.asum;
    }
    KG_POD_SUB(j, 0);
    const uint64_t* nk = norm + (size_t)j * kXrNorm;
    bool stop = false;
    if (nM > 0) {  // the normalisation of pod j must equal the round's (ballots only: no wave reductions)
      const bool of = (ov >> 7) & 1, cf = cur.feas;
      const uint32_t oval[4] = {(uint32_t)((ov >> 8) & 0xff), (uint32_t)((ov >> 16) & 0xff), ov2 >> 24, ov2 & 0xFFFFFFu};
      const uint32_t cval[4] = {(uint32_t)cur.raw, (uint32_t)cur.dsraw, (uint32_t)cur.tcnt, (uint32_t)cur.asum};
      const bool used[4] = {RP.score != 0, kDs && X.DP.score != 0, kDef && X.DF.taint_score != 0,
                            kDef && X.DF.aff_score != 0};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (!used[q]) continue;
        const uint32_t Menc = (uint32_t)(nk[1 + q] >> 32), C = (uint32_t)nk[1 + q];
        const uint32_t oe = (lane < nM && of) ? oval[q] + 1u : 0u, ce = (lane < nM && cf) ? cval[q] + 1u : 0u;
        const uint32_t lost = (uint32_t)__popcll(__ballot(oe != 0 && oe == Menc));
        // max over the modified rows > M, or every holder modified and none holds M any more
        if (__ballot(ce > Menc) || (lost >= C && !__ballot(ce == Menc))) stop = true;
      }
      if (RP.score) {  // the preferred node (smallest order label) must stay where it is, with the same order
        const uint64_t PK = nk[0];
        const uint64_t ck = (lane < nM && cf) ? rsv_pref_key(cur, midx) : 0ull;
        const uint32_t pn = (uint32_t)(~PK);
        const bool holder_mod = PK != 0 && ((bitmap[pn >> 5] >> (pn & 31)) & 1u);
        if (__ballot(ck > PK) || (holder_mod && !__ballot(ck == PK))) stop = true;
      }
    }
    if (stop) break;
    KG_POD_SUB(j, 1);
    const XrNorms N = xr_norms(nk);
    const uint64_t mkey = (lane < nM && cur.feas)
                              ? make_key(rsv_total(cv, cv2, (int64_t)midx == N.pref, N.mx, N.mds, N.mt, N.ma, RP, X), midx)
                              : 0ull;
    const uint64_t mbest = nM > 0 ? wave_max_key(mkey) : 0ull;
    const uint64_t key = lane < kC ? s_cand[(size_t)j * (kC + 1) + lane] : 0ull;
    const uint32_t kn = key_node(key);
    const bool unmod = key != 0 && !((bitmap[kn >> 5] >> (kn & 31)) & 1u);
    const uint64_t um = __ballot(unmod);
    uint64_t best = um ? readlane_u64(key, (int)__builtin_ctzll(um)) : 0ull;
    best = mbest > best ? mbest : best;
    if (best < s_cand[(size_t)j * (kC + 1) + kC]) break;  // an unlisted node could win
    ++consumed;
    if (best == 0) {
      if (lane == 0) {
        out_keys[jj] = 0;
        out_slot[jj] = -1;
        if (X.out_minors) X.out_minors[jj] = 0;
      }
      continue;
    }
    const uint32_t w = key_node(best);
    const uint64_t hit = __ballot(lane < nM && midx == w);
    const int owner = hit ? (int)__builtin_ctzll(hit) : nM;
    if (!hit) {
      if (lane == 0) bitmap[w >> 5] |= 1u << (w & 31);
      ++nM;
    }
    KG_POD_SUB(j, 2);
    uint64_t v = cv;
    if (lane == owner && !hit) {  // an unmodified winner: its round-start value, and its NUMA affinity for pod j
      midx = w;
      v = val[(size_t)j * stride + w];
      if (kNuma && X.aff) X.aff[w] = affk[(size_t)j * stride + w];
    }
    v = readlane_u64(v, owner);
    int32_t slot = -1;
    const bool placed = xr_reserve<kNuma, kDs>(T, RN, w, v, p, X, jj, owner, slot, j);
    KG_POD_SUB(j, 3);
    if (lane == 0) {
      out_keys[jj] = placed ? best : 0;
      out_slot[jj] = slot;
      if (placed && nq > 0 && p.quota >= 0) quota_row_charge(s_q[p.quota], qr, (p.flags & P_NONPREEMPT) != 0);
    }
    __syncthreads();
  }
  if (nq > 0) {  // the charged quota rows back to the table
    __syncthreads();
    const uint64_t* sq = reinterpret_cast<const uint64_t*>(s_q);
    uint64_t* qw = reinterpret_cast<uint64_t*>(X.quotas);
    for (int w = lane; w < nq * (int)(sizeof(QuotaRow) / 8); w += kWave) qw[w] = sq[w];
  }
  KG_POD_DIAG(consumed, 0u);
  __threadfence();
  if (lane == 0) {
    ws[3] = (unsigned long long)(first + consumed);
    ws[5] += 1;
    ws[6] += (unsigned long long)consumed;
  }
}
