// Microbenchmark (r6, diagnostic only): the latency of the NUMA resolver's two serial steps on one wave, on C4 rows.
//   eval:    every lane l < R evaluates numa_eval(row l, pod j) (the resolver's re-score of its modified rows)
//   reserve: numa_reserve of pod j on row j % R, wave-uniform (the resolver's Reserve), on a copy of the row
//   view:    make_view of row j % R on one lane (the resolver's view rebuild after a Reserve)
// s_memtime cycles per pod; the results (score, affinity, cpus) are written out so two builds of numa_dev.h can be
// compared bit for bit.  Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC -I<dir of numa_dev.h> numa_eval.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>

#include "koordgpu.h"
#include "numa_dev.h"

using namespace kg;

__device__ __forceinline__ uint64_t clk() {
  uint64_t t = __builtin_amdgcn_s_memtime();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  return t;
}

// MODE: 0 numa_eval + numa_reserve; eval part only: 1 numa_admit, 2 numa_filter, 3 numa_score (nil affinity);
// reserve part only: 4 numa_feasible, 5 the take_cpus of numa_reserve (over the row's available cpus)
template <int MODE>
__global__ __launch_bounds__(64) void k_numa(const NumaStatic* __restrict__ S, const NumaMut* __restrict__ M,
                                             const int64_t* __restrict__ nr, int R, const NumaPod* __restrict__ pods,
                                             int P, NumaParams NP, uint64_t* __restrict__ cyc, int64_t* __restrict__ res,
                                             uint64_t* __restrict__ cpus_out) {
  __shared__ NumaStatic s_s[64];
  __shared__ NumaMut s_m[64];
  const int lane = threadIdx.x;
  if (lane < R) {
    s_s[lane] = S[lane];
    s_m[lane] = M[lane];
  }
  __syncthreads();
  NumaView v;
  int64_t rc = 0, rm = 0, ac = 0, am = 0;
  if (lane < R) {
    v = make_view(&s_s[lane], &s_m[lane], NP);
    rc = nr[lane * 4], rm = nr[lane * 4 + 1], ac = nr[lane * 4 + 2], am = nr[lane * 4 + 3];
  }
  for (int j = 0; j < P; ++j) {
    const NumaPod p = pods[j];
    // eval
    const uint64_t t0 = clk();
    int64_t sc = 0;
    NumaHint aff{0, 1, 0, 0};
    bool ok = false;
    if (lane < R) {
      if (MODE == 1) {
        NumaHint b;
        ok = v.policy != 0 && v.nn > 0 ? numa_admit(v, p, NP, b) : true;
        aff = b;
      } else if (MODE == 2) {
        ok = numa_filter(v, p, NP, aff, rc, ac);
      } else if (MODE == 3) {
        sc = numa_score(v, p, NP, aff, rc, rm, ac, am);
        ok = true;
      } else if (MODE == 0) {
        ok = numa_eval(v, p, NP, rc, rm, ac, am, sc, aff);
      } else {
        ok = numa_filter(v, p, NP, aff, rc, ac);
      }
    }
    const uint64_t bm = __ballot(ok);
    asm volatile("" ::"s"(bm));
    const uint64_t t1 = clk();
    if (lane < R) {
      res[((size_t)j * 64 + lane) * 2] = ok ? sc : -1;
      res[((size_t)j * 64 + lane) * 2 + 1] = (int64_t)aff.mask | ((int64_t)aff.nil << 8) | ((int64_t)aff.preferred << 9) |
                                             ((int64_t)aff.score << 16);
    }
    // reserve, wave-uniform, on row w (the affinity Filter stored there)
    const int w = j % R;
    const NumaHint a{(uint32_t)__builtin_amdgcn_readlane((int)aff.mask, w), __builtin_amdgcn_readlane(aff.nil, w),
                     __builtin_amdgcn_readlane(aff.preferred, w), __builtin_amdgcn_readlane(aff.score, w)};
    const int okw = __builtin_amdgcn_readlane(ok ? 1 : 0, w);
    NumaView ov;
    {
      constexpr int kVw = (int)(sizeof(NumaView) / 4);
      uint32_t vw[kVw];
      __builtin_memcpy(vw, &v, sizeof(v));
#pragma unroll
      for (int q = 0; q < kVw; ++q) vw[q] = (uint32_t)__builtin_amdgcn_readlane((int)vw[q], w);
      __builtin_memcpy(&ov, vw, sizeof(ov));
    }
    const NumaStatic ns = s_s[w];
    NumaMut nm = s_m[w];
    const uint64_t t2 = clk();
    CpuSet cpus = cs_zero();
    NumaAlloc rec;
    int placed = 0;
    if (okw) {
      if (MODE == 4) {
        placed = numa_feasible(ov, p, a, rec) ? 1 : 0;
      } else if (MODE == 5) {
        const Topo t = make_topo(ns);
        const int bind = numa_pref_bind(ov, p.preferred);
        CpuSet avail = numa_available_cpus(t, ns, nm);
        if (p.required != 0) avail = filter_required(t, avail, bind);
        placed = p.cpu_bind && bind >= 0 && take_cpus(t, avail, p.needed, bind, ov.strategy, cpus, p.excl, cs_zero());
      } else {
        placed = numa_reserve(ns, nm, ov, p, a, cpus, rec) ? 1 : 0;
      }
    }
    asm volatile("" ::"s"(placed));
    const uint64_t t3 = clk();
    // view rebuild of the reserved row (lane w)
    if (lane == w) {
      const NumaView nv = make_view(&s_s[w], &nm, NP);
      rc += nv.tot[0];  // keep it live
    }
    const uint64_t t4 = clk();
    if (lane == 0) {
      cyc[(size_t)j * 3] = t1 - t0;
      cyc[(size_t)j * 3 + 1] = okw ? t3 - t2 : 0;
      cyc[(size_t)j * 3 + 2] = t4 - t3;
#pragma unroll
      for (int q = 0; q < kCpuWords; ++q) cpus_out[(size_t)j * 5 + q] = cpus.w[q];
      cpus_out[(size_t)j * 5 + 4] = (uint64_t)placed | ((uint64_t)okw << 1);
    }
  }
  if (lane < R) res[((size_t)P * 64 + lane) * 2] = rc;  // keep the view rebuilds live
}

// MODE 6 / 7: interference of two waves in one workgroup (blockDim 128 / 256): wave 0 evaluates the R rows as k_numa
// MODE 0's eval, the second wave (wave 1 for 6, wave 2 for 7) evaluates row 0 wave-uniformly at the same time; each
// wave's cycles per pod go to cyc[j*3] (wave 0) and cyc[j*3+1] (second wave)
template <int MODE>
__global__ __launch_bounds__(256) void k_pair(const NumaStatic* __restrict__ S, const NumaMut* __restrict__ M,
                                              const int64_t* __restrict__ nr, int R, const NumaPod* __restrict__ pods,
                                              int P, NumaParams NP, uint64_t* __restrict__ cyc,
                                              int64_t* __restrict__ res) {
  __shared__ NumaStatic s_s[64];
  __shared__ NumaMut s_m[64];
  const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
  const int second = MODE == 6 ? 1 : 2;
  if (threadIdx.x < R) {
    s_s[threadIdx.x] = S[threadIdx.x];
    s_m[threadIdx.x] = M[threadIdx.x];
  }
  __syncthreads();
  const int row = wave == 0 ? lane : 0;
  const bool act = (wave == 0 && lane < R) || wave == second;
  NumaView v;
  int64_t rc = 0, rm = 0, ac = 0, am = 0;
  if (act) {
    v = make_view(&s_s[row], &s_m[row], NP);
    rc = nr[row * 4], rm = nr[row * 4 + 1], ac = nr[row * 4 + 2], am = nr[row * 4 + 3];
  }
  int64_t acc = 0;
  for (int j = 0; j < P; ++j) {
    __syncthreads();
    if (wave != 0 && wave != second) continue;
    const NumaPod p = pods[j];
    const uint64_t t0 = clk();
    int64_t sc = 0;
    NumaHint aff{0, 1, 0, 0};
    bool ok = false;
    if (act) ok = numa_eval(v, p, NP, rc, rm, ac, am, sc, aff);
    const uint64_t bm = __ballot(ok);
    asm volatile("" ::"s"(bm));
    const uint64_t t1 = clk();
    acc += sc + aff.mask;
    if (lane == 0) cyc[(size_t)j * 3 + (wave == 0 ? 0 : 1)] = t1 - t0;
  }
  if (act) res[threadIdx.x] = acc;
}

static int decode_pod(const kg_pod& p, int default_bind, NumaPod& d) {
  std::memset(&d, 0, sizeof(d));
  d.req_cpu = p.requests[KG_RES_CPU];
  d.req_mem = p.requests[KG_RES_MEMORY];
  d.allow = (p.qos == KG_QOS_LSE || p.qos == KG_QOS_LSR) && p.priority_class == KG_PRIO_PROD;
  bool zero = true;
  for (int r = 0; r < KG_RES_MAX; ++r) zero &= p.requests[r] == 0;
  if (zero) {
    d.skip = 1;
    return 0;
  }
  if (!d.allow) return 0;
  int bind = (int)p.preferred_cpu_bind_policy;
  if (bind == KG_BIND_NONE || bind == KG_BIND_DEFAULT) bind = default_bind;
  int required = (int)p.required_cpu_bind_policy;
  if (required == KG_BIND_DEFAULT) required = default_bind;
  if (required != KG_BIND_NONE) bind = required;
  if (bind == KG_BIND_FULL_PCPUS || bind == KG_BIND_SPREAD_BY_PCPUS) {
    if (d.req_cpu % 1000 != 0) {
      d.prefilter_error = 1;
      return 0;
    }
    if (d.req_cpu > 0) {
      d.cpu_bind = 1;
      d.required = required;
      d.preferred = bind;
      d.needed = (int32_t)(d.req_cpu / 1000);
      d.excl = (int32_t)p.preferred_cpu_exclusive_policy;
    }
  }
  return 0;
}

static void decode_node(const kg_node_numa& n, NumaStatic& s, NumaMut& m) {
  std::memset(&s, 0, sizeof(s));
  std::memset(&m, 0, sizeof(m));
  if (n.has_topology) {
    s.sockets = (int32_t)n.sockets;
    s.nps = (int32_t)n.nodes_per_socket;
    s.cpn = (int32_t)n.cores_per_node;
    s.cpc = (int32_t)n.cpus_per_core;
    s.valid = n.sockets * n.nodes_per_socket * n.cores_per_node * n.cpus_per_core > 0;
  }
  s.policy = (int32_t)n.numa_policy;
  s.node_bind = (int32_t)n.node_cpu_bind_policy;
  s.strategy = (int32_t)n.numa_allocate_strategy;
  s.num_numa = (int32_t)n.num_numa;
  for (int i = 0; i < KG_MAX_NUMA; ++i) {
    s.numa_cpu[i] = i < n.num_numa ? n.numa_cpu[i] : 0;
    s.numa_mem[i] = i < n.num_numa ? n.numa_mem[i] : 0;
    m.alloc_cpu[i] = i < n.num_numa ? n.numa_alloc_cpu[i] : 0;
    m.alloc_mem[i] = i < n.num_numa ? n.numa_alloc_mem[i] : 0;
    if (m.alloc_cpu[i] != 0 || m.alloc_mem[i] != 0) m.present |= 1u << i;
  }
  s.cpu_amp = n.cpu_amplification_ratio;
  for (int w = 0; w < KG_MAX_CPUS / 64; ++w) {
    s.reserved[w] = n.reserved_cpus[w];
    m.allocated[w] = n.allocated_cpus[w];
    m.excl_pcpu[w] = n.exclusive_pcpu_cpus[w] & n.allocated_cpus[w];
    m.excl_numa[w] = n.exclusive_numa_cpus[w] & n.allocated_cpus[w];
  }
}

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
      return 1;                                                                \
    }                                                                          \
  } while (0)

// np: filter, score, weight, node_strategy, numa_strategy, w_cpu, w_mem, nw_cpu, nw_mem, default_alloc_strategy
extern "C" int micro_numa(const kg_node_numa* nodes, const int64_t* node_req, int R, const kg_pod* pods, int P,
                          const int32_t* np, int default_bind, uint64_t* cyc, int64_t* res, uint64_t* cpus, int mode) {
  if (R < 1 || R > 64 || P < 1) return 2;
  std::vector<NumaStatic> hs(R);
  std::vector<NumaMut> hm(R);
  std::vector<NumaPod> hp(P);
  for (int i = 0; i < R; ++i) decode_node(nodes[i], hs[i], hm[i]);
  for (int j = 0; j < P; ++j) decode_pod(pods[j], default_bind, hp[j]);
  NumaParams NP;
  std::memcpy(&NP, np, sizeof(NP));
  NumaStatic* dS;
  NumaMut* dM;
  NumaPod* dP;
  int64_t *dR, *dRes;
  uint64_t *dC, *dCp;
  CK(hipMalloc(&dS, sizeof(NumaStatic) * R));
  CK(hipMalloc(&dM, sizeof(NumaMut) * R));
  CK(hipMalloc(&dP, sizeof(NumaPod) * P));
  CK(hipMalloc(&dR, sizeof(int64_t) * 4 * R));
  CK(hipMalloc(&dRes, sizeof(int64_t) * 2 * 64 * (P + 1)));
  CK(hipMalloc(&dC, sizeof(uint64_t) * 3 * P));
  CK(hipMalloc(&dCp, sizeof(uint64_t) * 5 * P));
  CK(hipMemcpy(dS, hs.data(), sizeof(NumaStatic) * R, hipMemcpyHostToDevice));
  CK(hipMemcpy(dM, hm.data(), sizeof(NumaMut) * R, hipMemcpyHostToDevice));
  CK(hipMemcpy(dP, hp.data(), sizeof(NumaPod) * P, hipMemcpyHostToDevice));
  CK(hipMemcpy(dR, node_req, sizeof(int64_t) * 4 * R, hipMemcpyHostToDevice));
  CK(hipMemset(dRes, 0, sizeof(int64_t) * 2 * 64 * (P + 1)));
  for (int rep = 0; rep < 2; ++rep) {  // the first launch warms the instruction cache
#define KG_MICRO(m) k_numa<m><<<1, 64>>>(dS, dM, dR, R, dP, P, NP, dC, dRes, dCp)
    switch (mode) {
      case 1: KG_MICRO(1); break;
      case 2: KG_MICRO(2); break;
      case 3: KG_MICRO(3); break;
      case 4: KG_MICRO(4); break;
      case 5: KG_MICRO(5); break;
      case 6: k_pair<6><<<1, 128>>>(dS, dM, dR, R, dP, P, NP, dC, dRes); break;
      case 7: k_pair<7><<<1, 256>>>(dS, dM, dR, R, dP, P, NP, dC, dRes); break;
      default: KG_MICRO(0); break;
    }
#undef KG_MICRO
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
  }
  CK(hipMemcpy(cyc, dC, sizeof(uint64_t) * 3 * P, hipMemcpyDeviceToHost));
  CK(hipMemcpy(res, dRes, sizeof(int64_t) * 2 * 64 * P, hipMemcpyDeviceToHost));
  CK(hipMemcpy(cpus, dCp, sizeof(uint64_t) * 5 * P, hipMemcpyDeviceToHost));
  (void)hipFree(dS), (void)hipFree(dM), (void)hipFree(dP), (void)hipFree(dR), (void)hipFree(dRes), (void)hipFree(dC),
      (void)hipFree(dCp);
  return 0;
}
