// ds_dev.h — DeviceShare (GPU device type) on the device: per-(pod, node) Filter + raw Score for the wide passes
// and the resolver, and the winner's Reserve (minor selection + deviceUsed update).  Restates (paths under
// /root/reference/pkg/scheduler/plugins/deviceshare):
//   devicehandler_gpu.go:40-98   CalcDesiredRequestsAndCount, fillGPUTotalMem, memoryBytesToRatio/RatioToBytes
//   device_allocator.go:70-129   Prepare / Allocate;  :333-454 defaultAllocateDevices;  :499-522 score
//   device_cache.go:157-174      resetDeviceFree (free = SubtractWithNonNegativeResult(total, used));
//                :344-391        filter (a type whose free resources are all zero is dropped)
//   device_resources.go:164-208  scoreDevices + sortDeviceResourcesByMinor (score desc, minor asc)
//   scoring.go:183-279           scoreDevice / scoreNode / leastResourceScorer
// The pod's request is decoded on the host (GetPodDeviceRequests → ValidateDeviceRequest → ConvertDeviceRequest,
// utils.go:158-252); the per-node part (fillGPUTotalMem needs the node's GPU memory) runs here.
// Scope: GPU devices (and, ABI 17, the default handler's RDMA / FPGA types) without hints, joint allocation, VFs or NUMA
// affinity;
// ScoringStrategy LeastAllocated or MostAllocated (the latter is not monotone: an assume raises the node's score,
// which the round resolver handles by re-scoring its modified rows for every pod and ending a round when one of them
// raises the normalization max).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/koordgpu.h"
#include "kernels.h"

namespace kg {

constexpr int kMinors = 8;

// Device state of one node, 272 B (AoS: one node = 17 contiguous 16-B words).  Absent and unhealthy minors have
// zero totals (buildDeviceResources gives an unhealthy device an empty ResourceList, device_cache.go:513-515).
struct DsNode {
  int32_t tcore[kMinors], tratio[kMinors];  // deviceTotal: gpu-core, gpu-memory-ratio
  int32_t ucore[kMinors], uratio[kMinors];  // deviceUsed
  int64_t tmem[kMinors], umem[kMinors];     // gpu-memory bytes
  int32_t has_device;                        // a Device object exists for the node
  int32_t present;                           // bitmask of minors listed as GPU DeviceInfos
  int32_t first;                             // lowest minor with non-zero resources (fillGPUTotalMem), -1 none
  int32_t pad;
};
static_assert(sizeof(DsNode) == 272, "DsNode layout");

// (ABI 17) the default handler's device types (devicehandler_default.go): RDMA, FPGA — one percentage resource each
constexpr int kXTypes = KG_DEV_XTYPES;

// DeviceShare preFilterState of one pod (host-decoded), 48 B (a 16-B multiple).  skip = no device request at all
// (state.skip); nogpu = none of the GPU type (only RDMA / FPGA requests)
struct DsPod {
  int32_t skip, error, has_mem, nogpu;  // has_mem: the converted request names gpu-memory (else gpu-memory-ratio)
  int64_t core, mem, ratio;
  int32_t xq[kXTypes];                  // (ABI 17) koordinator.sh/rdma, koordinator.sh/fpga requests (0 = none)
};
static_assert(sizeof(DsPod) == 48, "DsPod layout");

// (ABI 17) the RDMA / FPGA devices of one node, 144 B: per type the minors listed as DeviceInfos, deviceTotal of the
// type's resource (0 for an unhealthy device: an empty ResourceList, device_cache.go:513-515) and deviceUsed
struct DsXNode {
  int32_t t[kXTypes][kMinors];
  int32_t u[kXTypes][kMinors];
  uint32_t listed[kXTypes];
  int32_t pad[2];
};
static_assert(sizeof(DsXNode) == 144, "DsXNode layout");

struct DsParams {
  int32_t filter, score, weight;
  int32_t w_core, w_mem, w_ratio;  // ScoringStrategy.Resources weights
  int32_t most;                    // ScoringStrategy.Type MostAllocated (mostResourceScorer, scoring.go:281-304)
  int32_t w_x[kXTypes];            // (ABI 17) koordinator.sh/rdma, koordinator.sh/fpga weights
  int32_t pad;
};

struct DsInst {
  int32_t ok, count;
  int64_t core, mem, ratio;
};

// CalcDesiredRequestsAndCount (devicehandler_gpu.go:40-66) + fillGPUTotalMem (:68-90)
__device__ __forceinline__ DsInst ds_instance(const DsNode& d, const DsPod& p) {
  DsInst in{0, 0, 0, 0, 0};
  if (!d.present || d.first < 0) return in;  // "Insufficient gpu devices" / "no healthy GPU Devices"
  int64_t tmem = 0;  // d.tmem[d.first] by selects: a dynamic index would send the whole row to scratch
#pragma unroll
  for (int m = 0; m < kMinors; ++m) tmem = m == d.first ? d.tmem[m] : tmem;
  int64_t core = p.core, mem = p.mem, ratio = p.ratio;
  if (p.has_mem) {
    // int64(float64(bytes)/float64(total)*100): IEEE division, then a separate multiply (-ffp-contract=off)
    const double q = (double)mem / (double)tmem;
    const double pc = q * 100.0;
    ratio = (int64_t)pc;
  } else {
    mem = ratio * tmem / 100;
  }
  in.count = 1;
  if (ratio > 100 && ratio % 100 == 0) {
    const int64_t n = ratio / 100;
    in.count = (int32_t)n;
    // x / n for 0 ≤ x < 2^52 and n ≥ 2: trunc of the correctly rounded f64 quotient is exact (a quotient just
    // below an integer k is ≤ k - 1/n, far more than an ulp below it), and avoids three 64-bit divide expansions
    auto qdiv = [](int64_t x, int64_t d) -> int64_t {
      return (x >= 0 && x < (1ll << 52)) ? (int64_t)((double)x / (double)d) : x / d;
    };
    core = qdiv(core, n);
    mem = qdiv(mem, n);
    ratio = qdiv(ratio, n);
  }
  in.ok = 1;
  in.core = core;
  in.mem = mem;
  in.ratio = ratio;
  return in;
}

__device__ __forceinline__ int64_t ds_sub0(int64_t a, int64_t b) { return a - b > 0 ? a - b : 0; }

// one resource term of least/mostResourceScorer over (total, free, request) (scoring.go:183-203, 254-304)
__device__ __forceinline__ void ds_term(int64_t w, int64_t total, int64_t free_, int64_t req, int64_t& num,
                                        int64_t& ws, bool most) {
  if (w == 0 || total == 0) return;
  const int64_t rq = total >= free_ ? total - free_ + req : total;
  num += (most ? most_requested64(rq, total) : least_requested(rq, total)) * w;
  ws += w;
}

// Filter (AutopilotAllocator.Allocate feasibility) and, when feasible, the raw Score (scoreNode over every listed
// minor).  A node without a Device object rejects device pods (NodeResourcesFit on the device resources).
__device__ __forceinline__ bool ds_eval(const DsNode& d, const DsPod& p, const DsParams& P, int64_t& raw) {
  raw = 0;
  if (p.skip) return true;
  if (p.error || !d.has_device) return false;
  if (p.nogpu) return true;  // (ABI 17) no GPU-type request: the GPU part allocates nothing
  const DsInst in = ds_instance(d, p);
  if (!in.ok) return false;
  int nfit = 0;
  bool any = false;
  int64_t Tc = 0, Tm = 0, Tr = 0, Fc = 0, Fm = 0, Fr = 0;
#pragma unroll
  for (int m = 0; m < kMinors; ++m) {
    const int64_t fc = ds_sub0(d.tcore[m], d.ucore[m]);
    const int64_t fr = ds_sub0(d.tratio[m], d.uratio[m]);
    const int64_t fm = ds_sub0(d.tmem[m], d.umem[m]);
    const bool nz = (fc | fr | fm) != 0;
    any |= nz;
    nfit += (nz && in.core <= fc && in.mem <= fm && in.ratio <= fr) ? 1 : 0;
    Tc += d.tcore[m];
    Tr += d.tratio[m];
    Tm += d.tmem[m];
    Fc += fc;
    Fr += fr;
    Fm += fm;
    // half the minors consumed before the other half is loaded (the accumulators pass through an opaque asm with a
    // memory clobber): xr_eval<DeviceShare> 214 → 164 VGPRs, a third wave per SIMD
    if (m == kMinors / 2 - 1)
      asm volatile("" : "+v"(Tc), "+v"(Tr), "+v"(Tm), "+v"(Fc), "+v"(Fr), "+v"(Fm), "+v"(nfit) : : "memory");
  }
  if (!any || nfit < in.count) return false;
  int64_t num = 0, ws = 0;
  const bool most = P.most != 0;
  ds_term(P.w_core, Tc, Fc, in.core, num, ws, most);
  ds_term(P.w_mem, Tm, Fm, in.mem, num, ws, most);
  ds_term(P.w_ratio, Tr, Fr, in.ratio, num, ws, most);
  raw = ws ? div_small(num, ws) : 0;
  return true;
}

// scoreDevice of one minor (scoring.go:183-203) and whether the per-instance request fits it
// (defaultAllocateDevices: skip a minor whose free resources are all zero, then LessThanOrEqual(request, free),
// device_allocator.go:412-421).  Reserve takes the first `count` fitting minors in (score desc, minor asc) order.
__device__ __forceinline__ int64_t ds_minor(const DsNode& d, int m, const DsInst& in, const DsParams& P, bool& fits,
                                            bool& nonzero) {
  const int64_t fc = ds_sub0(d.tcore[m], d.ucore[m]);
  const int64_t fr = ds_sub0(d.tratio[m], d.uratio[m]);
  const int64_t fm = ds_sub0(d.tmem[m], d.umem[m]);
  nonzero = (fc | fr | fm) != 0;
  fits = nonzero && ((d.present >> m) & 1) && in.core <= fc && in.mem <= fm && in.ratio <= fr;
  int64_t num = 0, ws = 0;
  const bool most = P.most != 0;
  ds_term(P.w_core, d.tcore[m], fc, in.core, num, ws, most);
  ds_term(P.w_mem, d.tmem[m], fm, in.mem, num, ws, most);
  ds_term(P.w_ratio, d.tratio[m], fr, in.ratio, num, ws, most);
  return ws ? div_small(num, ws) : 0;
}

// ---- (ABI 17) RDMA / FPGA: DefaultDeviceHandler (devicehandler_default.go:45-92) without hints ---------------------
// CalcDesiredRequestsAndCount: q > 100 and a multiple of 100 → q / 100 instances of 100, else one instance of q
__device__ __forceinline__ void dsx_inst(int32_t q, int32_t& count, int32_t& per) {
  const bool multi = q > 100 && q % 100 == 0;
  count = multi ? q / 100 : 1;
  per = multi ? 100 : q;
}
// scoreDevice / scoreNode of the type's one resource (scoring.go:183-243): the other weights see a zero total, so the
// weighted mean is the resource's own score when its weight is set, 0 otherwise
__device__ __forceinline__ int64_t dsx_term(int32_t w, int64_t total, int64_t free_, int64_t req, bool most) {
  if (w == 0 || total == 0) return 0;
  const int64_t rq = total >= free_ ? total - free_ + req : total;
  return most ? most_requested64(rq, total) : least_requested(rq, total);
}

// Filter and raw Score of the pod's RDMA / FPGA requests on one node (Allocate feasibility per requested type:
// "Insufficient %s devices" without listed minors of the type; nodeDevice.filter drops a type whose free resources are
// all zero; defaultAllocateDevices needs `count` minors with a non-zero free ≥ the per-instance request), the raw Score
// summed over the types (AutopilotAllocator.score, device_allocator.go:499-522).  pre = the type's preemptible
// amounts per minor (calcFreeWithPreemptible), nullptr = none.
__device__ __forceinline__ bool ds_eval_x(const DsXNode& x, bool has_device, const DsPod& p, const DsParams& P,
                                          int64_t& raw, const int32_t (*pre)[kMinors] = nullptr) {
  raw = 0;
  if (p.skip) return true;
  if (p.error) return false;
#pragma unroll
  for (int t = 0; t < kXTypes; ++t) {
    if (p.xq[t] == 0) continue;
    if (!has_device || x.listed[t] == 0) return false;
    int32_t count, per;
    dsx_inst(p.xq[t], count, per);
    int nfit = 0;
    bool any = false;
    int64_t T = 0, F = 0;
#pragma unroll
    for (int m = 0; m < kMinors; ++m) {
      if (!((x.listed[t] >> m) & 1u)) continue;
      const int64_t u = pre ? ds_sub0(x.u[t][m], pre[t][m]) : x.u[t][m];
      const int64_t f = ds_sub0(x.t[t][m], u);
      any |= f != 0;
      nfit += (f != 0 && per <= f) ? 1 : 0;
      T += x.t[t][m];
      F += f;
    }
    if (!any || nfit < count) return false;
    raw += dsx_term(P.w_x[t], T, F, per, P.most != 0);
  }
  return true;
}

// Reserve of the pod's RDMA / FPGA requests (one thread): per type the first `count` fitting minors in (scoreDevice
// desc, minor asc) order (device_allocator.go:384-454, device_resources.go:164-208), deviceUsed += the per-instance
// request.  Returns the masks packed as type t → bits 8·(t + 1) .. 8·(t + 1) + 7 (the GPU mask's byte is 0), -1 when a
// type cannot be allocated (nothing is written then).
__device__ __forceinline__ int32_t ds_reserve_x(DsXNode& x, bool has_device, const DsPod& p, const DsParams& P) {
  if (p.skip || !has_device) return 0;
  if (p.error) return -1;
  int32_t out = 0;
  uint32_t taken[kXTypes] = {0u, 0u};
#pragma unroll
  for (int t = 0; t < kXTypes; ++t) {
    if (p.xq[t] == 0) continue;
    if (x.listed[t] == 0) return -1;
    int32_t count, per;
    dsx_inst(p.xq[t], count, per);
    int64_t sc[kMinors];
    uint32_t fit = 0;
    bool any = false;
#pragma unroll
    for (int m = 0; m < kMinors; ++m) {
      sc[m] = 0;
      if (!((x.listed[t] >> m) & 1u)) continue;
      const int64_t f = ds_sub0(x.t[t][m], x.u[t][m]);
      any |= f != 0;
      fit |= (f != 0 && per <= f) ? (1u << m) : 0u;
      sc[m] = dsx_term(P.w_x[t], x.t[t][m], f, per, P.most != 0);
    }
    if (!any || __popc(fit) < count) return -1;
    for (int k = 0; k < count; ++k) {
      int best = -1;
#pragma unroll
      for (int m = 0; m < kMinors; ++m)
        if (((fit & ~taken[t]) >> m) & 1u)
          if (best < 0 || sc[m] > sc[best]) best = m;
      taken[t] |= 1u << best;
    }
    out |= (int32_t)(taken[t] << (8 * (t + 1)));
  }
#pragma unroll
  for (int t = 0; t < kXTypes; ++t) {
    if (!taken[t]) continue;
    int32_t count, per;
    dsx_inst(p.xq[t], count, per);
#pragma unroll
    for (int m = 0; m < kMinors; ++m)
      if ((taken[t] >> m) & 1u) x.u[t][m] += per;
  }
  return out;
}

// Unreserve of the RDMA / FPGA part of a packed minor record (updateDeviceUsed(add = false): non-negative subtract)
__device__ __forceinline__ void ds_release_x(DsXNode& x, const DsPod& p, int32_t packed) {
#pragma unroll
  for (int t = 0; t < kXTypes; ++t) {
    const uint32_t mk = ((uint32_t)packed >> (8 * (t + 1))) & 0xFFu;
    if (!mk || p.xq[t] == 0) continue;
    int32_t count, per;
    dsx_inst(p.xq[t], count, per);
#pragma unroll
    for (int m = 0; m < kMinors; ++m)
      if ((mk >> m) & 1u) x.u[t][m] = x.u[t][m] - per > 0 ? x.u[t][m] - per : 0;
  }
}

// DefaultNormalizeScore(MaxNodeScore, false) of one raw score given the max M over the feasible nodes
__device__ __forceinline__ int64_t ds_normalized(int64_t raw, uint32_t M) { return M ? div_small(100 * raw, M) : 0; }

}  // namespace kg
