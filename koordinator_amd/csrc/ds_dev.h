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
// Scope: GPU devices without hints, joint allocation, VFs, NUMA affinity, reservations or preemption;
// ScoringStrategy LeastAllocated or MostAllocated (the latter is not monotone: an assume raises the node's score,
// which the round resolver handles by re-scoring its modified rows for every pod and ending a round when one of them
// raises the normalization max).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

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

// DeviceShare preFilterState of one pod (host-decoded), 48 B (a 16-B multiple)
struct DsPod {
  int32_t skip, error, has_mem, pad;  // has_mem: the converted request names gpu-memory (else gpu-memory-ratio)
  int64_t core, mem, ratio, pad2;
};
static_assert(sizeof(DsPod) == 48, "DsPod layout");

struct DsParams {
  int32_t filter, score, weight;
  int32_t w_core, w_mem, w_ratio;  // ScoringStrategy.Resources weights
  int32_t most;                    // ScoringStrategy.Type MostAllocated (mostResourceScorer, scoring.go:281-304)
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

// DefaultNormalizeScore(MaxNodeScore, false) of one raw score given the max M over the feasible nodes
__device__ __forceinline__ int64_t ds_normalized(int64_t raw, uint32_t M) { return M ? div_small(100 * raw, M) : 0; }

}  // namespace kg
