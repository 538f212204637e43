// numa_dev.h — NodeNUMAResource on the device: per-(pod, node) Filter + Score (topology hints, topology-manager
// merge, Allocate feasibility) for the wide pass and the resolver, and the winner's Reserve (exact cpuset via
// the cpu accumulator) for the resolver.  Restates (paths under /root/reference/pkg/scheduler):
//   plugins/nodenumaresource/plugin.go        Filter :276-334, Reserve :375-415, getPreferredCPUBindPolicy :556-576
//   plugins/nodenumaresource/scoring.go       Score :55-120, calculateAllocatableAndRequested :122-168
//   plugins/nodenumaresource/resource_manager.go  hints :122-169/:418-532, Allocate :171-360, required :534-589
//   plugins/nodenumaresource/node_allocation.go   getAvailableCPUs :133-153, NUMA resources :155-177
//   plugins/nodenumaresource/cpu_accumulator.go   takeCPUs :87-232 and the sorted free lists :371-822
//   frameworkext/topologymanager/policy*.go   mergeFilteredHints + best-effort / restricted / single-numa-node
// CPU sets are 256-bit masks in buildCPUTopology numbering (cpu = ((socket·nps + node)·cpn + core)·cpc + t), so a
// NUMA node, a socket and a core are contiguous cpu ranges.  Scope: ≤ 4 NUMA nodes, cpus per core 1 or 2,
// maxRefCount 1; cpu amplification and exclusive policies included.  (r6) Reservations that hold cpusets
// (nodenumaresource/reservation.go, plugin.go:465-535): a pod nominated into one gets its reserved cpus as
// preferredCPUs at Score and Reserve (numa_alloc_pref / numa_score_pref / numa_reserve_pref below).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

namespace kg {

constexpr int kNumaMax = 4;
constexpr int kCpuWords = 4;

// static per-node NUMA data (ingest), 144 B
struct NumaStatic {
  uint64_t reserved[kCpuWords];
  int64_t numa_cpu[kNumaMax], numa_mem[kNumaMax];
  int32_t sockets, nps, cpn, cpc;  // topology (0 sockets = none)
  int32_t valid;                   // CPUTopology present and IsValid()
  int32_t policy;                  // KG_NUMA_POLICY_*
  int32_t node_bind;               // KG_NODE_BIND_*
  int32_t strategy;                // -1 = plugin default, else KG_STRATEGY_*
  int32_t num_numa;
  int32_t pad;
  double cpu_amp;                  // cpu amplification ratio (≤ 1 = none)
};
static_assert(sizeof(NumaStatic) == 144, "NumaStatic layout");

// mutable per-node NUMA state (NodeAllocation)
struct NumaMut {
  uint64_t allocated[kCpuWords];
  int64_t alloc_cpu[kNumaMax], alloc_mem[kNumaMax];
  uint32_t present;  // bit i: allocatedResources[i] exists (an allocation ever landed on NUMA node i)
  uint32_t pad;
  // allocated cpus whose CPUInfo.ExclusivePolicy is PCPULevel / NUMANodeLevel (read by Reserve only; past the
  // fields Filter / Score read, so the wide pass touches the same lines as without them)
  uint64_t excl_pcpu[kCpuWords], excl_numa[kCpuWords];
};
static_assert(sizeof(NumaMut) == 168, "NumaMut layout");

// extension.Amplify (apis/extension/node_resource_amplification.go:170-175): ceil in float64, as Go
__device__ __forceinline__ int64_t amplify(int64_t origin, double ratio) {
  return ratio > 1.0 ? (int64_t)__builtin_ceil((double)origin * ratio) : origin;
}

// per-pod NodeNUMAResource preFilterState (decoded on the host: plugin.go:220-270)
struct NumaPod {
  int64_t req_cpu, req_mem;
  int32_t skip, prefilter_error, cpu_bind, required;  // required/preferred: KG_BIND_*
  int32_t preferred, needed;
  int32_t excl;  // preferredCPUExclusivePolicy (KG_EXCL_*)
  int32_t allow;  // (r6) AllowUseCPUSet (util.go:42-49): RestoreReservation restores reserved cpus only for such pods
};
static_assert(sizeof(NumaPod) == 48, "NumaPod layout");

struct NumaParams {
  int32_t filter, score, weight;
  int32_t node_strategy, numa_strategy;  // ScoringStrategy / NUMAScoringStrategy types
  int32_t w_cpu, w_mem, nw_cpu, nw_mem;
  int32_t default_alloc_strategy;
};

struct CpuSet {
  uint64_t w[kCpuWords];
};

__device__ __forceinline__ CpuSet cs_zero() { return CpuSet{{0, 0, 0, 0}}; }
__device__ __forceinline__ int cs_count(const CpuSet& s) {
  return __popcll(s.w[0]) + __popcll(s.w[1]) + __popcll(s.w[2]) + __popcll(s.w[3]);
}
__device__ __forceinline__ bool cs_has(const CpuSet& s, int c) { return (s.w[c >> 6] >> (c & 63)) & 1ull; }
__device__ __forceinline__ void cs_set(CpuSet& s, int c) { s.w[c >> 6] |= 1ull << (c & 63); }
__device__ __forceinline__ void cs_clr(CpuSet& s, int c) { s.w[c >> 6] &= ~(1ull << (c & 63)); }
// cpus [lo, hi)
__device__ __forceinline__ CpuSet cs_range(int lo, int hi) {
  CpuSet s;
#pragma unroll
  for (int w = 0; w < kCpuWords; ++w) {
    const int a = lo - 64 * w, b = hi - 64 * w;
    const uint64_t hiMask = b >= 64 ? ~0ull : (b <= 0 ? 0ull : ((1ull << b) - 1));
    const uint64_t loMask = a <= 0 ? ~0ull : (a >= 64 ? 0ull : ~((1ull << a) - 1));
    s.w[w] = hiMask & loMask;
  }
  return s;
}
__device__ __forceinline__ CpuSet cs_and(CpuSet a, const CpuSet& b) {
#pragma unroll
  for (int w = 0; w < kCpuWords; ++w) a.w[w] &= b.w[w];
  return a;
}
__device__ __forceinline__ CpuSet cs_andnot(CpuSet a, const CpuSet& b) {
#pragma unroll
  for (int w = 0; w < kCpuWords; ++w) a.w[w] &= ~b.w[w];
  return a;
}
__device__ __forceinline__ CpuSet cs_or(CpuSet a, const CpuSet& b) {
#pragma unroll
  for (int w = 0; w < kCpuWords; ++w) a.w[w] |= b.w[w];
  return a;
}

struct Topo {
  int sockets, nps, cpn, cpc, nodes, cores, cpus;
  __device__ int core_of(int c) const { return c / cpc; }
  __device__ int node_of(int c) const { return c / (cpc * cpn); }
  __device__ int socket_of(int c) const { return c / (cpc * cpn * nps); }
  __device__ int per_node() const { return cpc * cpn; }
  __device__ int per_socket() const { return cpc * cpn * nps; }
  __device__ CpuSet all() const { return cs_range(0, cpus); }
  __device__ CpuSet node_cpus(int n) const { return cs_range(n * per_node(), (n + 1) * per_node()); }
  __device__ CpuSet socket_cpus(int s) const { return cs_range(s * per_socket(), (s + 1) * per_socket()); }
};

__device__ __forceinline__ Topo make_topo(const NumaStatic& s) {
  Topo t;
  t.sockets = s.sockets;
  t.nps = s.nps;
  t.cpn = s.cpn;
  t.cpc = s.cpc > 0 ? s.cpc : 1;
  t.nodes = s.sockets * s.nps;
  t.cores = t.nodes * s.cpn;
  t.cpus = t.cores * t.cpc;
  return t;
}

// even-position bits (the first cpu of every 2-cpu core)
constexpr uint64_t kEven = 0x5555555555555555ull;

// cpus of cores whose every cpu is in s (cpc 1: s itself)
__device__ __forceinline__ CpuSet full_core_cpus(const Topo& t, const CpuSet& s) {
  if (t.cpc == 1) return s;
  CpuSet r;
#pragma unroll
  for (int w = 0; w < kCpuWords; ++w) {
    const uint64_t f = s.w[w] & (s.w[w] >> 1) & kEven;
    r.w[w] = f | (f << 1);
  }
  return r;
}
// the first (lowest) cpu of every core with a cpu in s
__device__ __forceinline__ CpuSet first_cpu_per_core(const Topo& t, const CpuSet& s) {
  if (t.cpc == 1) return s;
  CpuSet r;
#pragma unroll
  for (int w = 0; w < kCpuWords; ++w) {
    const uint64_t ev = s.w[w] & kEven, od = s.w[w] & ~kEven;
    r.w[w] = ev | (od & ~(ev << 1));
  }
  return r;
}

// filterCPUsByRequiredCPUBindPolicy (resource_manager.go:534-566)
__device__ __forceinline__ CpuSet filter_required(const Topo& t, const CpuSet& avail, int policy) {
  if (policy == 2 /*FullPCPUs*/) return full_core_cpus(t, avail);
  if (policy == 3 /*SpreadByPCPUs*/) return first_cpu_per_core(t, avail);
  return avail;
}

// the lowest k cpus of s (k ≤ |s|)
__device__ __forceinline__ CpuSet lowest_k(CpuSet s, int k) {
  CpuSet r = cs_zero();
  for (int w = 0; w < kCpuWords && k > 0; ++w) {
    uint64_t v = s.w[w];
    const int c = __popcll(v);
    if (c <= k) {
      r.w[w] = v;
      k -= c;
    } else {
      while (k > 0) {
        const uint64_t low = v & (~v + 1);
        r.w[w] |= low;
        v ^= low;
        --k;
      }
    }
  }
  return r;
}

__device__ __forceinline__ bool better_free(int strategy, int a, int b) { return strategy == 1 ? a < b : a > b; }

// ---------------------------------------------------------------------------------------------------------
// takeCPUs (cpu_accumulator.go:87-232), single thread, on masks.  Returns false on "not enough cpus".
// ---------------------------------------------------------------------------------------------------------
// every cpu of the cores with a cpu in s (cpc ≤ 2)
__device__ __forceinline__ CpuSet expand_cores(const Topo& t, const CpuSet& s) {
  if (t.cpc == 1) return s;
  CpuSet r;
#pragma unroll
  for (int w = 0; w < kCpuWords; ++w) {
    const uint64_t e = (s.w[w] | (s.w[w] >> 1)) & kEven;
    r.w[w] = e | (e << 1);
  }
  return r;
}

struct Acc {
  Topo t;
  CpuSet avail;  // allocatableCPUs
  CpuSet result;
  int needed, strategy;
  int excl;      // the pod's CPUExclusivePolicy (KG_EXCL_*)
  CpuSet seed;   // the node's allocated cpus holding that policy (newCPUAccumulator, cpu_accumulator.go:256-264)
  __device__ void take(const CpuSet& s) {
    result = cs_or(result, s);
    avail = cs_andnot(avail, s);
    needed -= cs_count(s);
  }
  // the cpus a filterExclusive pass skips (isCPUExclusivePCPULevel / NUMANodeLevel, :318-330): every cpu of a core
  // (PCPULevel) or NUMA node (NUMANodeLevel) holding a seed cpu or a cpu this call took (take() grows the sets,
  // :290-304); pcpu / numa: the levels the calling list filters (freeCoresInNode NUMA only, freeCPUsInSocket PCPU
  // only, freeCPUsInNode / freeCPUs both)
  __device__ CpuSet excluded(bool pcpu, bool numa) const {
    if (!((excl == KG_EXCL_PCPU_LEVEL && pcpu) || (excl == KG_EXCL_NUMA_NODE_LEVEL && numa))) return cs_zero();
    const CpuSet held = cs_or(seed, result);
    if (excl == KG_EXCL_PCPU_LEVEL) return expand_cores(t, held);
    CpuSet r = cs_zero();
#pragma unroll
    for (int n = 0; n < 8; ++n)
      if (n < t.nodes && cs_count(cs_and(held, t.node_cpus(n))) > 0) r = cs_or(r, t.node_cpus(n));
    return r;
  }
};

// Group orders as sorted packed keys (ascending key = the reference's order; ids make every key unique, so the
// order is total): ≤ 8 groups sorted by a fixed network on compile-time indices, so the lists live in registers.
constexpr uint64_t kNoGroup = ~0ull;
__device__ __forceinline__ void cswap(uint64_t& a, uint64_t& b) {
  const uint64_t lo = a < b ? a : b, hi = a < b ? b : a;
  a = lo;
  b = hi;
}
// Batcher odd-even merge sort of 8 keys (19 comparators)
__device__ __forceinline__ void sort8(uint64_t* k) {
  cswap(k[0], k[1]); cswap(k[2], k[3]); cswap(k[4], k[5]); cswap(k[6], k[7]);
  cswap(k[0], k[2]); cswap(k[1], k[3]); cswap(k[4], k[6]); cswap(k[5], k[7]);
  cswap(k[1], k[2]); cswap(k[5], k[6]);
  cswap(k[0], k[4]); cswap(k[1], k[5]); cswap(k[2], k[6]); cswap(k[3], k[7]);
  cswap(k[2], k[4]); cswap(k[3], k[5]);
  cswap(k[1], k[2]); cswap(k[3], k[4]); cswap(k[5], k[6]);
}
// a free count as a key field: better_free first (MostAllocated: fewer free first, else more free first)
__device__ __forceinline__ uint64_t free_field(int strategy, int c) {
  return strategy == 1 ? (uint64_t)c : (uint64_t)(0xFFFF - c);
}
// k[g] for a run-time g without a dynamically indexed (scratch) array: a select chain over the 8 registers
__device__ __forceinline__ uint64_t kat(const uint64_t* k, int g) {
  uint64_t v = kNoGroup;
#pragma unroll
  for (int i = 0; i < 8; ++i) v = g == i ? k[i] : v;
  return v;
}
__device__ __forceinline__ int key_id(uint64_t k) { return (int)(k & 0xFFu); }
__device__ __forceinline__ int key_free(int strategy, uint64_t k) {
  const int f = (int)((k >> 32) & 0xFFFFu);
  return strategy == 1 ? f : 0xFFFF - f;
}

// groups (NUMA nodes or sockets) with cpus in `sel`, ordered as freeCoresInNode/Socket(full=true) order them:
// (group free count, [socket free count for nodes], id)
// (av: the allocatable cpus the list counts socket free scores over — filterExclusive passes drop the exclusive ones)
__device__ __forceinline__ void order_groups(const Acc& a, bool by_node, const CpuSet& sel, const CpuSet& av,
                                             uint64_t* k) {
  const int ng = by_node ? a.t.nodes : a.t.sockets;
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    k[g] = kNoGroup;
    if (g >= ng) continue;
    const int c = cs_count(cs_and(sel, by_node ? a.t.node_cpus(g) : a.t.socket_cpus(g)));
    if (c == 0) continue;
    uint64_t key = free_field(a.strategy, c) << 32 | (uint64_t)g;
    if (by_node) key |= free_field(a.strategy, cs_count(cs_and(av, a.t.socket_cpus(g / a.t.nps)))) << 16;
    k[g] = key;
  }
  sort8(k);
}

// first k cpus of a group list where cores are ordered (free count desc, id) and cpus ascending (cpc ≤ 2:
// full cores then single-cpu cores, each ascending)
__device__ __forceinline__ CpuSet first_k_cores_order(const Topo& t, const CpuSet& s, int k) {
  const CpuSet full = full_core_cpus(t, s);
  const int nf = cs_count(full);
  if (k <= nf) return lowest_k(full, k);
  return cs_or(full, lowest_k(cs_andnot(s, full), k - nf));
}

// spreadCPUs over an ascending cpu list: the first cpu of every core (ascending), then the rest (ascending);
// returns the first k
__device__ __forceinline__ CpuSet spread_first_k(const Topo& t, const CpuSet& s, int k) {
  const CpuSet first = first_cpu_per_core(t, s);
  const int nf = cs_count(first);
  if (k <= nf) return lowest_k(first, k);
  return cs_or(first, lowest_k(cs_andnot(s, first), k - nf));
}

// (r6) Not inlined: one shared copy.  Measured on MI355X (scripts/micro/numa_eval.hip, C4 rows, wave-uniform Reserve):
// the inlined copies (an earlier round's choice, to keep the masks in scalar registers) cost 27.9 k cycles per cpuset
// Reserve against 16.0 k for the call; the call's 64-bit mask arithmetic is vector but the body is a third the size.
__device__ __attribute__((noinline)) bool take_cpus(const Topo& t, const CpuSet& available, int needed, int bind, int strategy,
                                          CpuSet& out, int excl, const CpuSet& seed) {
  Acc a;
  a.t = t;
  a.avail = cs_and(available, t.all());
  a.result = cs_zero();
  a.needed = needed;
  a.strategy = strategy;
  a.excl = excl;
  a.seed = seed;
  out = cs_zero();
  if (a.needed < 1) return true;
  if (a.needed > cs_count(a.avail)) return false;
  const bool full = bind == 2;
  // (r6) One NUMA node, exact shortcut: Reserve calls this per NUMA node of the hint, so the available cpus usually lie
  // in one node.  Then freeCoresInNode (no exclusive policy: one pass, nothing excluded) lists that node alone, and
  // when its whole-core cpus cover the request the first branch below takes the lowest `needed` of them — taken here
  // without the eight-group orders.  Any other case runs the full accumulator.
  if ((full || t.cpc == 1) && a.excl == KG_EXCL_NONE && a.needed <= t.per_node()) {
    int lo = -1, hi = -1;
#pragma unroll
    for (int w = 0; w < kCpuWords; ++w)
      if (a.avail.w[w]) {
        if (lo < 0) lo = 64 * w + __builtin_ctzll(a.avail.w[w]);
        hi = 64 * w + 63 - __builtin_clzll(a.avail.w[w]);
      }
    if (lo >= 0 && t.node_of(lo) == t.node_of(hi)) {
      const CpuSet fc = full_core_cpus(t, a.avail);
      if (cs_count(fc) >= a.needed) {
        out = lowest_k(fc, a.needed);
        return true;
      }
    }
  }
  uint64_t k[8];
  if (full || t.cpc == 1) {
    if (a.needed <= t.per_node()) {
      // freeCoresInNode(true, filterExclusive) for filterExclusive true, false (the same list unless NUMANodeLevel)
      for (int fe = 0; fe < (a.excl == KG_EXCL_NUMA_NODE_LEVEL ? 2 : 1); ++fe) {
        const CpuSet av = fe == 0 ? cs_andnot(a.avail, a.excluded(false, true)) : a.avail;
        const CpuSet fc = full_core_cpus(t, av);
        order_groups(a, true, fc, av, k);
        for (int g = 0; g < 8; ++g) {
          const uint64_t kg = kat(k, g);
          if (kg != kNoGroup && key_free(a.strategy, kg) >= a.needed) {
            a.take(lowest_k(cs_and(fc, t.node_cpus(key_id(kg))), a.needed));
            out = a.result;
            return true;
          }
        }
      }
    }
    if (a.needed <= t.per_socket()) {
      const CpuSet fc = full_core_cpus(t, a.avail);
      order_groups(a, false, fc, a.avail, k);
      for (int g = 0; g < 8; ++g) {
        const uint64_t kg = kat(k, g);
        if (kg != kNoGroup && key_free(a.strategy, kg) >= a.needed) {
          a.take(lowest_k(cs_and(fc, t.socket_cpus(key_id(kg))), a.needed));
          out = a.result;
          return true;
        }
      }
    }
    {
      // sockets by (full-core cpu count desc, id): order_groups re-sorted stably by count, most first
      const CpuSet fc = full_core_cpus(t, a.avail);
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        k[s] = kNoGroup;
        if (s >= t.sockets) continue;
        const int c = cs_count(cs_and(fc, t.socket_cpus(s)));
        if (c > 0) k[s] = (uint64_t)(0xFFFF - c) << 32 | (uint64_t)s;
      }
      sort8(k);
      uint32_t um = 0;  // sockets the request does not fill, kept for the core-by-core pass
      for (int g = 0; g < 8; ++g) {
        const uint64_t kg = kat(k, g);
        if (kg == kNoGroup) continue;
        const int id = key_id(kg), c = 0xFFFF - (int)((kg >> 32) & 0xFFFFu);
        if (a.needed < c) {
          um |= 1u << id;
        } else {
          a.take(cs_and(fc, t.socket_cpus(id)));
          if (a.needed < 1) {
            out = a.result;
            return true;
          }
        }
      }
      if (a.needed >= t.cpc) {
        // those sockets by (count, id) ascending: the list above re-sorted stably, fewest first
#pragma unroll
        for (int s = 0; s < 8; ++s)
          k[s] = ((um >> s) & 1u) ? (uint64_t)cs_count(cs_and(fc, t.socket_cpus(s))) << 32 | (uint64_t)s : kNoGroup;
        sort8(k);
        for (int g = 0; g < 8; ++g) {
          const uint64_t kg = kat(k, g);
          if (kg == kNoGroup) continue;
          CpuSet list = cs_and(fc, t.socket_cpus(key_id(kg)));  // the group's full-core cpus, ascending
          while (cs_count(list) > 0) {
            const CpuSet chunk = lowest_k(list, t.cpc);
            list = cs_andnot(list, chunk);
            a.take(chunk);
            if (a.needed < 1) {
              out = a.result;
              return true;
            }
            if (a.needed < t.cpc) break;
          }
        }
      }
    }
  }
  if (!full) {
    if (a.needed <= t.per_node()) {
      for (int fe = 0; fe < 2; ++fe) {
        // freeCPUsInNode: nodes by (node free, socket free, id) on the unreduced counts; with
        // filterExclusive the exclusive cpus are skipped and each list keeps one cpu per core
        const CpuSet av = fe == 0 ? cs_andnot(a.avail, a.excluded(true, true)) : a.avail;
        order_groups(a, true, av, av, k);
        for (int g = 0; g < 8; ++g) {
          const uint64_t kg = kat(k, g);
          if (kg == kNoGroup) continue;
          const CpuSet in = cs_and(av, t.node_cpus(key_id(kg)));
          const CpuSet lst = fe == 0 ? first_cpu_per_core(t, in) : in;
          if (cs_count(lst) >= a.needed) {
            a.take(fe == 0 ? lowest_k(lst, a.needed) : spread_first_k(t, lst, a.needed));
            out = a.result;
            return true;
          }
        }
      }
    }
    if (a.needed <= t.per_socket()) {
      for (int fe = 0; fe < 2; ++fe) {
        // freeCPUsInSocket: sockets by (length of the (reduced) list, id); filterExclusive skips PCPU-level cpus
        const CpuSet av = fe == 0 ? cs_andnot(a.avail, a.excluded(true, false)) : a.avail;
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          k[s] = kNoGroup;
          if (s >= t.sockets) continue;
          const CpuSet in = cs_and(av, t.socket_cpus(s));
          if (cs_count(in) == 0) continue;
          const CpuSet lst = fe == 0 ? first_cpu_per_core(t, in) : in;
          k[s] = free_field(a.strategy, cs_count(lst)) << 32 | (uint64_t)s;
        }
        sort8(k);
        for (int g = 0; g < 8; ++g) {
          const uint64_t kg = kat(k, g);
          if (kg == kNoGroup) continue;
          if (key_free(a.strategy, kg) >= a.needed) {
            const CpuSet in = cs_and(av, t.socket_cpus(key_id(kg)));
            const CpuSet lst = fe == 0 ? first_cpu_per_core(t, in) : in;
            a.take(fe == 0 ? lowest_k(lst, a.needed) : spread_first_k(t, lst, a.needed));
            out = a.result;
            return true;
          }
        }
      }
    }
  }
  // freeCPUs: cores by (socket colo desc, socket free, node free, core free asc, socket, core), then spread;
  // take one by one.  Classes of (socket, node) share the first three keys; inside a run of equal classes
  // single-free cores come before full ones, each by core id (= (socket, core) order in this numbering).
  // filterExclusive true, then false: without an exclusive policy the first list is every free cpu, so the second
  // has nothing left
  for (int fe = 0; fe < (a.excl != KG_EXCL_NONE ? 2 : 1); ++fe) {
    const CpuSet av = fe == 0 ? cs_andnot(a.avail, a.excluded(true, true)) : a.avail;
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      k[n] = kNoGroup;
      if (n >= t.nodes) continue;
      const int nf = cs_count(cs_and(av, t.node_cpus(n)));
      if (nf == 0) continue;
      const int s = n / t.nps;
      const int colo = cs_count(cs_and(a.result, t.socket_cpus(s)));
      const int sf = cs_count(cs_and(av, t.socket_cpus(s)));
      k[n] = (uint64_t)(0xFFFF - colo) << 48 | free_field(a.strategy, sf) << 32 | free_field(a.strategy, nf) << 16 |
             (uint64_t)n;
    }
    sort8(k);
    // the ordered cpu list as runs of equal class (key >> 16), each read as [single-free cores, full cores] in
    // ascending cpu order; the node masks are taken before any cpu is
    const CpuSet avail0 = av;
    // spreadCPUs over the concatenated list: first pass takes the first cpu of each core, second the rest
    for (int pass = 0; pass < 2; ++pass) {
      CpuSet run = cs_zero();
      for (int r = 0; r < 8; ++r) {
        const uint64_t kr = kat(k, r);
        if (kr == kNoGroup) continue;
        run = cs_or(run, cs_and(avail0, t.node_cpus(key_id(kr))));
        const uint64_t nxt = kat(k, r + 1);  // kNoGroup past the end
        if (nxt != kNoGroup && (nxt >> 16) == (kr >> 16)) continue;
        const CpuSet fc = full_core_cpus(t, run);
        const CpuSet parts[2] = {cs_andnot(run, fc), fc};
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const CpuSet first = first_cpu_per_core(t, parts[q]);
          const CpuSet part = pass == 0 ? first : cs_andnot(parts[q], first);
          const int c = cs_count(part);
          if (c == 0) continue;
          a.take(lowest_k(part, c < a.needed ? c : a.needed));
          if (a.needed < 1) {
            out = a.result;
            return true;
          }
        }
        run = cs_zero();
      }
    }
  }
  out = cs_zero();
  return false;
}

// ---------------------------------------------------------------------------------------------------------
// Filter / Score / Reserve
// ---------------------------------------------------------------------------------------------------------
struct NumaHint {
  uint32_t mask;
  int nil, preferred, score;
};

// IterateBitMasks order over ≤ 4 NUMA nodes (size, then lexicographic bit lists), one nibble per mask
__device__ __forceinline__ uint32_t mask_at(int k) {
  // 1,2,4,8 | 3,5,9,6,10,12 | 7,11,13,14 | 15
  constexpr uint64_t order = (1ull << 0) | (2ull << 4) | (4ull << 8) | (8ull << 12) | (3ull << 16) | (5ull << 20) |
                             (9ull << 24) | (6ull << 28) | (10ull << 32) | (12ull << 36) | (7ull << 40) |
                             (11ull << 44) | (13ull << 48) | (14ull << 52) | (15ull << 56);
  return (uint32_t)((order >> (4 * k)) & 15ull);
}

// resourceAllocationScorer.score (scoring.go:191-230) over cpu + memory with least/mostResourceScorer.  The
// strategy is a profile constant: an explicit branch keeps the unused scorer out of the instruction stream.
__device__ __forceinline__ int64_t numa_scorer(int strategy, int32_t w_cpu, int32_t w_mem, int64_t req_c, int64_t req_m,
                                               int64_t alloc_c, int64_t alloc_m, int64_t pod_c, int64_t pod_m) {
  int64_t s = 0, ws = 0;
  if (strategy == 1) {
    if (w_cpu != 0 && alloc_c != 0) {
      s += most_requested64(req_c + pod_c, alloc_c) * w_cpu;
      ws += w_cpu;
    }
    if (w_mem != 0 && alloc_m != 0) {
      s += most_requested64(req_m + pod_m, alloc_m) * w_mem;
      ws += w_mem;
    }
  } else {
    if (w_cpu != 0 && alloc_c != 0) {
      s += least_requested(req_c + pod_c, alloc_c) * w_cpu;
      ws += w_cpu;
    }
    if (w_mem != 0 && alloc_m != 0) {
      s += least_requested(req_m + pod_m, alloc_m) * w_mem;
      ws += w_mem;
    }
  }
  return ws ? div_small(s, ws) : 0;
}

__device__ __forceinline__ CpuSet numa_available_cpus(const Topo& t, const NumaStatic& s, const NumaMut& m) {
  CpuSet a = t.all();
#pragma unroll
  for (int w = 0; w < kCpuWords; ++w) a.w[w] &= ~(m.allocated[w] | s.reserved[w]);
  return a;
}

// ---------------------------------------------------------------------------------------------------------
// Pod-independent view of one node (recomputed when its NodeAllocation changes): every quantity Filter and
// Score read, as counts.  Per NUMA node i: the available cpus (getAvailableCPUs ∩ NUMA node i) raw, reduced
// to whole free cores (filterCPUsByRequiredCPUBindPolicy FullPCPUs) and to one cpu per core (SpreadByPCPUs).
// Every array is indexed only by unrolled compile-time indices, so the view lives in registers.
// ---------------------------------------------------------------------------------------------------------
struct NumaView {
  double amp;  // cpu amplification ratio (≤ 1 = none)
  int32_t valid, policy, node_bind, cpc, nn, strategy, n_alloc;
  int32_t cnt[3][kNumaMax];  // [kind: 0 raw, 1 full cores, 2 one per core][NUMA node]
  int32_t tot[3];
  int64_t numa_cpu[kNumaMax], numa_mem[kNumaMax], alloc_cpu[kNumaMax], alloc_mem[kNumaMax];
};

// which count a cpu-bind policy reads (filterCPUsByRequiredCPUBindPolicy only reduces for FullPCPUs / Spread)
__device__ __forceinline__ int kind_of(int bind) { return bind == 2 ? 1 : (bind == 3 ? 2 : 0); }
// (value selects laundered as in kernels.h pick(): a select of the three loads must not become a load of a
// selected address, which would move the whole view to scratch)
__device__ __forceinline__ int32_t sel3(int kind, int32_t a, int32_t b, int32_t c) {
  asm("" : "+v"(a), "+v"(b), "+v"(c));
  return kind == 1 ? b : (kind == 2 ? c : a);
}
__device__ __forceinline__ int32_t cnt_at(const NumaView& v, int kind, int i) {
  return sel3(kind, v.cnt[0][i], v.cnt[1][i], v.cnt[2][i]);
}
__device__ __forceinline__ int32_t tot_at(const NumaView& v, int kind) { return sel3(kind, v.tot[0], v.tot[1], v.tot[2]); }

__device__ __forceinline__ NumaView make_view(const NumaStatic* __restrict__ s, const NumaMut* __restrict__ m,
                                              const NumaParams& NP) {
  NumaView v;
  Topo t;
  t.sockets = s->sockets;
  t.nps = s->nps;
  t.cpn = s->cpn;
  t.cpc = s->cpc > 0 ? s->cpc : 1;
  t.nodes = t.sockets * t.nps;
  t.cores = t.nodes * t.cpn;
  t.cpus = t.cores * t.cpc;
  v.amp = s->cpu_amp;
  v.valid = s->valid;
  v.policy = s->policy;
  v.node_bind = s->node_bind;
  v.cpc = t.cpc;
  v.nn = s->num_numa;
  v.strategy = s->strategy >= 0 ? s->strategy : NP.default_alloc_strategy;
  CpuSet alloc, avail = t.all();
#pragma unroll
  for (int w = 0; w < kCpuWords; ++w) {
    alloc.w[w] = m->allocated[w];
    avail.w[w] &= ~(alloc.w[w] | s->reserved[w]);
  }
  v.n_alloc = cs_count(alloc);
  const CpuSet full = full_core_cpus(t, avail), spread = first_cpu_per_core(t, avail);
  v.tot[0] = cs_count(avail);
  v.tot[1] = cs_count(full);
  v.tot[2] = cs_count(spread);
  int32_t acnt[kNumaMax];  // allocated cpus per NUMA node
  const int pn = t.per_node();
  if (pn > 0 && (pn & 63) == 0) {
    // NUMA nodes of whole 64-cpu words (e.g. 64 / 128 cpus per node): per-word popcounts summed per node, instead of
    // building each node's range mask (a view is rebuilt per pod on the resolvers' serial path)
    const int wpn = pn >> 6;
    int32_t pa[kCpuWords], pf[kCpuWords], ps[kCpuWords], pl[kCpuWords];
#pragma unroll
    for (int w = 0; w < kCpuWords; ++w) {
      pa[w] = __popcll(avail.w[w]);
      pf[w] = __popcll(full.w[w]);
      ps[w] = __popcll(spread.w[w]);
      pl[w] = __popcll(alloc.w[w]);
    }
#pragma unroll
    for (int i = 0; i < kNumaMax; ++i) {
      int32_t c0 = 0, c1 = 0, c2 = 0, cl = 0;
#pragma unroll
      for (int w = 0; w < kCpuWords; ++w) {
        const bool in = w >= i * wpn && w < (i + 1) * wpn;
        c0 += in ? pa[w] : 0;
        c1 += in ? pf[w] : 0;
        c2 += in ? ps[w] : 0;
        cl += in ? pl[w] : 0;
      }
      v.cnt[0][i] = c0;
      v.cnt[1][i] = c1;
      v.cnt[2][i] = c2;
      acnt[i] = cl;
    }
  } else {
#pragma unroll
    for (int i = 0; i < kNumaMax; ++i) {
      const CpuSet nc = t.node_cpus(i);
      v.cnt[0][i] = cs_count(cs_and(avail, nc));
      v.cnt[1][i] = cs_count(cs_and(full, nc));
      v.cnt[2][i] = cs_count(cs_and(spread, nc));
      acnt[i] = cs_count(cs_and(alloc, nc));
    }
  }
#pragma unroll
  for (int i = 0; i < kNumaMax; ++i) {
    v.numa_cpu[i] = s->numa_cpu[i];
    v.numa_mem[i] = s->numa_mem[i];
    // getAvailableNUMANodeResources (node_allocation.go:155-177): with a cpu ratio > 1 the cpuset part of an
    // allocatedResources entry (allocated cpus on NUMA node i × 1000) counts amplified
    const bool present = (m->present >> i) & 1u;
    const int64_t sets = (int64_t)acnt[i] * 1000;
    v.alloc_cpu[i] = present ? m->alloc_cpu[i] - sets + amplify(sets, v.amp) : 0;
    v.alloc_mem[i] = present ? m->alloc_mem[i] : 0;
  }
  return v;
}

// getResourceOptions (plugin.go:470-510): a cpu-bind pod's cpu request amplified by the node's ratio
// (AmplifyResourceList), for the hints, the NUMA allocation and the score
__device__ __forceinline__ int64_t opt_cpu(const NumaView& v, const NumaPod& p) {
  return p.cpu_bind ? amplify(p.req_cpu, v.amp) : p.req_cpu;
}

// getPreferredCPUBindPolicy (plugin.go:556-576); -1: getResourceOptions fails (topology missing / invalid)
__device__ __forceinline__ int numa_pref_bind(const NumaView& v, int preferred) {
  if (!v.valid) return -1;
  if (v.node_bind == 2 /*SpreadByPCPUs*/) return 3;
  if (v.node_bind == 1 /*FullPCPUsOnly*/) return 2;
  return preferred;
}

// One provider list of the topology manager: a single "don't care" (nil) hint, or hints over the masks of a
// set of enumeration positions, each preferred or not; `empty` = no hint at all
struct HintList {
  uint32_t set;   // positions k (mask_at(k)) in enumeration order
  uint32_t pref;  // positions whose hint is preferred
  int nil, nil_pref, empty;
};

// enumeration positions of the masks of one size: mask_at enumerates by size, so a size class is a contiguous run
// (generateResourceHints marks a mask preferred iff its size is the list's minimum, resource_manager.go:511-525)
__device__ __forceinline__ uint32_t size_class(int size) {
  return size == 1 ? 0x000Fu : size == 2 ? 0x03F0u : size == 3 ? 0x3C00u : 0x4000u;
}

// positions of a list's preferred hints
__device__ __forceinline__ uint32_t preferred_positions(const HintList& L) {
  if (L.nil) return L.nil_pref ? 1u : 0u;
  return L.set & L.pref;
}

// mergeFilteredHints (policy.go:127-185) over the permutations of ≤ 2 lists (the last varies fastest).
// Exact pruning: the first preferred permutation with a non-empty merge always replaces a non-preferred best,
// and after it no non-preferred one can; so when any preferred permutation merges non-empty the result is the
// same fold restricted to the preferred permutations (≤ 6 × 6 of them instead of ≤ 15 × 15), in the same order.
// Only when none does (every merge among them empty, so none changed the best) are all permutations folded.
template <typename ScoreOf>
__device__ __forceinline__ NumaHint merge_hints(uint32_t def, const HintList L0, const HintList L1, int nl,
                                                const ScoreOf& score_of) {
  NumaHint best{def, 0, 0, 0};
  if (L0.empty || (nl > 1 && L1.empty)) return best;
  const uint32_t s0 = L0.nil ? 1u : L0.set;
  const uint32_t s1 = nl > 1 ? (L1.nil ? 1u : L1.set) : 1u;
  const bool nilb = nl > 1 ? L1.nil != 0 : true;
  const uint32_t q0 = preferred_positions(L0), q1 = nl > 1 ? preferred_positions(L1) : 1u;
  KG_COUNT(0);
  // (r6) Single-NUMA fast path, exact: when every preferred hint of both lists is a single-NUMA mask (positions 0-3,
  // mask_at(k) = 1 << k: every pod whose request fits one NUMA node), pass 0's non-empty merges are the NUMA nodes in
  // both lists, met in ascending order, all preferred, each scored with its own mask; the fold takes the first and
  // then replaces it only on a higher score (a wider mask is never narrower) — the first of the highest score.  Only
  // those ≤ 4 scores are computed, not the pass's ≤ 16 iterations with a divergent score inside.
  if (!L0.nil && (nl == 1 || !L1.nil) && !(q0 & ~0xFu) && (nl == 1 || !(q1 & ~0xFu))) {
    const uint32_t c = q0 & (nl > 1 ? q1 : 0xFu);
    if (c) {
      int bi = 0, bs = -1;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if ((c >> i) & 1u) {
          const int sc = score_of(1u << i);
          if (sc > bs) {
            bs = sc;
            bi = i;
          }
        }
      return NumaHint{1u << bi, 0, 1, bs};
    }
  }
#pragma unroll 1
  for (int pass = 0; pass < 2; ++pass) {
    if (pass == 1) KG_COUNT(1);
    const uint32_t t0 = pass == 0 ? q0 : s0, t1 = pass == 0 ? q1 : s1;
    for (uint32_t a = t0; a; a &= a - 1) {
      const int ka = __builtin_ctz(a);
      const uint32_t ma = L0.nil ? def : mask_at(ka);
      const bool pa = L0.nil ? L0.nil_pref != 0 : ((L0.pref >> ka) & 1u) != 0;
      for (uint32_t b = t1; b; b &= b - 1) {
        const int kb = __builtin_ctz(b);
        const uint32_t mb = nilb ? def : mask_at(kb);
        const bool pb = nl > 1 ? (nilb ? L1.nil_pref != 0 : ((L1.pref >> kb) & 1u) != 0) : true;
        const uint32_t merged = def & ma & mb;
        if (merged == 0) continue;
        const int preferred = pa && pb;
        // a hint's score is its mask's (generateResourceHints), so the permutation's is that of the merged mask
        // when some hint equals it — computed only then
        const int score = ((!L0.nil && ma == merged) || (!nilb && mb == merged)) ? score_of(merged) : 0;
        const int pm = __popc(merged), pbst = __popc(best.mask);
        if (preferred && !best.preferred) {
          best = NumaHint{merged, 0, 1, score};
        } else if (!preferred && best.preferred) {
        } else {
          const bool narrower = pm == pbst ? merged < best.mask : pm < pbst;
          if (!narrower) {
            if (pm == pbst && score > best.score) best = NumaHint{merged, 0, preferred, score};
          } else {
            best = NumaHint{merged, 0, preferred, score};
          }
        }
      }
    }
    if (best.preferred) break;
  }
  return best;
}

__device__ __forceinline__ HintList single_numa_only(HintList L) {
  // filterSingleNumaHints: "don't care" hints that are preferred, and preferred single-NUMA hints
  if (L.nil) {
    if (!L.nil_pref) L.empty = 1;
    return L;
  }
  const uint32_t keep = L.set & L.pref & size_class(1);  // positions 0..3 are the single-NUMA masks
  L.set = keep;
  if (!keep) L.empty = 1;
  return L;
}

// Policy.Merge + canAdmitPodResult (policy_best_effort.go:43-48, policy_restricted.go:41-46,
// policy_single_numa_node.go:62-77) over ≤ 2 provider lists.  One merge for every policy (lanes of one wave hold
// nodes of different policies: a single inlined merge keeps the divergent path to one copy).
template <typename ScoreOf>
__device__ __forceinline__ bool policy_merge(int policy, uint32_t def, const HintList& L0, const HintList& L1, int nl,
                                             const ScoreOf& score_of, NumaHint& best) {
  const bool single = policy == 3 /*SingleNUMANode*/;
  best = merge_hints(def, single ? single_numa_only(L0) : L0, single ? single_numa_only(L1) : L1, nl, score_of);
  if (single) {
    if (!best.nil && best.mask == def) best = NumaHint{0, 1, best.preferred, 0};
    return best.preferred != 0;
  }
  if (policy == 2 /*Restricted*/) return best.preferred != 0;
  return true;  // BestEffort
}

// Topology-manager Admit for the NodeNUMAResource provider alone (manager.go:58-100, policy_*.go) with the
// hints of generateResourceHints (resource_manager.go:418-532).  Returns admit; writes the best hint.
__device__ __forceinline__ bool numa_admit(const NumaView& v, const NumaPod& p, const NumaParams& NP, NumaHint& best) {
  const int nn = v.nn;
  const uint32_t def = (1u << nn) - 1u;
  const int bind = numa_pref_bind(v, p.preferred);
  HintList L0{0, 0, 1, 1, 0}, L1{0, 0, 1, 1, 0};
  int nl = 1;
  const bool req_c = p.req_cpu > 0, req_m = p.req_mem > 0;
  const int64_t rqc = opt_cpu(v, p);
  int64_t av_cpu[kNumaMax], av_mem[kNumaMax];
#pragma unroll
  for (int i = 0; i < kNumaMax; ++i) av_cpu[i] = av_mem[i] = 0;
  // the score of a hint mask (resource_manager.go:479-500: scorer over the mask's NUMA nodes), computed lazily
  // by the merge for the masks it actually compares
  const auto score_of = [&](uint32_t mk) -> int {
    int64_t a_c = 0, a_m = 0, tot_c = 0, tot_m = 0;
#pragma unroll
    for (int i = 0; i < kNumaMax; ++i)
      if ((mk >> i) & 1u) {
        a_c += av_cpu[i];
        a_m += av_mem[i];
        tot_c += v.numa_cpu[i];
        tot_m += v.numa_mem[i];
      }
    const int64_t rq_c = tot_c - a_c > 0 ? tot_c - a_c : 0, rq_m = tot_m - a_m > 0 ? tot_m - a_m : 0;
    return (int)numa_scorer(NP.numa_strategy, NP.nw_cpu, NP.nw_mem, rq_c, rq_m, tot_c, tot_m, rqc, p.req_mem);
  };
  if (bind >= 0 && (req_c || req_m)) {
    const bool trim = p.cpu_bind && p.required != 0;
    const int kind = kind_of(bind);
#pragma unroll
    for (int i = 0; i < kNumaMax; ++i) {
      const int64_t ac = v.numa_cpu[i] - v.alloc_cpu[i], am = v.numa_mem[i] - v.alloc_mem[i];
      av_cpu[i] = i < nn && ac > 0 ? ac : 0;
      av_mem[i] = i < nn && am > 0 ? am : 0;
      if (trim && av_cpu[i] != 0) {  // trimNUMANodeResources (:140-169)
        const int64_t raw = (int64_t)v.cnt[0][i] * 1000;
        const int64_t c = raw >= av_cpu[i] ? (int64_t)cnt_at(v, kind, i) * 1000 : raw;
        if (c < av_cpu[i]) av_cpu[i] = c;
      }
    }
    uint32_t hc = 0, hm = 0;
    int min_c = nn, min_m = nn;
#pragma unroll  // constant masks: each subset sum is a fixed 0-3 adds
    for (int k = 0; k < 15; ++k) {
      const uint32_t mk = mask_at(k);
      if (mk & ~def) continue;
      int64_t a_c = 0, a_m = 0, tot_c = 0, tot_m = 0;
#pragma unroll
      for (int i = 0; i < kNumaMax; ++i)
        if ((mk >> i) & 1u) {
          a_c += av_cpu[i];
          a_m += av_mem[i];
          tot_c += v.numa_cpu[i];
          tot_m += v.numa_mem[i];
        }
      const int cnt = __popc(mk);
      if (req_m && tot_m >= p.req_mem) {
        if (cnt < min_m) min_m = cnt;
        if (a_m >= p.req_mem) hm |= 1u << k;
      }
      if (req_c && tot_c >= rqc) {
        if (cnt < min_c) min_c = cnt;
        if (a_c >= rqc) hc |= 1u << k;
      }
    }
    // filterProvidersHints (policy.go:94-125): resources in sorted-name order (cpu, memory); a present but
    // empty list becomes one non-preferred "don't care" hint
    const HintList lc = hc ? HintList{hc, size_class(min_c), 0, 0, 0} : HintList{0, 0, 1, 0, 0};
    const HintList lm = hm ? HintList{hm, size_class(min_m), 0, 0, 0} : HintList{0, 0, 1, 0, 0};
    if (req_c) {
      L0 = lc;
      if (req_m) {
        L1 = lm;
        nl = 2;
      }
    } else {
      L0 = lm;
    }
  }
  return policy_merge(v.policy, def, L0, L1, nl, score_of, best);
}

// allocateResourcesByHint (resource_manager.go:195-250): per NUMA node i (ascending within the hint) the cpu /
// memory taken; `res` = bit i when NUMA node i got an entry.  False on insufficient NUMA resources.
struct NumaAlloc {
  uint32_t res;
  int64_t cpu[kNumaMax], mem[kNumaMax];
};

__device__ __forceinline__ bool alloc_by_hint(const NumaView& v, const NumaPod& p, uint32_t mask, NumaAlloc& a) {
  a.res = 0;
#pragma unroll
  for (int i = 0; i < kNumaMax; ++i) a.cpu[i] = a.mem[i] = 0;
  if (v.nn == 0) return false;
  // a cpu-bind pod splits its ORIGINAL requests (resource_manager.go:205-210, options.originalRequests), never the
  // amplified ones the hints and Score use; other pods' requests are not amplified at all
  int64_t rq_c = p.req_cpu, rq_m = p.req_mem;
  const bool key_c = p.req_cpu > 0, key_m = p.req_mem > 0;
  bool done = false;
#pragma unroll
  for (int i = 0; i < kNumaMax; ++i) {
    if (done || i >= v.nn || !((mask >> i) & 1u)) continue;
    int64_t ac = 0, am = 0;
    if (key_c) {
      const int64_t av = v.numa_cpu[i] - v.alloc_cpu[i] > 0 ? v.numa_cpu[i] - v.alloc_cpu[i] : 0;
      ac = rq_c < av ? rq_c : av;
      rq_c -= ac;
    }
    if (key_m) {
      const int64_t av = v.numa_mem[i] - v.alloc_mem[i] > 0 ? v.numa_mem[i] - v.alloc_mem[i] : 0;
      am = rq_m < av ? rq_m : av;
      rq_m -= am;
    }
    if (ac != 0 || am != 0) {
      a.res |= 1u << i;
      a.cpu[i] = ac;
      a.mem[i] = am;
    }
    if (rq_c == 0 && rq_m == 0) done = true;
  }
  return !((key_c && rq_c != 0) || (key_m && rq_m != 0));
}

// resourceManager.Allocate feasibility (resource_manager.go:171-360) from counts: the per-NUMA takes of
// allocateCPUSet never fail, and a FullPCPUs take of k cpus from whole-core lists is whole cores iff k is a
// multiple of cpus-per-core, so satisfiedRequiredCPUBindPolicy reduces to that parity.
__device__ __forceinline__ bool numa_feasible(const NumaView& v, const NumaPod& p, const NumaHint& h, NumaAlloc& a) {
  a.res = 0;
  const int bind = numa_pref_bind(v, p.preferred);
  if (bind < 0) return false;
  if (!h.nil && !alloc_by_hint(v, p, h.mask, a)) return false;
  if (!p.cpu_bind) return true;
  const bool required = p.required != 0;
  const int kind = required ? kind_of(bind) : 0;
  if (tot_at(v, kind) < p.needed) return false;
  const bool whole = required && bind == 2 && v.cpc > 1;
  if (a.res) {
    int got = 0;
    bool ok = true;
#pragma unroll
    for (int i = 0; i < kNumaMax; ++i) {
      if (!((a.res >> i) & 1u)) continue;
      int num = cnt_at(v, kind, i);
      const int want = (int)(a.cpu[i] / 1000);
      if (want < num) num = want;
      ok &= !(whole && (num % v.cpc) != 0);
      got += num;
    }
    return ok && got == p.needed;
  }
  return !(whole && p.needed % v.cpc != 0);
}

__device__ __forceinline__ bool skip_the_node(const NumaPod& p, int policy) {
  return p.skip || (!p.cpu_bind && policy == 0);
}

// NodeNUMAResource.Filter (plugin.go:276-334); writes the affinity the topology manager stores
// `fa` / `fa_ok`: when Filter passes and has run Allocate feasibility for the affinity it stores, that
// allocation (Score runs the same check on the same state and reuses it)
__device__ __forceinline__ bool numa_filter(const NumaView& v, const NumaPod& p, const NumaParams& NP, NumaHint& aff,
                                            int64_t node_req_cpu, int64_t node_alloc_cpu, NumaAlloc& fa,
                                            bool& fa_ok) {
  fa_ok = false;
  aff = NumaHint{0, 1, 0, 0};
  if (p.prefilter_error) return false;
  if (p.req_cpu != 0 && v.amp > 1.0) {  // filterAmplifiedCPUs (plugin.go:336-373)
    const int64_t pod = opt_cpu(v, p);
    const int64_t am = v.valid ? (int64_t)v.n_alloc * 1000 : 0;  // GetAvailableCPUs needs a valid topology
    int64_t req = node_req_cpu;
    if (req >= am && am > 0) req = req - am + amplify(am, v.amp);
    if (pod > node_alloc_cpu - req) return false;  // ErrInsufficientAmplifiedCPU
  }
  if (skip_the_node(p, v.policy)) return true;
  if (p.cpu_bind) {
    if (!v.valid) return false;
    const bool full_only = v.node_bind == 1;
    if (full_only || p.required == 2) {
      if (p.needed % v.cpc != 0) return false;                                // SMT alignment
      if (full_only && (p.required != 2 || p.preferred != 2)) return false;  // required FullPCPUs policy
    }
  }
  // Allocate feasibility runs once: on "don't care" for a required cpu-bind pod without a NUMA policy, on the
  // admitted hint otherwise (the two cases exclude each other)
  bool feas = p.cpu_bind && p.required != 0 && v.policy == 0;
  if (v.policy != 0) {
    if (v.nn == 0) return false;
    NumaHint best;
    if (!numa_admit(v, p, NP, best)) return false;
    aff = best;
    feas = true;
  }
  if (feas) {
    if (!numa_feasible(v, p, aff, fa)) return false;
    fa_ok = true;
  }
  return true;
}
__device__ __forceinline__ bool numa_filter(const NumaView& v, const NumaPod& p, const NumaParams& NP, NumaHint& aff,
                                            int64_t node_req_cpu, int64_t node_alloc_cpu) {
  NumaAlloc fa;
  bool fa_ok;
  return numa_filter(v, p, NP, aff, node_req_cpu, node_alloc_cpu, fa, fa_ok);
}

// NodeNUMAResource.Score (scoring.go:55-168) with the stored affinity; node_* = NodeInfo.Requested/Allocatable
__device__ __forceinline__ int64_t numa_score(const NumaView& v, const NumaPod& p, const NumaParams& NP,
                                              const NumaHint& aff, int64_t node_req_cpu, int64_t node_req_mem,
                                              int64_t node_alloc_cpu, int64_t node_alloc_mem,
                                              const NumaAlloc* known = nullptr) {
  // both branches end in one scorer call (a single inlined copy on the divergent path)
  int64_t ac = node_alloc_cpu, am = node_alloc_mem, rc = node_req_cpu, rm = node_req_mem, pc = p.req_cpu;
  if (skip_the_node(p, v.policy)) {
    if (p.skip) return 0;
    if (numa_pref_bind(v, p.preferred) < 0) return 0;  // scoreWithAmplifiedCPUs: getResourceOptions
    if (p.req_cpu != 0 && v.amp > 1.0) {  // the cpuset part of Requested counts amplified (scoring.go:95-120)
      const int64_t an = (int64_t)v.n_alloc * 1000;
      rc = rc - an + amplify(an, v.amp);
    }
  } else {
    if (p.cpu_bind && !v.valid) return 0;
    NumaAlloc a;
    if (known) a = *known;
    else if (!numa_feasible(v, p, aff, a)) return 0;
    if (a.res) {  // calculateAllocatableAndRequested (:122-168): the hint's NUMA nodes
      ac = am = rc = rm = 0;
#pragma unroll
      for (int i = 0; i < kNumaMax; ++i)
        if ((a.res >> i) & 1u) {
          rc += v.alloc_cpu[i];
          rm += v.alloc_mem[i];
          ac += v.numa_cpu[i];
          am += v.numa_mem[i];
        }
    }
    // a cpuset pod: requested cpu = Amplify(|allocated cpus| · 1000) (needed ≥ 1 whenever cpu_bind)
    if (p.cpu_bind) rc = amplify((int64_t)v.n_alloc * 1000, v.amp);
    pc = opt_cpu(v, p);
  }
  return numa_scorer(NP.node_strategy, NP.w_cpu, NP.w_mem, rc, rm, ac, am, pc, p.req_mem);
}

// Filter (when the profile has it) + Score of one node: feasibility and the unweighted plugin score
__device__ __forceinline__ bool numa_eval(const NumaView& v, const NumaPod& p, const NumaParams& NP,
                                          int64_t node_req_cpu, int64_t node_req_mem, int64_t node_alloc_cpu,
                                          int64_t node_alloc_mem, int64_t& score, NumaHint& aff) {
  aff = NumaHint{0, 1, 0, 0};
  score = 0;
  NumaAlloc fa;
  bool fa_ok = false;
  if (NP.filter && !numa_filter(v, p, NP, aff, node_req_cpu, node_alloc_cpu, fa, fa_ok)) return false;
  if (NP.score)
    score = numa_score(v, p, NP, aff, node_req_cpu, node_req_mem, node_alloc_cpu, node_alloc_mem, fa_ok ? &fa : nullptr);
  return true;
}

// NodeNUMAResource.Reserve (plugin.go:375-415) → Allocate with the exact cpuset (cpu accumulator) →
// addPodAllocation (node_allocation.go:76-103).  False: the allocation fails and the pod is not placed.
// (inlined: the resolvers call it wave-uniformly, see take_cpus)
__device__ __forceinline__ bool numa_reserve(const NumaStatic& s, NumaMut& m, const NumaView& v, const NumaPod& p,
                                             const NumaHint& aff, CpuSet& cpus, NumaAlloc& rec) {
  cpus = cs_zero();
  rec.res = 0;  // the PodAllocation's NUMANodeResources, kept for Release (node_allocation.go:105-131)
  if (skip_the_node(p, v.policy)) return true;
  if (p.cpu_bind && !v.valid) return false;
  NumaAlloc a;
  if (!numa_feasible(v, p, aff, a)) return false;
  if (p.cpu_bind) {  // allocateCPUSet (:273-360), exact
    const Topo t = make_topo(s);
    const int bind = numa_pref_bind(v, p.preferred);
    CpuSet avail = numa_available_cpus(t, s, m);
    if (p.required != 0) avail = filter_required(t, avail, bind);
    CpuSet seed = cs_zero();  // the allocated cpus holding the pod's exclusive policy
#pragma unroll
    for (int w = 0; w < kCpuWords; ++w)
      seed.w[w] = p.excl == KG_EXCL_PCPU_LEVEL ? m.excl_pcpu[w] : p.excl == KG_EXCL_NUMA_NODE_LEVEL ? m.excl_numa[w] : 0;
    // per NUMA node of the hint (ascending), or once over every available cpu: one inlined take_cpus
    const int parts = a.res ? kNumaMax : 1;
    for (int i = 0; i < parts; ++i) {
      if (a.res && !((a.res >> i) & 1u)) continue;
      const CpuSet in = a.res ? cs_and(avail, t.node_cpus(i)) : avail;
      int num = p.needed;
      if (a.res) {
        num = cs_count(in);
        const int want = (int)(a.cpu[i] / 1000);
        if (want < num) num = want;
      }
      CpuSet one;
      if (!take_cpus(t, in, num, bind, v.strategy, one, p.excl, seed)) return false;
      cpus = cs_or(cpus, one);
    }
    if (p.required != 0) {  // satisfiedRequiredCPUBindPolicy (:568-589), exact
      if (bind == 2 && t.cpc > 1 && cs_count(full_core_cpus(t, cpus)) != cs_count(cpus)) return false;
      if (bind == 3 && cs_count(first_cpu_per_core(t, cpus)) != cs_count(cpus)) return false;
    }
  }
#pragma unroll
  for (int w = 0; w < kCpuWords; ++w) {
    m.allocated[w] |= cpus.w[w];
    // addPodAllocation: the pod's cpus carry its exclusive policy (node_allocation.go:82-90)
    m.excl_pcpu[w] = (m.excl_pcpu[w] & ~cpus.w[w]) | (p.excl == KG_EXCL_PCPU_LEVEL ? cpus.w[w] : 0ull);
    m.excl_numa[w] = (m.excl_numa[w] & ~cpus.w[w]) | (p.excl == KG_EXCL_NUMA_NODE_LEVEL ? cpus.w[w] : 0ull);
  }
#pragma unroll
  for (int i = 0; i < kNumaMax; ++i)
    if ((a.res >> i) & 1u) {
      m.alloc_cpu[i] += a.cpu[i];
      m.alloc_mem[i] += a.mem[i];
    }
  m.present |= a.res;
  rec = a;
  return true;
}

// ---------------------------------------------------------------------------------------------------------
// (r6) Reservations holding cpusets.  getResourceOptions (plugin.go:465-510) gives a pod nominated into a reservation
// preferredCPUs P = the reservation's reserved cpus (RestoreReservation: its cpuset minus its assigned pods', every one
// of them held by the reservation alone, RefCount 1) and reusableResources = Amplify(|P on NUMA node i| × 1000) of cpu
// per NUMA node holding some.  GetAvailableCPUs(P) drops P's RefCounts to 0, so P is available and its cpus leave the
// allocated CPUDetails; getAvailableNUMANodeResources subtracts the reusable cpu from allocatedResources (≥ 0).
// ---------------------------------------------------------------------------------------------------------
// the view with P: the reusable cpu off each NUMA node's allocated cpu (the counts of `v` are not used with P)
__device__ __forceinline__ NumaView view_with_pref(NumaView v, const NumaStatic& s, const CpuSet& P) {
  const Topo t = make_topo(s);
  const CpuSet pin = cs_and(P, t.all());
#pragma unroll
  for (int i = 0; i < kNumaMax; ++i) {
    const int k = cs_count(cs_and(pin, t.node_cpus(i)));
    const int64_t reusable = k > 0 ? amplify((int64_t)k * 1000, v.amp) : 0;
    const int64_t ac = v.alloc_cpu[i] - reusable;
    v.alloc_cpu[i] = ac > 0 ? ac : 0;  // 0 stays 0 for a NUMA node without an allocatedResources entry
  }
  return v;
}

// takePreferredCPUs (cpu_accumulator.go:33-85): up to `needed` cpus from the preferred ones among `in` (one takeCPUs
// over them), then the rest from the others — one inlined take_cpus in a two-pass loop
__device__ __forceinline__ bool take_preferred(const Topo& t, const CpuSet& in, const CpuSet& P, int needed, int bind,
                                               int strategy, CpuSet& out, int excl, const CpuSet& seed) {
  out = cs_zero();
  const CpuSet pc = cs_and(in, P);
  const int np = cs_count(pc);
  for (int ph = 0; ph < 2; ++ph) {
    if (ph == 0 && np == 0) continue;
    if (ph == 1 && needed <= 0) break;
    const CpuSet set = ph == 0 ? pc : cs_andnot(in, pc);
    const int k = ph == 0 ? (needed < np ? needed : np) : needed;
    CpuSet one;
    if (!take_cpus(t, set, k, bind, strategy, one, excl, seed)) return false;
    out = cs_or(out, one);
    needed -= cs_count(one);
  }
  return true;
}

// resourceManager.Allocate (resource_manager.go:171-360) with preferredCPUs P, exact: allocateResourcesByHint on the
// reusable-adjusted view `vp`, then allocateCPUSet — GetAvailableCPUs(P), the required-policy filter, per NUMA node of
// the allocation (or once) takePreferredCPUs, satisfiedRequiredCPUBindPolicy.  The accumulator's exclusive seed is
// the allocated CPUDetails after P's RefCount drop.
__device__ __forceinline__ bool numa_alloc_pref(const NumaStatic& s, const NumaMut& m, const NumaView& vp,
                                                const NumaPod& p, const NumaHint& aff, const CpuSet& P, NumaAlloc& a,
                                                CpuSet& cpus) {
  cpus = cs_zero();
  a.res = 0;
  const int bind = numa_pref_bind(vp, p.preferred);
  if (bind < 0) return false;
  if (!aff.nil && !alloc_by_hint(vp, p, aff.mask, a)) return false;
  if (!p.cpu_bind) return true;
  const Topo t = make_topo(s);
  CpuSet held, avail = t.all(), seed;
#pragma unroll
  for (int w = 0; w < kCpuWords; ++w) {
    held.w[w] = m.allocated[w] & ~P.w[w];
    avail.w[w] &= ~(held.w[w] | s.reserved[w]);
    seed.w[w] = (p.excl == KG_EXCL_PCPU_LEVEL ? m.excl_pcpu[w] : p.excl == KG_EXCL_NUMA_NODE_LEVEL ? m.excl_numa[w] : 0ull) &
                held.w[w];
  }
  if (p.required != 0) avail = filter_required(t, avail, bind);
  if (cs_count(avail) < p.needed) return false;
  const int parts = a.res ? kNumaMax : 1;
  for (int i = 0; i < parts; ++i) {
    if (a.res && !((a.res >> i) & 1u)) continue;
    const CpuSet in = a.res ? cs_and(avail, t.node_cpus(i)) : avail;
    int num = p.needed;
    if (a.res) {
      num = cs_count(in);
      const int want = (int)(a.cpu[i] / 1000);
      if (want < num) num = want;
    }
    CpuSet one;
    if (!take_preferred(t, in, P, num, bind, vp.strategy, one, p.excl, seed)) return false;
    cpus = cs_or(cpus, one);
  }
  if (cs_count(cpus) != p.needed) return false;  // "not enough cpus available to satisfy request"
  if (p.required != 0) {
    if (bind == 2 && t.cpc > 1 && cs_count(full_core_cpus(t, cpus)) != cs_count(cpus)) return false;
    if (bind == 3 && cs_count(first_cpu_per_core(t, cpus)) != cs_count(cpus)) return false;
  }
  return true;
}

// NodeNUMAResource.Score with preferredCPUs P (scoring.go:55-168): v = the node's plain view
__device__ __forceinline__ int64_t numa_score_pref(const NumaStatic& s, const NumaMut& m, const NumaView& v,
                                                   const NumaPod& p, const NumaParams& NP, const NumaHint& aff,
                                                   const CpuSet& P, int64_t node_req_cpu, int64_t node_req_mem,
                                                   int64_t node_alloc_cpu, int64_t node_alloc_mem) {
  int64_t ac = node_alloc_cpu, am = node_alloc_mem, rc = node_req_cpu, rm = node_req_mem, pc = p.req_cpu;
  CpuSet alloc;
#pragma unroll
  for (int w = 0; w < kCpuWords; ++w) alloc.w[w] = m.allocated[w];
  if (skip_the_node(p, v.policy)) {
    if (p.skip) return 0;
    if (numa_pref_bind(v, p.preferred) < 0) return 0;
    if (p.req_cpu != 0 && v.amp > 1.0) {  // scoreWithAmplifiedCPUs: GetAvailableCPUs(node, P)'s allocated CPUDetails
      const int64_t an = (int64_t)cs_count(cs_andnot(alloc, P)) * 1000;
      rc = rc - an + amplify(an, v.amp);
    }
  } else {
    if (p.cpu_bind && !v.valid) return 0;
    const NumaView vp = view_with_pref(v, s, P);
    NumaAlloc a;
    CpuSet c;
    if (!numa_alloc_pref(s, m, vp, p, aff, P, a, c)) return 0;
    if (a.res) {  // calculateAllocatableAndRequested: totalAllocated with the reusable cpu subtracted
      ac = am = rc = rm = 0;
#pragma unroll
      for (int i = 0; i < kNumaMax; ++i)
        if ((a.res >> i) & 1u) {
          rc += vp.alloc_cpu[i];
          rm += vp.alloc_mem[i];
          ac += vp.numa_cpu[i];
          am += vp.numa_mem[i];
        }
    }
    // getAvailableCPUs with preferred = P − the pod's cpus: the allocated CPUDetails' size
    if (p.cpu_bind) rc = amplify((int64_t)cs_count(cs_andnot(alloc, cs_andnot(P, c))) * 1000, v.amp);
    pc = opt_cpu(v, p);
  }
  return numa_scorer(NP.node_strategy, NP.w_cpu, NP.w_mem, rc, rm, ac, am, pc, p.req_mem);
}

// NodeNUMAResource.Reserve with preferredCPUs P (plugin.go:375-415 → Allocate → addPodAllocation); as numa_reserve
__device__ __forceinline__ bool numa_reserve_pref(const NumaStatic& s, NumaMut& m, const NumaView& v, const NumaPod& p,
                                                  const NumaHint& aff, const CpuSet& P, CpuSet& cpus, NumaAlloc& rec) {
  cpus = cs_zero();
  rec.res = 0;
  if (skip_the_node(p, v.policy)) return true;
  if (p.cpu_bind && !v.valid) return false;
  NumaAlloc a;
  if (!numa_alloc_pref(s, m, view_with_pref(v, s, P), p, aff, P, a, cpus)) return false;
#pragma unroll
  for (int w = 0; w < kCpuWords; ++w) {
    m.allocated[w] |= cpus.w[w];
    m.excl_pcpu[w] = (m.excl_pcpu[w] & ~cpus.w[w]) | (p.excl == KG_EXCL_PCPU_LEVEL ? cpus.w[w] : 0ull);
    m.excl_numa[w] = (m.excl_numa[w] & ~cpus.w[w]) | (p.excl == KG_EXCL_NUMA_NODE_LEVEL ? cpus.w[w] : 0ull);
  }
#pragma unroll
  for (int i = 0; i < kNumaMax; ++i)
    if ((a.res >> i) & 1u) {
      m.alloc_cpu[i] += a.cpu[i];
      m.alloc_mem[i] += a.mem[i];
    }
  m.present |= a.res;
  rec = a;
  return true;
}

// per-pod NUMA allocation record (kg_pods_unreserve): [0] NUMA-node mask, [1 + i] cpu, [1 + kNumaMax + i] memory
constexpr int kNumaRecWords = 1 + 2 * kNumaMax;

// resourceManager.Release → NodeAllocation.release (node_allocation.go:105-131): the pod's cpus leave the
// allocated set (maxRefCount 1), its NUMANodeResources are subtracted with a non-negative result
// (r6) `keep`: the cpus the node's reservations hold — a pod's cpu among them keeps RefCount 1 (the reservation's), so
// it stays allocated with its CPUInfo (node_allocation.go:115-126)
__device__ __forceinline__ void numa_release(NumaMut& m, const uint64_t* cpus, const int64_t* rec,
                                             const uint64_t* keep = nullptr) {
#pragma unroll
  for (int w = 0; w < kCpuWords; ++w) {
    const uint64_t gone = cpus[w] & ~(keep ? keep[w] : 0ull);
    m.allocated[w] &= ~gone;
    m.excl_pcpu[w] &= ~gone;  // RefCount 0: the CPUInfo and its policy are deleted
    m.excl_numa[w] &= ~gone;
  }
#pragma unroll
  for (int i = 0; i < kNumaMax; ++i)
    if ((rec[0] >> i) & 1) {
      const int64_t c = m.alloc_cpu[i] - rec[1 + i], mm = m.alloc_mem[i] - rec[1 + kNumaMax + i];
      m.alloc_cpu[i] = c > 0 ? c : 0;
      m.alloc_mem[i] = mm > 0 ? mm : 0;
    }
}

}  // namespace kg
