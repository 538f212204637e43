/*
 * numa.h — CPU restatement of koord-scheduler's NodeNUMAResource plugin (TEST INFRASTRUCTURE ONLY, like
 * oracle.h).  Implementation and reference citations: numa.c.
 */
#ifndef KG_ORACLE_NUMA_H_
#define KG_ORACLE_NUMA_H_

#include <stdint.h>

#include "../include/koordgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

#define OR_CPUSET_WORDS (KG_MAX_CPUS / 64)

typedef struct {
  uint64_t w[OR_CPUSET_WORDS];
} or_cpuset;

/* CPUTopology in buildCPUTopologyForTest numbering (cpu_accumulator_test.go:30-57) */
typedef struct {
  int num_sockets, num_nodes, num_cores, num_cpus;
  int cpus_per_core, cores_per_node, nodes_per_socket;
  or_cpuset all;
} or_topology;

/* One node's NodeNUMAResource state: TopologyOptions + NodeAllocation (maxRefCount 1).  (r6) `ref` is each cpu's
 * CPUInfo.RefCount (node_allocation.go:76-131): 1 per holder — a pod or a reservation (its reserve pod) — so a cpu a
 * pod took from its reservation's reserved cpus has RefCount 2; `allocated` is the set with RefCount ≥ 1. */
typedef struct {
  int has_topology, valid_topology;
  or_topology topo;
  int numa_policy, node_cpu_bind_policy, numa_allocate_strategy;
  int num_numa;
  int64_t numa_cpu[KG_MAX_NUMA], numa_mem[KG_MAX_NUMA];
  double cpu_amp; /* cpu amplification ratio (≤ 1 = none) */
  or_cpuset reserved;
  /* mutable */
  or_cpuset allocated;
  or_cpuset excl_pcpu, excl_numa; /* allocated cpus whose CPUInfo.ExclusivePolicy is PCPULevel / NUMANodeLevel */
  int64_t numa_alloc_cpu[KG_MAX_NUMA], numa_alloc_mem[KG_MAX_NUMA];
  int numa_alloc_present[KG_MAX_NUMA]; /* allocatedResources[numa] exists */
  uint8_t ref[KG_MAX_CPUS];            /* (r6) CPUInfo.RefCount                                     */
  int refs_ready;                      /* (r6) the reservations' RefCount-2 cpus were counted         */
} or_numa_node;

/* NodeNUMAResource preFilterState (plugin.go:177-186, PreFilter :220-270) */
typedef struct {
  int skip, prefilter_error;
  int request_cpu_bind;
  int required_policy, preferred_policy; /* KG_BIND_* */
  int num_cpus_needed;
  int excl_policy;          /* preferredCPUExclusivePolicy (KG_EXCL_*) */
  int64_t req_cpu, req_mem; /* PodRequestsAndLimits cpu (milli) / memory */
  int allow_cpuset;         /* (r6) AllowUseCPUSet (util.go:42-49): PreRestoreReservation's skip = !allow_cpuset */
} or_numa_pod;

/* the affinity the topology manager stores for a node (store.SetAffinity, manager.go:73) */
typedef struct {
  int nil;       /* NUMANodeAffinity == nil */
  uint32_t mask;
  int preferred;
  int64_t score;
} or_hint;

void or_topology_build(or_topology* t, int sockets, int nodes_per_socket, int cores_per_node, int cpus_per_core);
int or_take_cpus(const or_topology* t, or_cpuset available, int needed, int bind_policy, int strategy,
                 or_cpuset* out);
/* takeCPUs with a CPUExclusivePolicy: excl_seed = the node's allocated cpus holding that policy */
int or_take_cpus_ex(const or_topology* t, or_cpuset available, int needed, int bind_policy, int strategy,
                    int excl_policy, or_cpuset excl_seed, or_cpuset* out);
or_cpuset or_filter_required(const or_topology* t, or_cpuset available, int policy);

void or_numa_node_init(or_numa_node* n, const kg_node_numa* src);
void or_numa_pod_init(const kg_config* cfg, const kg_pod* pod, or_numa_pod* out);

/* Filter (plugin.go:276-334; filterAmplifiedCPUs :336-373 reads NodeInfo.Requested / Allocatable cpu).  Returns 1
 * when the node passes; writes the stored affinity. */
int or_numa_filter(const kg_config* cfg, const or_numa_node* n, const or_numa_pod* p, or_hint* affinity,
                   int64_t node_req_cpu, int64_t node_alloc_cpu);
/* Score (scoring.go:55-120) with the affinity Filter stored; req/alloc = NodeInfo.Requested/Allocatable. */
int64_t or_numa_score(const kg_config* cfg, const or_numa_node* n, const or_numa_pod* p, const or_hint* affinity,
                      int64_t node_req_cpu, int64_t node_req_mem, int64_t node_alloc_cpu, int64_t node_alloc_mem);
/* Reserve (plugin.go:375-415): Allocate with the stored affinity, then Update.  Returns 0 (and the cpuset in
 * *cpus) or -1 when the allocation fails (the pod is not placed). */
/* the per-pod NUMA allocation record: [0] NUMA-node bitmask, [1 + i] cpu and [1 + KG_MAX_NUMA + i] memory on NUMA i */
#define OR_NUMA_ALLOC_WORDS (1 + 2 * KG_MAX_NUMA)
int or_numa_reserve(const kg_config* cfg, or_numa_node* n, const or_numa_pod* p, const or_hint* affinity,
                    or_cpuset* cpus, int64_t* alloc);
void or_numa_release(or_numa_node* n, const or_cpuset* cpus, const int64_t* alloc);

/* (r6) NodeNUMAResource with reservations holding cpusets (nodenumaresource/reservation.go, plugin.go:465-535).
 * pref = the nominated reservation's reservedCPUs (getReservationReservedCPUs), NULL or empty = none. */
int64_t or_numa_score_pref(const kg_config* cfg, const or_numa_node* n, const or_numa_pod* p, const or_hint* affinity,
                           const or_cpuset* pref, int64_t node_req_cpu, int64_t node_req_mem, int64_t node_alloc_cpu,
                           int64_t node_alloc_mem);
int or_numa_reserve_pref(const kg_config* cfg, or_numa_node* n, const or_numa_pod* p, const or_hint* affinity,
                         const or_cpuset* pref, or_cpuset* cpus, int64_t* alloc);
/* RefCount 2 for the cpus a reservation holds that one of its assigned pods holds too (once per state) */
void or_numa_rsv_refs(or_numa_node* n, const kg_node_reservations* r);
/* RestoreReservation's reservedCPUs of reservation slot s (reservation.go:76-113): its cpuset minus its assigned pods' */
or_cpuset or_numa_rsv_reserved(const kg_node_reservations* r, int s);

#ifdef __cplusplus
}
#endif
#endif
