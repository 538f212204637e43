/*
 * numa.c — plain-C restatement of koord-scheduler's NodeNUMAResource plugin (TEST INFRASTRUCTURE ONLY).
 *
 * Restated from (paths under /root/reference):
 *   pkg/scheduler/plugins/nodenumaresource/plugin.go            PreFilter :220-270, Filter :276-373, Reserve :375-415,
 *                                                               getResourceOptions :465-511, getPreferredCPUBindPolicy :556-576
 *   pkg/scheduler/plugins/nodenumaresource/scoring.go           Score :55-120, calculateAllocatableAndRequested :122-168,
 *                                                               resourceAllocationScorer :191-230
 *   pkg/scheduler/plugins/nodenumaresource/least_allocated.go / most_allocated.go
 *   pkg/scheduler/plugins/nodenumaresource/resource_manager.go  GetTopologyHints :122-138, trim :140-169, Allocate :171-360,
 *                                                               generateResourceHints :418-532, filter/satisfied :534-589
 *   pkg/scheduler/plugins/nodenumaresource/node_allocation.go   addPodAllocation :76-103, getAvailableCPUs :133-153,
 *                                                               getAvailableNUMANodeResources :155-177
 *   pkg/scheduler/plugins/nodenumaresource/cpu_accumulator.go   takePreferredCPUs / takeCPUs / cpuAccumulator :29-822
 *   pkg/scheduler/plugins/nodenumaresource/topology_hint.go     FilterByNUMANode / GetPodTopologyHints / Allocate
 *   pkg/scheduler/plugins/nodenumaresource/util.go              AllowUseCPUSet, getNUMATopologyPolicy, skipTheNode
 *   pkg/scheduler/frameworkext/topologymanager/{manager.go :58-111, policy.go :65-224, policy_best_effort.go,
 *                                               policy_restricted.go, policy_single_numa_node.go}
 *   pkg/util/bitmask/bitmask.go                                 IterateBitMasks :206-222, IsNarrowerThan :146-151
 * Scope: maxRefCount 1, CPU amplification included, CPU exclusive policies (PCPULevel / NUMANodeLevel,
 * cpu_accumulator.go:247-330), no reservations (preferred CPUs empty), ≤ 4 NUMA nodes, ≤ 256 CPUs.  Go map iteration never decides a result here: every
 * accumulator sort ends on an ID, and the hint providers' resources are taken in sorted-name order (cpu, memory).
 */
#include "numa.h"

#include <math.h>

#include <string.h>

#define MAX_NODE_SCORE 100

/* ---------------------------------------------------------------------------------------------------- */
/* cpu sets and topology                                                                                  */
/* ---------------------------------------------------------------------------------------------------- */
static int cs_has(const or_cpuset* s, int c) { return (int)((s->w[c >> 6] >> (c & 63)) & 1u); }
static void cs_add(or_cpuset* s, int c) { s->w[c >> 6] |= 1ull << (c & 63); }
static void cs_del(or_cpuset* s, int c) { s->w[c >> 6] &= ~(1ull << (c & 63)); }
static int cs_size(const or_cpuset* s) {
  int n = 0;
  for (int i = 0; i < OR_CPUSET_WORDS; i++) n += __builtin_popcountll(s->w[i]);
  return n;
}
static or_cpuset cs_and(or_cpuset a, or_cpuset b) {
  for (int i = 0; i < OR_CPUSET_WORDS; i++) a.w[i] &= b.w[i];
  return a;
}
static or_cpuset cs_andnot(or_cpuset a, or_cpuset b) {
  for (int i = 0; i < OR_CPUSET_WORDS; i++) a.w[i] &= ~b.w[i];
  return a;
}
static or_cpuset cs_or(or_cpuset a, or_cpuset b) {
  for (int i = 0; i < OR_CPUSET_WORDS; i++) a.w[i] |= b.w[i];
  return a;
}
static or_cpuset cs_empty(void) {
  or_cpuset s;
  memset(&s, 0, sizeof(s));
  return s;
}

void or_topology_build(or_topology* t, int sockets, int nodes_per_socket, int cores_per_node, int cpus_per_core) {
  memset(t, 0, sizeof(*t));
  t->num_sockets = sockets;
  t->num_nodes = sockets * nodes_per_socket;
  t->num_cores = t->num_nodes * cores_per_node;
  t->num_cpus = t->num_cores * cpus_per_core;
  t->cpus_per_core = cpus_per_core;
  t->cores_per_node = cores_per_node;
  t->nodes_per_socket = nodes_per_socket;
  for (int c = 0; c < t->num_cpus && c < KG_MAX_CPUS; c++) cs_add(&t->all, c);
}
/* buildCPUTopologyForTest numbering (cpu_accumulator_test.go:38-55) */
static int core_of(const or_topology* t, int c) { return c / t->cpus_per_core; }
static int node_of(const or_topology* t, int c) { return c / (t->cpus_per_core * t->cores_per_node); }
static int socket_of(const or_topology* t, int c) {
  return c / (t->cpus_per_core * t->cores_per_node * t->nodes_per_socket);
}
/* CPUTopology.IsValid / CPUsPerCore / CPUsPerSocket / CPUsPerNode (cpu_topology.go:77-103) */
static int topo_valid(const or_topology* t) {
  return t->num_sockets != 0 && t->num_nodes != 0 && t->num_cores != 0 && t->num_cpus != 0;
}
static int cpus_per_core(const or_topology* t) { return t->num_cores ? t->num_cpus / t->num_cores : 0; }
static int cpus_per_socket(const or_topology* t) { return t->num_sockets ? t->num_cpus / t->num_sockets : 0; }
static int cpus_per_node(const or_topology* t) { return t->num_nodes ? t->num_cpus / t->num_nodes : 0; }
static or_cpuset cpus_in_numa(const or_topology* t, int numa) {
  or_cpuset s = cs_empty();
  for (int c = 0; c < t->num_cpus; c++)
    if (node_of(t, c) == numa) cs_add(&s, c);
  return s;
}

/* ---------------------------------------------------------------------------------------------------- */
/* cpuAccumulator (cpu_accumulator.go:234-822), maxRefCount 1                                            */
/* ---------------------------------------------------------------------------------------------------- */
typedef struct {
  const or_topology* t;
  or_cpuset allocatable;
  int needed;
  int strategy;
  or_cpuset result;
  int excl_policy;     /* KG_EXCL_* of the pod (a.exclusivePolicy) */
  or_cpuset excl_seed; /* allocated cpus holding that policy (newCPUAccumulator :256-264) */
} acc_t;

/* The cpus a filterExclusive pass skips (isCPUExclusivePCPULevel / isCPUExclusiveNUMANodeLevel :318-330): every cpu
 * of a core (PCPULevel) or NUMA node (NUMANodeLevel) in exclusiveInCores / exclusiveInNUMANodes — seeded from the
 * allocated cpus holding the pod's policy and grown by every take() of this call (:290-304).  `pcpu` / `numa`:
 * whether the calling list filters on that level (freeCoresInNode: NUMA only; freeCPUsInSocket: PCPU only;
 * freeCPUsInNode / freeCPUs: both). */
static or_cpuset acc_excluded(const acc_t* a, int pcpu, int numa) {
  or_cpuset r = cs_empty();
  const int pol = a->excl_policy;
  if (!((pol == KG_EXCL_PCPU_LEVEL && pcpu) || (pol == KG_EXCL_NUMA_NODE_LEVEL && numa))) return r;
  const or_cpuset held = cs_or(a->excl_seed, a->result);
  const or_topology* t = a->t;
  for (int c = 0; c < t->num_cpus; c++) {
    if (!cs_has(&held, c)) continue;
    if (pol == KG_EXCL_PCPU_LEVEL) {
      const int core = core_of(t, c);
      for (int q = 0; q < t->num_cpus; q++)
        if (core_of(t, q) == core) cs_add(&r, q);
    } else {
      const int node = node_of(t, c);
      for (int q = 0; q < t->num_cpus; q++)
        if (node_of(t, q) == node) cs_add(&r, q);
    }
  }
  return r;
}

typedef struct {
  int n;
  int v[KG_MAX_CPUS];
} list_t;

static void acc_take(acc_t* a, const int* cpus, int n) {
  for (int i = 0; i < n; i++) {
    cs_add(&a->result, cpus[i]);
    cs_del(&a->allocatable, cpus[i]);
  }
  a->needed -= n;
}
static int acc_needs(const acc_t* a, int n) { return a->needed >= n; }
static int acc_satisfied(const acc_t* a) { return a->needed < 1; }
static int acc_failed(const acc_t* a) { return a->needed > cs_size(&a->allocatable); }

static int core_cpus(const or_topology* t, const or_cpuset* set, int core, int* out) {
  int n = 0;
  for (int p = 0; p < t->cpus_per_core; p++) {
    const int c = core * t->cpus_per_core + p;
    if (cs_has(set, c)) out[n++] = c;
  }
  return n;
}

static int better_free(int strategy, int a, int b) { /* "a sorts before b" on a free score */
  return strategy == KG_STRATEGY_MOST_ALLOCATED ? a < b : a > b;
}

static void swap_groups(list_t* g, int* gid, int i, int j) {
  list_t tl = g[i];
  g[i] = g[j];
  g[j] = tl;
  int tg = gid[i];
  gid[i] = gid[j];
  gid[j] = tg;
}

/* freeCoresInNode(filterFullFreeCore, _) / freeCoresInSocket(filterFullFreeCore) (:371-527): per group (NUMA
 * node or socket) the cpus of its (full) free cores, cores by (free count desc, id), cpus ascending; groups by
 * (group free, [socket free for nodes], id). */
static int free_cores_in(const acc_t* a, int by_node, int full, int filter_excl, list_t* out) {
  const or_topology* t = a->t;
  const int ng = by_node ? t->num_nodes : t->num_sockets;
  /* freeCoresInNode(_, filterExclusive) skips NUMA-level exclusive cpus (:377); freeCoresInSocket never filters */
  const or_cpuset alloc = (by_node && filter_excl) ? cs_andnot(a->allocatable, acc_excluded(a, 0, 1)) : a->allocatable;
  int socket_free[KG_MAX_CPUS] = {0}, core_cnt[KG_MAX_CPUS] = {0};
  for (int c = 0; c < t->num_cpus; c++)
    if (cs_has(&alloc, c)) {
      core_cnt[core_of(t, c)]++;
      socket_free[socket_of(t, c)]++;
    }
  const int cpc = cpus_per_core(t);
  int ngroups = 0, gid[KG_MAX_CPUS];
  for (int g = 0; g < ng; g++) {
    list_t l;
    l.n = 0;
    for (int cnt = cpc; cnt >= 1; cnt--) {
      if (full && cnt != cpc) break;
      for (int core = 0; core < t->num_cores; core++) {
        if (core_cnt[core] != cnt) continue;
        int cpus[KG_MAX_CPUS];
        const int k = core_cpus(t, &alloc, core, cpus);
        const int grp = by_node ? node_of(t, cpus[0]) : socket_of(t, cpus[0]);
        if (grp != g) continue;
        for (int i = 0; i < k; i++) l.v[l.n++] = cpus[i];
      }
    }
    if (l.n == 0) continue;
    out[ngroups] = l;
    gid[ngroups++] = g;
  }
  for (int i = 0; i < ngroups; i++) { /* selection sort on a total order */
    int best = i;
    for (int j = i + 1; j < ngroups; j++) {
      int before;
      if (out[j].n != out[best].n) before = better_free(a->strategy, out[j].n, out[best].n);
      else if (by_node) {
        const int sj = socket_free[socket_of(t, out[j].v[0])], sb = socket_free[socket_of(t, out[best].v[0])];
        before = sj != sb ? better_free(a->strategy, sj, sb) : gid[j] < gid[best];
      } else {
        before = gid[j] < gid[best];
      }
      if (before) best = j;
    }
    if (best != i) swap_groups(out, gid, i, best);
  }
  return ngroups;
}

/* freeCPUsInNode / freeCPUsInSocket (:530-656): per group its free cpus ascending — with filterExclusive
 * reduced to the first cpu of each core (extractCPU :332-343); groups by (node free, socket free, id) on the
 * unreduced counts / (length of the group's list, id). */
static int free_cpus_in(const acc_t* a, int by_node, int extract, list_t* out) {
  const or_topology* t = a->t;
  const int ng = by_node ? t->num_nodes : t->num_sockets;
  /* filterExclusive (= extract): freeCPUsInNode skips PCPU- and NUMA-level exclusive cpus (:535), freeCPUsInSocket
   * PCPU-level ones (:612), before counting */
  const or_cpuset alloc = extract ? cs_andnot(a->allocatable, acc_excluded(a, 1, by_node)) : a->allocatable;
  int node_free[KG_MAX_CPUS] = {0}, socket_free[KG_MAX_CPUS] = {0};
  for (int c = 0; c < t->num_cpus; c++)
    if (cs_has(&alloc, c)) {
      node_free[node_of(t, c)]++;
      socket_free[socket_of(t, c)]++;
    }
  int ngroups = 0, gid[KG_MAX_CPUS];
  for (int g = 0; g < ng; g++) {
    list_t l;
    l.n = 0;
    int last_core = -1;
    for (int c = 0; c < t->num_cpus; c++)
      if (cs_has(&alloc, c) && (by_node ? node_of(t, c) : socket_of(t, c)) == g) {
        if (extract && core_of(t, c) == last_core) continue;
        last_core = core_of(t, c);
        l.v[l.n++] = c;
      }
    if (l.n == 0) continue;
    out[ngroups] = l;
    gid[ngroups++] = g;
  }
  for (int i = 0; i < ngroups; i++) {
    int best = i;
    for (int j = i + 1; j < ngroups; j++) {
      int before;
      if (by_node) {
        const int nj = node_free[gid[j]], nb = node_free[gid[best]];
        const int sj = socket_free[socket_of(t, out[j].v[0])], sb = socket_free[socket_of(t, out[best].v[0])];
        if (nj != nb) before = better_free(a->strategy, nj, nb);
        else if (sj != sb) before = better_free(a->strategy, sj, sb);
        else before = gid[j] < gid[best];
      } else {
        before = out[j].n != out[best].n ? better_free(a->strategy, out[j].n, out[best].n) : gid[j] < gid[best];
      }
      if (before) best = j;
    }
    if (best != i) swap_groups(out, gid, i, best);
  }
  return ngroups;
}

/* freeCPUs (:666-774): every free cpu; cores by (socket colo desc, socket free, node free, core free asc,
 * socket asc, core asc), cpus ascending within a core. */
static void free_cpus_all(const acc_t* a, int filter_excl, list_t* out) {
  const or_topology* t = a->t;
  /* freeCPUs(filterExclusive) skips PCPU- and NUMA-level exclusive cpus (:674) */
  const or_cpuset alloc = filter_excl ? cs_andnot(a->allocatable, acc_excluded(a, 1, 1)) : a->allocatable;
  int node_free[KG_MAX_CPUS] = {0}, socket_free[KG_MAX_CPUS] = {0}, core_cnt[KG_MAX_CPUS] = {0};
  int socket_colo[KG_MAX_CPUS] = {0};
  for (int c = 0; c < t->num_cpus; c++) {
    if (cs_has(&alloc, c)) {
      node_free[node_of(t, c)]++;
      socket_free[socket_of(t, c)]++;
      core_cnt[core_of(t, c)]++;
    }
    if (cs_has(&a->result, c)) socket_colo[socket_of(t, c)]++;
  }
  int cores[KG_MAX_CPUS], n = 0;
  for (int core = 0; core < t->num_cores; core++)
    if (core_cnt[core] > 0) cores[n++] = core;
  for (int i = 0; i < n; i++) {
    int best = i;
    for (int j = i + 1; j < n; j++) {
      const int cj = cores[j], cb = cores[best];
      const int fj = cj * t->cpus_per_core, fb = cb * t->cpus_per_core;
      const int sj = socket_of(t, fj), sb = socket_of(t, fb);
      const int nj = node_of(t, fj), nb = node_of(t, fb);
      int before;
      if (socket_colo[sj] != socket_colo[sb]) before = socket_colo[sj] > socket_colo[sb];
      else if (socket_free[sj] != socket_free[sb]) before = better_free(a->strategy, socket_free[sj], socket_free[sb]);
      else if (node_free[nj] != node_free[nb]) before = better_free(a->strategy, node_free[nj], node_free[nb]);
      else if (core_cnt[cj] != core_cnt[cb]) before = core_cnt[cj] < core_cnt[cb];
      else if (sj != sb) before = sj < sb;
      else before = cj < cb;
      if (before) best = j;
    }
    const int tmp = cores[i];
    cores[i] = cores[best];
    cores[best] = tmp;
  }
  out->n = 0;
  for (int i = 0; i < n; i++) {
    int cpus[KG_MAX_CPUS];
    const int k = core_cpus(t, &alloc, cores[i], cpus);
    for (int q = 0; q < k; q++) out->v[out->n++] = cpus[q];
  }
}

/* spreadCPUs (:798-822): round-robin over cores in list order */
static void spread_cpus(const acc_t* a, list_t* l) {
  if (l->n <= cpus_per_core(a->t)) return;
  list_t prepared = *l, out;
  out.n = 0;
  while (prepared.n > 0) {
    list_t reserved;
    reserved.n = 0;
    unsigned char seen[KG_MAX_CPUS] = {0};
    for (int i = 0; i < prepared.n; i++) {
      const int cpu = prepared.v[i], core = core_of(a->t, cpu);
      if (seen[core]) {
        reserved.v[reserved.n++] = cpu;
        continue;
      }
      out.v[out.n++] = cpu;
      seen[core] = 1;
    }
    prepared = reserved;
  }
  *l = out;
}

static void insertion_sort_len(list_t* g, int n, int desc) { /* stable (sort.Slice over pre-sorted groups) */
  for (int i = 1; i < n; i++) {
    list_t x = g[i];
    int j = i - 1;
    while (j >= 0 && (desc ? g[j].n < x.n : g[j].n > x.n)) {
      g[j + 1] = g[j];
      j--;
    }
    g[j + 1] = x;
  }
}

/* takeCPUs (:87-232).  0 and the set, or -1 ("not enough cpus" / "failed to allocate cpus"). */
int or_take_cpus(const or_topology* t, or_cpuset available, int needed, int bind_policy, int strategy,
                 or_cpuset* out) {
  return or_take_cpus_ex(t, available, needed, bind_policy, strategy, KG_EXCL_NONE, cs_empty(), out);
}

int or_take_cpus_ex(const or_topology* t, or_cpuset available, int needed, int bind_policy, int strategy,
                    int excl_policy, or_cpuset excl_seed, or_cpuset* out) {
  static _Thread_local list_t groups[KG_MAX_CPUS], unsat[KG_MAX_CPUS]; /* per scheduling thread */
  acc_t a;
  a.t = t;
  a.allocatable = cs_and(available, t->all);
  a.needed = needed;
  a.strategy = strategy;
  a.result = cs_empty();
  a.excl_policy = excl_policy;
  a.excl_seed = excl_seed;
  *out = cs_empty();
  if (acc_satisfied(&a)) return 0;
  if (acc_failed(&a)) return -1;
  const int cpc = cpus_per_core(t);
  const int full = bind_policy == KG_BIND_FULL_PCPUS;
  if (full || cpc == 1) {
    if (a.needed <= cpus_per_node(t)) {
      for (int fe = 0; fe < 2; fe++) { /* filterExclusive true, then false */
        const int ng = free_cores_in(&a, 1, 1, fe == 0, groups);
        for (int g = 0; g < ng; g++)
          if (groups[g].n >= a.needed) {
            acc_take(&a, groups[g].v, a.needed);
            *out = a.result;
            return 0;
          }
      }
    }
    if (a.needed <= cpus_per_socket(t)) {
      const int ng = free_cores_in(&a, 0, 1, 0, groups);
      for (int g = 0; g < ng; g++)
        if (groups[g].n >= a.needed) {
          acc_take(&a, groups[g].v, a.needed);
          *out = a.result;
          return 0;
        }
    }
    int ng = free_cores_in(&a, 0, 1, 0, groups);
    insertion_sort_len(groups, ng, 1);
    int nu = 0;
    for (int g = 0; g < ng; g++) {
      if (!acc_needs(&a, groups[g].n)) {
        unsat[nu++] = groups[g];
      } else {
        acc_take(&a, groups[g].v, groups[g].n);
        if (acc_satisfied(&a)) {
          *out = a.result;
          return 0;
        }
      }
    }
    if (acc_needs(&a, cpc)) {
      insertion_sort_len(unsat, nu, 0);
      for (int g = 0; g < nu; g++) {
        for (int i = 0; i < unsat[g].n; i += cpc) {
          acc_take(&a, &unsat[g].v[i], cpc);
          if (acc_satisfied(&a)) {
            *out = a.result;
            return 0;
          }
          if (!acc_needs(&a, cpc)) break;
        }
      }
    }
  }
  if (!full) {
    if (a.needed <= cpus_per_node(t)) {
      for (int fe = 0; fe < 2; fe++) { /* filterExclusive true (one cpu per core), then false */
        const int ng = free_cpus_in(&a, 1, fe == 0, groups);
        for (int g = 0; g < ng; g++)
          if (groups[g].n >= a.needed) {
            spread_cpus(&a, &groups[g]);
            acc_take(&a, groups[g].v, a.needed);
            *out = a.result;
            return 0;
          }
      }
    }
    if (a.needed <= cpus_per_socket(t)) {
      for (int fe = 0; fe < 2; fe++) {
        const int ng = free_cpus_in(&a, 0, fe == 0, groups);
        for (int g = 0; g < ng; g++)
          if (groups[g].n >= a.needed) {
            spread_cpus(&a, &groups[g]);
            acc_take(&a, groups[g].v, a.needed);
            *out = a.result;
            return 0;
          }
      }
    }
  }
  for (int fe = 0; fe < 2; fe++) {
    list_t l;
    free_cpus_all(&a, fe == 0, &l);
    spread_cpus(&a, &l);
    for (int i = 0; i < l.n; i++) {
      if (acc_needs(&a, 1)) acc_take(&a, &l.v[i], 1);
      if (acc_satisfied(&a)) {
        *out = a.result;
        return 0;
      }
    }
  }
  *out = cs_empty();
  return -1;
}

/* filterCPUsByRequiredCPUBindPolicy (resource_manager.go:534-566) */
or_cpuset or_filter_required(const or_topology* t, or_cpuset available, int policy) {
  if (policy != KG_BIND_FULL_PCPUS && policy != KG_BIND_SPREAD_BY_PCPUS) return available;
  or_cpuset r = cs_empty();
  const int cpc = cpus_per_core(t);
  for (int core = 0; core < t->num_cores; core++) {
    int cpus[KG_MAX_CPUS];
    const int k = core_cpus(t, &available, core, cpus);
    if (k == 0) continue;
    if (policy == KG_BIND_FULL_PCPUS) {
      if (k == cpc)
        for (int i = 0; i < k; i++) cs_add(&r, cpus[i]);
    } else {
      cs_add(&r, cpus[0]);
    }
  }
  return r;
}

/* satisfiedRequiredCPUBindPolicy (resource_manager.go:568-589) */
static int satisfied_required(const or_topology* t, or_cpuset cpus, int policy) {
  if (policy != KG_BIND_FULL_PCPUS && policy != KG_BIND_SPREAD_BY_PCPUS) return 1;
  int ncores = 0;
  for (int core = 0; core < t->num_cores; core++) {
    int tmp[KG_MAX_CPUS];
    if (core_cpus(t, &cpus, core, tmp) > 0) ncores++;
  }
  if (policy == KG_BIND_FULL_PCPUS) return ncores * cpus_per_core(t) == cs_size(&cpus);
  return ncores == cs_size(&cpus);
}

/* ---------------------------------------------------------------------------------------------------- */
/* state                                                                                                  */
/* ---------------------------------------------------------------------------------------------------- */
void or_numa_node_init(or_numa_node* n, const kg_node_numa* s) {
  memset(n, 0, sizeof(*n));
  n->has_topology = s->has_topology != 0;
  if (n->has_topology)
    or_topology_build(&n->topo, (int)s->sockets, (int)s->nodes_per_socket, (int)s->cores_per_node,
                      (int)s->cpus_per_core);
  n->valid_topology = n->has_topology && topo_valid(&n->topo);
  n->numa_policy = (int)s->numa_policy;
  n->node_cpu_bind_policy = (int)s->node_cpu_bind_policy;
  n->numa_allocate_strategy = (int)s->numa_allocate_strategy;
  n->num_numa = (int)s->num_numa;
  n->cpu_amp = s->cpu_amplification_ratio;
  for (int i = 0; i < KG_MAX_NUMA; i++) {
    n->numa_cpu[i] = s->numa_cpu[i];
    n->numa_mem[i] = s->numa_mem[i];
    n->numa_alloc_cpu[i] = s->numa_alloc_cpu[i];
    n->numa_alloc_mem[i] = s->numa_alloc_mem[i];
    n->numa_alloc_present[i] = s->numa_alloc_cpu[i] != 0 || s->numa_alloc_mem[i] != 0;
  }
  for (int i = 0; i < OR_CPUSET_WORDS; i++) {
    n->reserved.w[i] = s->reserved_cpus[i];
    n->allocated.w[i] = s->allocated_cpus[i];
    n->excl_pcpu.w[i] = s->exclusive_pcpu_cpus[i] & s->allocated_cpus[i];
    n->excl_numa.w[i] = s->exclusive_numa_cpus[i] & s->allocated_cpus[i];
  }
  for (int c = 0; c < KG_MAX_CPUS; c++) n->ref[c] = (uint8_t)cs_has(&n->allocated, c);
  n->refs_ready = 0;
}

/* (r6) A cpu a reservation holds (GetAllocatedCPUSet(node, reservation UID)) that one of its assigned pods took from
 * the reservation's reserved cpus was added twice (addPodAllocation, node_allocation.go:76-103): RefCount 2. */
void or_numa_rsv_refs(or_numa_node* n, const kg_node_reservations* r) {
  if (n->refs_ready || !r) return;
  n->refs_ready = 1;
  for (int s = 0; s < (int)r->n && s < KG_MAX_RSV_SLOTS; s++)
    for (int c = 0; c < KG_MAX_CPUS; c++)
      if (((r->cpus[s][c >> 6] >> (c & 63)) & 1u) && ((r->cpus_assigned[s][c >> 6] >> (c & 63)) & 1u) &&
          n->ref[c] == 1)
        n->ref[c] = 2;
}

/* (r6) RestoreReservation (nodenumaresource/reservation.go:76-113): the reservation's allocated cpus, minus each
 * assigned pod's (allocatedCPUs.Difference(podCPUs) over rInfo.AssignedPods) */
or_cpuset or_numa_rsv_reserved(const kg_node_reservations* r, int s) {
  or_cpuset c;
  for (int w = 0; w < OR_CPUSET_WORDS; w++) c.w[w] = r->cpus[s][w] & ~r->cpus_assigned[s][w];
  return c;
}

/* AllowUseCPUSet (util.go:42-49) + PreFilter (plugin.go:220-270) */
void or_numa_pod_init(const kg_config* cfg, const kg_pod* pod, or_numa_pod* p) {
  memset(p, 0, sizeof(*p));
  p->req_cpu = pod->requests[KG_RES_CPU];
  p->req_mem = pod->requests[KG_RES_MEMORY];
  const int allow = (pod->qos == KG_QOS_LSE || pod->qos == KG_QOS_LSR) && pod->priority_class == KG_PRIO_PROD;
  p->allow_cpuset = allow; /* PreRestoreReservation (reservation.go:68-74) */
  int zero = 1;
  for (int r = 0; r < KG_RES_MAX; r++) zero &= pod->requests[r] == 0;
  if (zero) {
    p->skip = 1;
    return;
  }
  if (!allow) return;
  int bind = (int)pod->preferred_cpu_bind_policy;
  if (bind == KG_BIND_NONE || bind == KG_BIND_DEFAULT) bind = (int)cfg->numa_default_cpu_bind_policy;
  int required = (int)pod->required_cpu_bind_policy;
  if (required == KG_BIND_DEFAULT) required = (int)cfg->numa_default_cpu_bind_policy;
  if (required != KG_BIND_NONE) bind = required;
  if (bind == KG_BIND_FULL_PCPUS || bind == KG_BIND_SPREAD_BY_PCPUS) {
    if (p->req_cpu % 1000 != 0) {
      p->prefilter_error = 1; /* "the requested CPUs must be integer" */
      return;
    }
    if (p->req_cpu > 0) {
      p->request_cpu_bind = 1;
      p->required_policy = required;
      p->preferred_policy = bind;
      p->num_cpus_needed = (int)(p->req_cpu / 1000);
      p->excl_policy = (int)pod->preferred_cpu_exclusive_policy; /* plugin.go:261 */
    }
  }
}

static int skip_the_node(const or_numa_pod* p, int policy) {
  return p->skip || (!p->request_cpu_bind && policy == KG_NUMA_POLICY_NONE);
}

/* getPreferredCPUBindPolicy (plugin.go:556-576); -1 when the topology is missing or invalid */
static int preferred_bind(const or_numa_node* n, int preferred) {
  if (!n->valid_topology) return -1;
  if (n->node_cpu_bind_policy == KG_NODE_BIND_SPREAD_BY_PCPUS) return KG_BIND_SPREAD_BY_PCPUS;
  if (n->node_cpu_bind_policy == KG_NODE_BIND_FULL_PCPUS_ONLY) return KG_BIND_FULL_PCPUS;
  return preferred;
}

static int allocate_strategy(const kg_config* cfg, const or_numa_node* n) {
  if (n->numa_allocate_strategy >= 0) return n->numa_allocate_strategy;
  return cfg->numa_numa_scoring_strategy == KG_STRATEGY_MOST_ALLOCATED ? KG_STRATEGY_MOST_ALLOCATED
                                                                        : KG_STRATEGY_LEAST_ALLOCATED;
}

/* getAvailableCPUs (node_allocation.go:133-153), preferred empty, maxRefCount 1 */
static or_cpuset available_cpus(const or_numa_node* n) {
  return cs_andnot(cs_andnot(n->topo.all, n->allocated), n->reserved);
}

/* (r6) getAvailableCPUs (node_allocation.go:133-153) with preferredCPUs, maxRefCount 1: on a copy of the allocated
 * CPUInfos every preferred cpu's RefCount drops by one (deleted at 0); the cpus still at RefCount ≥ maxRefCount are
 * unavailable, and so are the kubelet-reserved ones.  *held = the copy's cpus (the allocateInfo CPUDetails). */
static or_cpuset available_pref(const or_numa_node* n, const or_cpuset* pref, or_cpuset* held) {
  or_cpuset h = cs_empty();
  for (int c = 0; c < KG_MAX_CPUS; c++) {
    int r = n->ref[c];
    if (pref && r > 0 && cs_has(pref, c)) r--;
    if (r >= 1) cs_add(&h, c);
  }
  if (held) *held = h;
  return cs_andnot(cs_andnot(n->topo.all, h), n->reserved);
}

static int cs_nonempty(const or_cpuset* s) { return s && cs_size(s) > 0; }

/* extension.Amplify (apis/extension/node_resource_amplification.go:170-175) */
static int64_t amplify(int64_t origin, double ratio) {
  if (ratio <= 1) return origin;
  return (int64_t)ceil((double)origin * ratio);
}

/* getResourceOptions (plugin.go:470-510): a cpu-bind pod's cpu request is amplified by the node's cpu ratio
 * (AmplifyResourceList) for the hints, the NUMA allocation and the score */
static int64_t opt_req_cpu(const or_numa_node* n, const or_numa_pod* p) {
  return (p->request_cpu_bind && n->cpu_amp > 1) ? amplify(p->req_cpu, n->cpu_amp) : p->req_cpu;
}

/* allocatedResources[i] cpu as getAvailableNUMANodeResources sees it (node_allocation.go:155-177): with a cpu
 * ratio > 1 the cpuset part (allocated cpus on NUMA node i × 1000) counts amplified; 0 when no entry */
static int64_t numa_allocated_cpu(const or_numa_node* n, int i) {
  if (!n->numa_alloc_present[i]) return 0;
  int64_t c = n->numa_alloc_cpu[i];
  if (n->cpu_amp > 1) {
    const or_cpuset in = cs_and(n->allocated, cpus_in_numa(&n->topo, i));
    const int64_t sets = (int64_t)cs_size(&in) * 1000;
    c = c - sets + amplify(sets, n->cpu_amp);
  }
  return c;
}

/* (r6) getResourceOptions' reusableResources (plugin.go:482-493): per NUMA node holding a preferred cpu (CPUDetails.
 * KeepOnly), Amplify(its preferred cpus × 1000) of cpu; 0 elsewhere */
static int64_t reusable_cpu(const or_numa_node* n, const or_cpuset* pref, int i) {
  if (!cs_nonempty(pref)) return 0;
  const or_cpuset in = cs_and(cs_and(*pref, n->topo.all), cpus_in_numa(&n->topo, i));
  const int k = cs_size(&in);
  return k > 0 ? amplify((int64_t)k * 1000, n->cpu_amp) : 0;
}

/* allocatedResources[i] cpu after SubtractWithNonNegativeResult(allocatedRes, reusableResources[i]) (:166) */
static int64_t numa_allocated_cpu_pref(const or_numa_node* n, const or_cpuset* pref, int i) {
  const int64_t ac = numa_allocated_cpu(n, i) - reusable_cpu(n, pref, i);
  return ac > 0 ? ac : 0;
}

/* getAvailableNUMANodeResources (node_allocation.go:155-177); (r6) with the reusable cpu of preferred cpus */
static void numa_available(const or_numa_node* n, const or_cpuset* pref, int64_t avail_cpu[], int64_t avail_mem[]) {
  for (int i = 0; i < n->num_numa; i++) {
    const int64_t ac = n->numa_alloc_present[i] ? numa_allocated_cpu_pref(n, pref, i) : 0;
    const int64_t am = n->numa_alloc_present[i] ? n->numa_alloc_mem[i] : 0;
    avail_cpu[i] = n->numa_cpu[i] - ac > 0 ? n->numa_cpu[i] - ac : 0;
    avail_mem[i] = n->numa_mem[i] - am > 0 ? n->numa_mem[i] - am : 0;
  }
}

/* resourceAllocationScorer.score (scoring.go:191-230) with least/mostResourceScorer */
static int64_t least_requested(int64_t requested, int64_t capacity) {
  if (capacity == 0 || requested > capacity) return 0;
  return ((capacity - requested) * MAX_NODE_SCORE) / capacity;
}
static int64_t most_requested(int64_t requested, int64_t capacity) {
  if (capacity == 0) return 0;
  if (requested > capacity) requested = capacity;
  return (requested * MAX_NODE_SCORE) / capacity;
}
static int64_t scorer(int strategy, const int64_t w[2], int64_t req_cpu, int64_t req_mem, int64_t alloc_cpu,
                      int64_t alloc_mem, int64_t pod_cpu, int64_t pod_mem) {
  int64_t node_score = 0, wsum = 0;
  const int64_t alloc[2] = {alloc_cpu, alloc_mem}, req[2] = {req_cpu + pod_cpu, req_mem + pod_mem};
  for (int r = 0; r < 2; r++) {
    if (w[r] == 0 || alloc[r] == 0) continue; /* only resources in the weight map; zero allocatable skipped */
    const int64_t s = strategy == KG_STRATEGY_MOST_ALLOCATED ? most_requested(req[r], alloc[r])
                                                              : least_requested(req[r], alloc[r]);
    node_score += s * w[r];
    wsum += w[r];
  }
  return wsum ? node_score / wsum : 0;
}

/* ---------------------------------------------------------------------------------------------------- */
/* topology hints and the topology manager                                                                */
/* ---------------------------------------------------------------------------------------------------- */
typedef struct {
  int n;
  or_hint h[16];
} hint_list;

/* trimNUMANodeResources (resource_manager.go:140-169) */
static void trim_numa(const or_numa_node* n, int bind, int64_t avail_cpu[]) {
  const or_cpuset avail = available_cpus(n);
  for (int i = 0; i < n->num_numa; i++) {
    if (avail_cpu[i] == 0) continue;
    or_cpuset in_node = cs_and(avail, cpus_in_numa(&n->topo, i));
    if ((int64_t)cs_size(&in_node) * 1000 >= avail_cpu[i]) in_node = or_filter_required(&n->topo, in_node, bind);
    if ((int64_t)cs_size(&in_node) * 1000 < avail_cpu[i]) avail_cpu[i] = (int64_t)cs_size(&in_node) * 1000;
  }
}

/* GetPodTopologyHints → GetTopologyHints → generateResourceHints (resource_manager.go:122-138, 418-532).
 * Returns 0 with the per-resource lists (has_* = the resource key is present in the provider's map), or -1
 * when the provider returns an error (no hints: treated as "no preference" by the policy). */
static int numa_hints(const kg_config* cfg, const or_numa_node* n, const or_numa_pod* p, hint_list* hc,
                      int* has_c, hint_list* hm, int* has_m) {
  hc->n = hm->n = 0;
  *has_c = *has_m = 0;
  const int bind = preferred_bind(n, p->preferred_policy);
  if (bind < 0) return -1; /* getResourceOptions error */
  if (n->num_numa == 0) return -1;
  int64_t avail_cpu[KG_MAX_NUMA], avail_mem[KG_MAX_NUMA];
  numa_available(n, NULL, avail_cpu, avail_mem);
  if (p->request_cpu_bind && p->required_policy != KG_BIND_NONE) trim_numa(n, bind, avail_cpu);
  const int req_c = p->req_cpu > 0, req_m = p->req_mem > 0; /* keys of PodRequestsAndLimits */
  int min_c = n->num_numa, min_m = n->num_numa;
  const int64_t wn[2] = {cfg->numa_numa_scoring_weights[0], cfg->numa_numa_scoring_weights[1]};
  /* IterateBitMasks (bitmask.go:206-222): every subset by size, then lexicographic */
  uint32_t masks[16];
  int nm = 0;
  for (int size = 1; size <= n->num_numa; size++)
    for (uint32_t m = 1; m < (1u << n->num_numa); m++)
      if (__builtin_popcount(m) == size) masks[nm++] = m;
  /* lexicographic order of the bit lists inside one size: sort masks of equal size by their bit lists */
  for (int i = 0; i < nm; i++)
    for (int j = i + 1; j < nm; j++) {
      if (__builtin_popcount(masks[i]) != __builtin_popcount(masks[j])) continue;
      /* compare ascending bit lists */
      uint32_t a = masks[i], b = masks[j];
      int swap = 0;
      while (a && b) {
        const int ba = __builtin_ctz(a), bb = __builtin_ctz(b);
        if (ba != bb) {
          swap = bb < ba;
          break;
        }
        a &= a - 1;
        b &= b - 1;
      }
      if (swap) {
        const uint32_t t = masks[i];
        masks[i] = masks[j];
        masks[j] = t;
      }
    }
  for (int k = 0; k < nm; k++) {
    const uint32_t m = masks[k];
    int64_t av_c = 0, av_m = 0, tot_c = 0, tot_m = 0;
    for (int i = 0; i < n->num_numa; i++)
      if ((m >> i) & 1) {
        av_c += avail_cpu[i];
        av_m += avail_mem[i];
        tot_c += n->numa_cpu[i];
        tot_m += n->numa_mem[i];
      }
    const int64_t rq_c = tot_c - av_c > 0 ? tot_c - av_c : 0, rq_m = tot_m - av_m > 0 ? tot_m - av_m : 0;
    const int64_t score = scorer((int)cfg->numa_numa_scoring_strategy, wn, rq_c, rq_m, tot_c, tot_m, opt_req_cpu(n, p),
                                 p->req_mem);
    const int cnt = __builtin_popcount(m);
    /* generateHints(mask, ..., memory) then (..., cpu): total ≥ request gates the min affinity size, free ≥
     * request gates the hint */
    if (req_m && tot_m >= p->req_mem) {
      if (cnt < min_m) min_m = cnt;
      if (av_m >= p->req_mem) {
        or_hint h = {0, m, 0, score};
        hm->h[hm->n++] = h;
      }
    }
    if (req_c && tot_c >= opt_req_cpu(n, p)) {
      if (cnt < min_c) min_c = cnt;
      if (av_c >= opt_req_cpu(n, p)) {
        or_hint h = {0, m, 0, score};
        hc->h[hc->n++] = h;
      }
    }
  }
  for (int i = 0; i < hc->n; i++) hc->h[i].preferred = __builtin_popcount(hc->h[i].mask) == min_c;
  for (int i = 0; i < hm->n; i++) hm->h[i].preferred = __builtin_popcount(hm->h[i].mask) == min_m;
  /* keys: every requested resource the NUMA zones define (cpu, memory here) */
  *has_c = req_c;
  *has_m = req_m;
  return 0;
}

/* IsNarrowerThan (bitmask.go:146-151) */
static int narrower(uint32_t a, uint32_t b) {
  const int ca = __builtin_popcount(a), cb = __builtin_popcount(b);
  return ca == cb ? a < b : ca < cb;
}

/* mergeFilteredHints (policy.go:127-185) over the permutations of `lists` (iterateAllProviderTopologyHints) */
static or_hint merge_filtered(uint32_t def, hint_list* lists, int nl) {
  or_hint best = {0, def, 0, 0};
  int idx[8] = {0};
  for (int i = 0; i < nl; i++)
    if (lists[i].n == 0) return best; /* an empty provider list: no permutation at all */
  for (;;) {
    /* mergePermutation */
    int preferred = 1;
    uint32_t merged = def;
    for (int i = 0; i < nl; i++) {
      const or_hint* h = &lists[i].h[idx[i]];
      merged &= h->nil ? def : h->mask;
      if (!h->preferred) preferred = 0;
    }
    if (merged != 0) {
      int64_t score = 0;
      for (int i = 0; i < nl; i++) {
        const or_hint* h = &lists[i].h[idx[i]];
        if (!h->nil && h->mask == merged && h->score > score) score = h->score;
      }
      const or_hint mh = {0, merged, preferred, score};
      if (mh.preferred && !best.preferred) {
        best = mh;
      } else if (!mh.preferred && best.preferred) {
        /* never replace a preferred hint */
      } else if (!narrower(mh.mask, best.mask)) {
        if (__builtin_popcount(mh.mask) == __builtin_popcount(best.mask) && mh.score > best.score) best = mh;
      } else {
        best = mh;
      }
    }
    /* next permutation: the last provider list varies fastest */
    int i = nl - 1;
    while (i >= 0 && ++idx[i] == lists[i].n) idx[i--] = 0;
    if (i < 0) break;
  }
  return best;
}

/* filterSingleNumaHints (policy_single_numa_node.go:38-53): keep "don't care" and single-NUMA hints, preferred only */
static void single_numa_filter(hint_list* lists, int nl) {
  for (int i = 0; i < nl; i++) {
    int k = 0;
    for (int j = 0; j < lists[i].n; j++) {
      const or_hint h = lists[i].h[j];
      if ((h.nil && h.preferred) || (!h.nil && __builtin_popcount(h.mask) == 1 && h.preferred)) lists[i].h[k++] = h;
    }
    lists[i].n = k;
  }
}

/* Policy.Merge + canAdmitPodResult over filtered provider lists (policy_best_effort.go:43-48,
 * policy_restricted.go:41-46, policy_single_numa_node.go:62-77).  Returns admit. */
static int policy_merge_lists(int policy, uint32_t def, hint_list* lists, int nl, or_hint* best) {
  if (policy == KG_NUMA_POLICY_SINGLE_NUMA_NODE) {
    single_numa_filter(lists, nl);
    *best = merge_filtered(def, lists, nl);
    if (!best->nil && best->mask == def) *best = (or_hint){1, 0, best->preferred, 0};
    return best->preferred;
  }
  *best = merge_filtered(def, lists, nl);
  if (policy == KG_NUMA_POLICY_RESTRICTED) return best->preferred;
  return 1; /* best-effort */
}

/* Policy.Merge for the NodeNUMAResource provider alone (manager.go:82-100; policy_*.go).  Returns admit. */
static int policy_merge(const or_numa_node* n, int hints_ok, hint_list* hc, int has_c, hint_list* hm, int has_m,
                        or_hint* best) {
  const uint32_t def = (1u << n->num_numa) - 1;
  hint_list lists[2];
  int nl = 0;
  /* filterProvidersHints (policy.go:94-125): no hints → one preferred any-NUMA hint; a present but empty list
   * → one non-preferred any-NUMA hint; resources in sorted-name order */
  if (!hints_ok || (!has_c && !has_m)) {
    lists[0].n = 1;
    lists[0].h[0] = (or_hint){1, 0, 1, 0};
    nl = 1;
  } else {
    if (has_c) {
      lists[nl] = *hc;
      if (hc->n == 0) {
        lists[nl].n = 1;
        lists[nl].h[0] = (or_hint){1, 0, 0, 0};
      }
      nl++;
    }
    if (has_m) {
      lists[nl] = *hm;
      if (hm->n == 0) {
        lists[nl].n = 1;
        lists[nl].h[0] = (or_hint){1, 0, 0, 0};
      }
      nl++;
    }
  }
  return policy_merge_lists(n->numa_policy, def, lists, nl, best);
}

/* ---------------------------------------------------------------------------------------------------- */
/* Allocate (resource_manager.go:171-360)                                                                 */
/* ---------------------------------------------------------------------------------------------------- */
typedef struct {
  int n;
  int numa[KG_MAX_NUMA];
  int64_t cpu[KG_MAX_NUMA], mem[KG_MAX_NUMA];
} numa_alloc;

/* the node's allocated cpus holding the pod's exclusive policy (GetAvailableCPUs' allocatedCPUs → newCPUAccumulator) */
static or_cpuset excl_seed(const or_numa_node* n, const or_numa_pod* p) {
  if (p->excl_policy == KG_EXCL_PCPU_LEVEL) return n->excl_pcpu;
  if (p->excl_policy == KG_EXCL_NUMA_NODE_LEVEL) return n->excl_numa;
  return cs_empty();
}

/* takePreferredCPUs (cpu_accumulator.go:33-85): the preferred cpus among the available ones first (as many as are
 * needed, one takeCPUs over them), then the rest from the other available cpus */
static int take_preferred(const or_topology* t, or_cpuset avail, const or_cpuset* pref, int needed, int bind,
                          int strategy, int excl, or_cpuset seed, or_cpuset* out) {
  or_cpuset result = cs_empty();
  const or_cpuset pc = pref ? cs_and(avail, *pref) : cs_empty();
  if (cs_size(&pc) > 0) {
    const int k = needed < cs_size(&pc) ? needed : cs_size(&pc);
    if (or_take_cpus_ex(t, pc, k, bind, strategy, excl, seed, &result) != 0) return -1;
    needed -= cs_size(&result);
    avail = cs_andnot(avail, pc);
  }
  if (needed > 0) {
    or_cpuset got;
    if (or_take_cpus_ex(t, avail, needed, bind, strategy, excl, seed, &got) != 0) return -1;
    result = cs_or(result, got);
  }
  *out = result;
  return 0;
}

/* resourceManager.Allocate (resource_manager.go:171-360); (r6) pref = ResourceOptions.preferredCPUs (the nominated
 * reservation's reserved cpus; NULL / empty = none), which also makes its NUMA cpu reusable */
static int allocate(const kg_config* cfg, const or_numa_node* n, const or_numa_pod* p, const or_hint* hint,
                    const or_cpuset* pref, numa_alloc* res, or_cpuset* cpus) {
  res->n = 0;
  *cpus = cs_empty();
  if (!cs_nonempty(pref)) pref = NULL;
  const int bind = preferred_bind(n, p->preferred_policy);
  if (bind < 0) return -1; /* getResourceOptions error */
  if (!hint->nil) {
    /* allocateResourcesByHint (:195-250) */
    if (n->num_numa == 0) return -1;
    int64_t avail_cpu[KG_MAX_NUMA], avail_mem[KG_MAX_NUMA];
    numa_available(n, pref, avail_cpu, avail_mem);
    /* a cpu-bind pod splits its ORIGINAL (un-amplified) requests (:205-210: options.originalRequests); any other
     * pod's requests are never amplified, so the plain request is right for both */
    int64_t rq_c = p->req_cpu, rq_m = p->req_mem;
    const int key_c = p->req_cpu > 0, key_m = p->req_mem > 0;
    int inter_c = 0, inter_m = 0;
    for (int i = 0; i < n->num_numa; i++) {
      if (!((hint->mask >> i) & 1)) continue;
      int64_t ac = 0, am = 0;
      if (key_c) { /* every NUMA zone defines cpu and memory */
        inter_c = 1;
        ac = rq_c < avail_cpu[i] ? rq_c : avail_cpu[i];
        rq_c -= ac;
      }
      if (key_m) {
        inter_m = 1;
        am = rq_m < avail_mem[i] ? rq_m : avail_mem[i];
        rq_m -= am;
      }
      if (ac != 0 || am != 0) {
        res->numa[res->n] = i;
        res->cpu[res->n] = ac;
        res->mem[res->n] = am;
        res->n++;
      }
      if (rq_c == 0 && rq_m == 0) break;
    }
    if ((inter_c && rq_c != 0) || (inter_m && rq_m != 0)) return -1; /* Insufficient NUMA cpu/memory */
  }
  if (p->request_cpu_bind) {
    /* allocateCPUSet (:273-360): GetAvailableCPUs(node, preferredCPUs), then per NUMA node of the allocation (or once)
     * takePreferredCPUs */
    or_cpuset held = n->allocated;
    or_cpuset avail = pref ? available_pref(n, pref, &held) : available_cpus(n);
    const int required = p->required_policy != KG_BIND_NONE;
    if (required) avail = or_filter_required(&n->topo, avail, bind);
    if (cs_size(&avail) < p->num_cpus_needed) return -1;
    const int strategy = allocate_strategy(cfg, n);
    const or_cpuset seed = cs_and(excl_seed(n, p), held); /* the allocateInfo the accumulator seeds from */
    int needed = p->num_cpus_needed;
    or_cpuset result = cs_empty();
    if (res->n > 0) {
      for (int k = 0; k < res->n; k++) {
        const or_cpuset in_node = cs_and(avail, cpus_in_numa(&n->topo, res->numa[k]));
        int num = cs_size(&in_node);
        const int node_need = (int)(res->cpu[k] / 1000);
        if (node_need < num) num = node_need;
        or_cpuset got;
        if (take_preferred(&n->topo, in_node, pref, num, bind, strategy, p->excl_policy, seed, &got) != 0) return -1;
        result = cs_or(result, got);
      }
      needed -= cs_size(&result);
      if (needed != 0) return -1;
    }
    if (needed > 0) {
      or_cpuset got;
      if (take_preferred(&n->topo, cs_andnot(avail, result), pref, needed, bind, strategy, p->excl_policy, seed,
                         &got) != 0)
        return -1;
      result = cs_or(result, got);
    }
    if (required && !satisfied_required(&n->topo, result, bind)) return -1;
    *cpus = result;
  }
  return 0;
}

/* ---------------------------------------------------------------------------------------------------- */
/* plugin extension points                                                                                */
/* ---------------------------------------------------------------------------------------------------- */
int or_numa_filter(const kg_config* cfg, const or_numa_node* n, const or_numa_pod* p, or_hint* affinity,
                   int64_t node_req_cpu, int64_t node_alloc_cpu) {
  *affinity = (or_hint){1, 0, 0, 0};
  if (p->prefilter_error) return 0;
  if (p->req_cpu != 0 && n->cpu_amp > 1) { /* filterAmplifiedCPUs (plugin.go:336-373) */
    const int64_t pod = p->request_cpu_bind ? amplify(p->req_cpu, n->cpu_amp) : p->req_cpu;
    /* GetAvailableCPUs fails without a valid topology: no allocated cpus */
    const int64_t am = (n->has_topology && n->valid_topology) ? (int64_t)cs_size(&n->allocated) * 1000 : 0;
    int64_t req = node_req_cpu;
    if (req >= am && am > 0) req = req - am + amplify(am, n->cpu_amp);
    if (pod > node_alloc_cpu - req) return 0; /* ErrInsufficientAmplifiedCPU */
  }
  const int policy = n->numa_policy;
  if (skip_the_node(p, policy)) return 1;
  if (p->request_cpu_bind) {
    if (!n->has_topology || !n->valid_topology) return 0; /* ErrNotFoundCPUTopology / ErrInvalidCPUTopology */
    const int full_only = n->node_cpu_bind_policy == KG_NODE_BIND_FULL_PCPUS_ONLY;
    if (full_only || p->required_policy == KG_BIND_FULL_PCPUS) {
      if (p->num_cpus_needed % cpus_per_core(&n->topo) != 0) return 0; /* ErrSMTAlignmentError */
      if (full_only && (p->required_policy != KG_BIND_FULL_PCPUS || p->preferred_policy != KG_BIND_FULL_PCPUS))
        return 0; /* ErrRequiredFullPCPUsPolicy */
    }
    if (p->required_policy != KG_BIND_NONE && policy == KG_NUMA_POLICY_NONE) {
      numa_alloc res;
      or_cpuset cpus;
      const or_hint none = {1, 0, 0, 0};
      if (allocate(cfg, n, p, &none, NULL, &res, &cpus) != 0) return 0;
    }
  }
  if (policy != KG_NUMA_POLICY_NONE) {
    /* FilterByNUMANode → RunNUMATopologyManagerAdmit (topology_hint.go:30-39, manager.go:58-80) */
    if (n->num_numa == 0) return 0; /* node(s) missing NUMA resources */
    hint_list hc, hm;
    int has_c, has_m;
    const int ok = numa_hints(cfg, n, p, &hc, &has_c, &hm, &has_m) == 0;
    or_hint best;
    if (!policy_merge(n, ok, &hc, has_c, &hm, has_m, &best)) return 0; /* NUMA Topology affinity error */
    *affinity = best;
    numa_alloc res;
    or_cpuset cpus;
    if (allocate(cfg, n, p, &best, NULL, &res, &cpus) != 0) return 0;
  }
  return 1;
}

int64_t or_numa_score(const kg_config* cfg, const or_numa_node* n, const or_numa_pod* p, const or_hint* affinity,
                      int64_t node_req_cpu, int64_t node_req_mem, int64_t node_alloc_cpu, int64_t node_alloc_mem) {
  return or_numa_score_pref(cfg, n, p, affinity, NULL, node_req_cpu, node_req_mem, node_alloc_cpu, node_alloc_mem);
}

int64_t or_numa_score_pref(const kg_config* cfg, const or_numa_node* n, const or_numa_pod* p, const or_hint* affinity,
                           const or_cpuset* pref, int64_t node_req_cpu, int64_t node_req_mem, int64_t node_alloc_cpu,
                           int64_t node_alloc_mem) {
  const int64_t w[2] = {cfg->numa_scoring_weights[0], cfg->numa_scoring_weights[1]};
  const int strategy = (int)cfg->numa_scoring_strategy;
  const int policy = n->numa_policy;
  if (!cs_nonempty(pref)) pref = NULL;
  if (skip_the_node(p, policy)) {
    if (p->skip) return 0;
    /* scoreWithAmplifiedCPUs (:95-120): getResourceOptions needs a valid topology */
    if (preferred_bind(n, p->preferred_policy) < 0) return 0;
    int64_t rc = node_req_cpu;
    if (p->req_cpu != 0 && n->cpu_amp > 1) { /* the cpuset part of Requested counts amplified */
      /* GetAvailableCPUs(node, preferredCPUs): the allocated CPUDetails after the preferred cpus' RefCount drop */
      or_cpuset held = n->allocated;
      if (pref) available_pref(n, pref, &held);
      const int64_t am = (int64_t)cs_size(&held) * 1000;
      rc = rc - am + amplify(am, n->cpu_amp);
    }
    return scorer(strategy, w, rc, node_req_mem, node_alloc_cpu, node_alloc_mem, p->req_cpu, p->req_mem);
  }
  if (p->request_cpu_bind && (!n->has_topology || !n->valid_topology)) return 0;
  numa_alloc res;
  or_cpuset cpus;
  if (allocate(cfg, n, p, affinity, pref, &res, &cpus) != 0) return 0;
  /* calculateAllocatableAndRequested (:122-168) */
  int64_t alloc_c, alloc_m, req_c, req_m;
  if (res.n > 0) {
    alloc_c = alloc_m = req_c = req_m = 0;
    for (int k = 0; k < res.n; k++) {
      const int i = res.numa[k];
      if (n->numa_alloc_present[i]) { /* getAvailableNUMANodeResources' totalAllocated, reusable subtracted */
        req_c += numa_allocated_cpu_pref(n, pref, i);
        req_m += n->numa_alloc_mem[i];
      }
      alloc_c += n->numa_cpu[i];
      alloc_m += n->numa_mem[i];
    }
  } else {
    alloc_c = node_alloc_cpu;
    alloc_m = node_alloc_mem;
    req_c = node_req_cpu;
    req_m = node_req_mem;
  }
  if (cs_size(&cpus) > 0) {
    /* getAvailableCPUs with preferred = preferredCPUs − the pod's cpus: the allocated CPUDetails' size */
    or_cpuset held = n->allocated;
    if (pref) {
      const or_cpuset rest = cs_andnot(*pref, cpus);
      available_pref(n, &rest, &held);
    }
    req_c = amplify((int64_t)cs_size(&held) * 1000, n->cpu_amp);
  }
  return scorer(strategy, w, req_c, req_m, alloc_c, alloc_m, opt_req_cpu(n, p), p->req_mem);
}

int or_numa_reserve(const kg_config* cfg, or_numa_node* n, const or_numa_pod* p, const or_hint* affinity,
                    or_cpuset* cpus, int64_t* alloc) {
  return or_numa_reserve_pref(cfg, n, p, affinity, NULL, cpus, alloc);
}

int or_numa_reserve_pref(const kg_config* cfg, or_numa_node* n, const or_numa_pod* p, const or_hint* affinity,
                         const or_cpuset* pref, or_cpuset* cpus, int64_t* alloc) {
  *cpus = cs_empty();
  if (alloc) memset(alloc, 0, sizeof(int64_t) * OR_NUMA_ALLOC_WORDS);
  if (skip_the_node(p, n->numa_policy)) return 0;
  if (p->request_cpu_bind && (!n->has_topology || !n->valid_topology)) return -1;
  numa_alloc res;
  if (allocate(cfg, n, p, affinity, pref, &res, cpus) != 0) return -1;
  /* resourceManager.Update → addPodAllocation (node_allocation.go:76-103): RefCount + 1 per cpu, which takes the pod's
   * exclusive policy */
  for (int c = 0; c < KG_MAX_CPUS; c++)
    if (cs_has(cpus, c) && n->ref[c] < 255) n->ref[c]++;
  n->allocated = cs_or(n->allocated, *cpus);
  n->excl_pcpu = cs_andnot(n->excl_pcpu, *cpus);
  n->excl_numa = cs_andnot(n->excl_numa, *cpus);
  if (p->excl_policy == KG_EXCL_PCPU_LEVEL) n->excl_pcpu = cs_or(n->excl_pcpu, *cpus);
  if (p->excl_policy == KG_EXCL_NUMA_NODE_LEVEL) n->excl_numa = cs_or(n->excl_numa, *cpus);
  for (int k = 0; k < res.n; k++) {
    const int i = res.numa[k];
    n->numa_alloc_cpu[i] += res.cpu[k];
    n->numa_alloc_mem[i] += res.mem[k];
    n->numa_alloc_present[i] = 1;
    if (alloc) { /* the PodAllocation's NUMANodeResources, kept for Release */
      alloc[0] |= (int64_t)1 << i;
      alloc[1 + i] += res.cpu[k];
      alloc[1 + KG_MAX_NUMA + i] += res.mem[k];
    }
  }
  return 0;
}

/* resourceManager.Release → NodeAllocation.release (node_allocation.go:105-131): the pod's cpus leave the
 * allocated set (maxRefCount 1) and its NUMANodeResources are subtracted (SubtractWithNonNegativeResult). */
void or_numa_release(or_numa_node* n, const or_cpuset* cpus, const int64_t* alloc) {
  for (int c = 0; c < KG_MAX_CPUS; c++) {
    if (!cs_has(cpus, c) || n->ref[c] == 0) continue;
    if (--n->ref[c] > 0) continue; /* (r6) still held (its reservation): the CPUInfo stays, policy and all */
    cs_del(&n->allocated, c);
    cs_del(&n->excl_pcpu, c); /* RefCount 0: the CPUInfo (and its policy) is deleted */
    cs_del(&n->excl_numa, c);
  }
  for (int i = 0; i < KG_MAX_NUMA; i++) {
    if (!((alloc[0] >> i) & 1)) continue;
    n->numa_alloc_cpu[i] = n->numa_alloc_cpu[i] - alloc[1 + i] > 0 ? n->numa_alloc_cpu[i] - alloc[1 + i] : 0;
    const int64_t m = alloc[1 + KG_MAX_NUMA + i];
    n->numa_alloc_mem[i] = n->numa_alloc_mem[i] - m > 0 ? n->numa_alloc_mem[i] - m : 0;
  }
}

/* ---------------------------------------------------------------------------------------------------- */
/* flat entry points for the Python binding (oracle/oracle.py)                                            */
/* ---------------------------------------------------------------------------------------------------- */
int64_t or_numa_state_size(void) { return (int64_t)sizeof(or_numa_node); }

void or_numa_states_init(const kg_node_numa* src, int64_t n, void* out) {
  or_numa_node* s = (or_numa_node*)out;
  for (int64_t i = 0; i < n; i++) or_numa_node_init(&s[i], &src[i]);
}

void or_numa_state_read(const void* states, int64_t i, uint64_t* allocated, int64_t* alloc_cpu, int64_t* alloc_mem) {
  const or_numa_node* s = &((const or_numa_node*)states)[i];
  for (int w = 0; w < OR_CPUSET_WORDS; w++) allocated[w] = s->allocated.w[w];
  for (int k = 0; k < KG_MAX_NUMA; k++) {
    alloc_cpu[k] = s->numa_alloc_cpu[k];
    alloc_mem[k] = s->numa_alloc_mem[k];
  }
}

int or_take_cpus_flat(int sockets, int nodes_per_socket, int cores_per_node, int cpus_per_core,
                      const uint64_t* available, int needed, int bind_policy, int strategy, uint64_t* out) {
  or_topology t;
  or_topology_build(&t, sockets, nodes_per_socket, cores_per_node, cpus_per_core);
  or_cpuset a, r;
  for (int w = 0; w < OR_CPUSET_WORDS; w++) a.w[w] = available[w];
  const int rc = or_take_cpus(&t, a, needed, bind_policy, strategy, &r);
  for (int w = 0; w < OR_CPUSET_WORDS; w++) out[w] = r.w[w];
  return rc;
}

int or_take_cpus_excl_flat(int sockets, int nodes_per_socket, int cores_per_node, int cpus_per_core,
                           const uint64_t* available, int needed, int bind_policy, int strategy, int excl_policy,
                           const uint64_t* excl_seed, uint64_t* out) {
  or_topology t;
  or_topology_build(&t, sockets, nodes_per_socket, cores_per_node, cpus_per_core);
  or_cpuset a, seed, r;
  for (int w = 0; w < OR_CPUSET_WORDS; w++) {
    a.w[w] = available[w];
    seed.w[w] = excl_seed[w];
  }
  const int rc = or_take_cpus_ex(&t, a, needed, bind_policy, strategy, excl_policy, seed, &r);
  for (int w = 0; w < OR_CPUSET_WORDS; w++) out[w] = r.w[w];
  return rc;
}

/* Filter + Score + the stored affinity of one pod on one node (the golden tables of plugin_test.go /
 * scoring_test.go).  Returns 1 when the node passes Filter. */
int or_numa_eval_flat(const kg_config* cfg, const kg_node_numa* node, const kg_pod* pod, int64_t node_req_cpu,
                      int64_t node_req_mem, int64_t node_alloc_cpu, int64_t node_alloc_mem, int64_t* score,
                      int64_t* affinity_mask) {
  or_numa_node n;
  or_numa_node_init(&n, node);
  or_numa_pod p;
  or_numa_pod_init(cfg, pod, &p);
  or_hint h = {1, 0, 0, 0};  /* no Filter in the profile: Score reads no stored affinity (nil) */
  const int ok = cfg->numa_filter ? or_numa_filter(cfg, &n, &p, &h, node_req_cpu, node_alloc_cpu) : 1;
  *affinity_mask = h.nil ? -1 : (int64_t)h.mask;
  *score = ok ? or_numa_score(cfg, &n, &p, &h, node_req_cpu, node_req_mem, node_alloc_cpu, node_alloc_mem) : 0;
  return ok;
}

/* Reserve of one pod on one node from its Filter affinity; writes the chosen cpuset.  0 ok, -1 failure. */
int or_numa_reserve_flat(const kg_config* cfg, const kg_node_numa* node, const kg_pod* pod, uint64_t* cpuset) {
  or_numa_node n;
  or_numa_node_init(&n, node);
  or_numa_pod p;
  or_numa_pod_init(cfg, pod, &p);
  or_hint h;
  or_numa_filter(cfg, &n, &p, &h, 0, INT64_MAX / 4);
  or_cpuset cs;
  const int rc = or_numa_reserve(cfg, &n, &p, &h, &cs, NULL);
  for (int w = 0; w < OR_CPUSET_WORDS; w++) cpuset[w] = cs.w[w];
  return rc;
}

/* Test hook: Policy.Merge on caller-given filtered provider lists (filterProvidersHints already applied: nl lists,
 * counts[i] hints each, hints[4 * (16 * i + j)] = {nil, mask, preferred, score}).  out = {admit, nil, mask,
 * preferred, score}.  Pins mergeFilteredHints + the policies with the reference's topologymanager test tables. */
int or_debug_policy_merge(int policy, int num_numa, int nl, const int32_t* counts, const int64_t* hints, int64_t* out) {
  if (nl < 0 || nl > 8) return -1;
  hint_list lists[8];
  for (int i = 0; i < nl; i++) {
    if (counts[i] < 0 || counts[i] > 16) return -1;
    lists[i].n = counts[i];
    for (int j = 0; j < counts[i]; j++) {
      const int64_t* h = hints + 4 * (16 * i + j);
      lists[i].h[j] = (or_hint){(int)h[0], (uint32_t)h[1], (int)h[2], h[3]};
    }
  }
  or_hint best;
  const int admit = policy_merge_lists(policy, (1u << num_numa) - 1u, lists, nl, &best);
  out[0] = admit;
  out[1] = best.nil;
  out[2] = best.mask;
  out[3] = best.preferred;
  out[4] = best.score;
  return 0;
}

/* Test hook: filterSingleNumaHints on caller-given lists (same encoding); writes the filtered counts and hints. */
int or_debug_single_numa_filter(int nl, const int32_t* counts, const int64_t* hints, int32_t* out_counts,
                                int64_t* out_hints) {
  if (nl < 0 || nl > 8) return -1;
  hint_list lists[8];
  for (int i = 0; i < nl; i++) {
    if (counts[i] < 0 || counts[i] > 16) return -1;
    lists[i].n = counts[i];
    for (int j = 0; j < counts[i]; j++) {
      const int64_t* h = hints + 4 * (16 * i + j);
      lists[i].h[j] = (or_hint){(int)h[0], (uint32_t)h[1], (int)h[2], h[3]};
    }
  }
  single_numa_filter(lists, nl);
  for (int i = 0; i < nl; i++) {
    out_counts[i] = lists[i].n;
    for (int j = 0; j < lists[i].n; j++) {
      int64_t* h = out_hints + 4 * (16 * i + j);
      h[0] = lists[i].h[j].nil, h[1] = lists[i].h[j].mask, h[2] = lists[i].h[j].preferred, h[3] = lists[i].h[j].score;
    }
  }
  return 0;
}

/* (r6) Test hooks for NodeNUMAResource with reservation cpusets (golden tables of node_allocation_test.go,
 * cpu_accumulator_test.go and plugin_test.go).  getAvailableCPUs with preferred cpus on a node whose allocated cpus
 * all have RefCount 1: writes the available cpus. */
void or_numa_available_pref_flat(const kg_node_numa* node, const uint64_t* preferred, uint64_t* out) {
  or_numa_node n;
  or_numa_node_init(&n, node);
  or_cpuset pref;
  for (int w = 0; w < OR_CPUSET_WORDS; w++) pref.w[w] = preferred[w];
  const or_cpuset a = available_pref(&n, &pref, NULL);
  for (int w = 0; w < OR_CPUSET_WORDS; w++) out[w] = a.w[w];
}

/* takePreferredCPUs (cpu_accumulator.go:33-85) on buildCPUTopologyForTest(sockets, nps, cpn, cpc), no exclusive
 * policy; 0 ok, -1 error */
int or_take_preferred_flat(int sockets, int nodes_per_socket, int cores_per_node, int cpus_per_core,
                           const uint64_t* available, const uint64_t* preferred, int needed, int bind_policy,
                           int strategy, uint64_t* out) {
  or_topology t;
  or_topology_build(&t, sockets, nodes_per_socket, cores_per_node, cpus_per_core);
  or_cpuset a, pref, r;
  for (int w = 0; w < OR_CPUSET_WORDS; w++) {
    a.w[w] = available[w];
    pref.w[w] = preferred[w];
  }
  const int rc = take_preferred(&t, a, &pref, needed, bind_policy, strategy, KG_EXCL_NONE, cs_empty(), &r);
  for (int w = 0; w < OR_CPUSET_WORDS; w++) out[w] = rc == 0 ? r.w[w] : 0;
  return rc;
}

/* Reserve of one pod on one node whose reservation slot 0 (rsv) holds cpus, the pod nominated into it: the node's
 * allocated cpus and the reservation's RefCounts as the reference's NodeAllocation holds them, the preferred cpus from
 * RestoreReservation.  Writes the chosen cpuset; 0 ok, -1 failure. */
int or_numa_reserve_rsv_flat(const kg_config* cfg, const kg_node_numa* node, const kg_node_reservations* rsv,
                             const kg_pod* pod, uint64_t* cpuset) {
  or_numa_node n;
  or_numa_node_init(&n, node);
  or_numa_rsv_refs(&n, rsv);
  or_numa_pod p;
  or_numa_pod_init(cfg, pod, &p);
  or_hint h;
  or_numa_filter(cfg, &n, &p, &h, 0, INT64_MAX / 4);
  const or_cpuset pref = or_numa_rsv_reserved(rsv, 0);
  or_cpuset cs;
  const int rc = or_numa_reserve_pref(cfg, &n, &p, &h, p.allow_cpuset ? &pref : NULL, &cs, NULL);
  for (int w = 0; w < OR_CPUSET_WORDS; w++) cpuset[w] = cs.w[w];
  return rc;
}

/* RestoreReservation's reservedCPUs of slot s as words (plugin_test.go TestRestoreReservation) */
void or_numa_rsv_reserved_flat(const kg_node_reservations* r, int s, uint64_t* out) {
  const or_cpuset c = or_numa_rsv_reserved(r, s);
  for (int w = 0; w < OR_CPUSET_WORDS; w++) out[w] = c.w[w];
}

/* (r6) The NodeAllocation of node i as a kg_node_numa row's mutable fields (allocated cpus, their exclusive policies,
 * allocatedResources), written over `row`: what a caller re-sends with a rewritten NodeResourceTopology
 * (topology_eventhandler.go:62-113 updates TopologyOptions; the NodeAllocation stays). */
void or_numa_state_export(const void* states, int64_t i, kg_node_numa* row) {
  const or_numa_node* s = &((const or_numa_node*)states)[i];
  for (int w = 0; w < OR_CPUSET_WORDS; w++) {
    row->allocated_cpus[w] = s->allocated.w[w];
    row->exclusive_pcpu_cpus[w] = s->excl_pcpu.w[w];
    row->exclusive_numa_cpus[w] = s->excl_numa.w[w];
  }
  for (int k = 0; k < KG_MAX_NUMA; k++) {
    row->numa_alloc_cpu[k] = s->numa_alloc_cpu[k];
    row->numa_alloc_mem[k] = s->numa_alloc_mem[k];
  }
}

/* (r6) Re-initialise node i's state from a row (the NodeResourceTopology / NodeAllocation upsert) */
void or_numa_state_set(void* states, int64_t i, const kg_node_numa* row) {
  or_numa_node_init(&((or_numa_node*)states)[i], row);
}
