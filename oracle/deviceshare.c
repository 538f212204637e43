/* deviceshare.c — CPU restatement of the DeviceShare GPU path.  TEST INFRASTRUCTURE ONLY (see deviceshare.h). */
#include "deviceshare.h"

#include <string.h>

/* combination flags (utils.go:37-46) */
enum { F_NVIDIA = 1, F_DCU = 2, F_KGPU = 4, F_CORE = 8, F_MEM = 16, F_RATIO = 32 };

/* ValidatePercentageResource (utils.go:151-156) */
static int valid_percentage(int64_t v) { return !(v > 100 && v % 100 != 0); }

/* GetPodDeviceRequests (utils.go:232-252) for the GPU type: Mask → ValidateDeviceRequest (:158-179) →
 * ConvertDeviceRequest (:181-192, mapper table :92-149) */
int or_ds_pod_init(const kg_pod* pod, or_ds_pod* out) {
  memset(out, 0, sizeof(*out));
  out->reserve = (pod->flags & KG_POD_RESERVE) != 0;
  const int64_t* q = pod->device_requests;
  for (int r = 0; r < KG_DEV_RES_MAX; r++)
    if (q[r] < 0) { out->error = 1; return 0; }
  /* (ABI 17) RDMA / FPGA: one resource per type (DeviceResourceNames, utils.go:47-58), ValidatePercentageResource */
  out->xq[KG_XTYPE_RDMA] = q[KG_DEV_RDMA];
  out->xq[KG_XTYPE_FPGA] = q[KG_DEV_FPGA];
  for (int t = 0; t < KG_DEV_XTYPES; t++)
    if (out->xq[t] && !valid_percentage(out->xq[t])) out->error = 1; /* "invalid resource unit" */
  static const int flag_of[6] = {F_NVIDIA, F_DCU, F_KGPU, F_CORE, F_MEM, F_RATIO};
  unsigned comb = 0;
  for (int r = 0; r < 6; r++)
    if (q[r] != 0) comb |= (unsigned)flag_of[r]; /* quotav1.RemoveZeros */
  if (comb == 0) {
    out->nogpu = 1;
    out->skip = out->xq[0] == 0 && out->xq[1] == 0; /* state.skip: no request of any device type */
    return 0;
  }
  if ((q[KG_DEV_KOORD_GPU] && !valid_percentage(q[KG_DEV_KOORD_GPU])) ||
      (q[KG_DEV_GPU_CORE] && !valid_percentage(q[KG_DEV_GPU_CORE])) ||
      (q[KG_DEV_GPU_MEMORY_RATIO] && !valid_percentage(q[KG_DEV_GPU_MEMORY_RATIO]))) {
    out->error = 1; /* "invalid resource unit" */
    return 0;
  }
  switch (comb) {
    case F_NVIDIA: out->core = out->ratio = q[KG_DEV_NVIDIA_GPU] * 100; break;
    case F_DCU: out->core = out->ratio = q[KG_DEV_HYGON_DCU] * 100; break;
    case F_KGPU: out->core = out->ratio = q[KG_DEV_KOORD_GPU]; break;
    case F_MEM: out->mem = q[KG_DEV_GPU_MEMORY]; out->has_mem = 1; break;
    case F_RATIO: out->ratio = q[KG_DEV_GPU_MEMORY_RATIO]; break;
    case F_CORE | F_MEM: out->core = q[KG_DEV_GPU_CORE]; out->mem = q[KG_DEV_GPU_MEMORY]; out->has_mem = 1; break;
    case F_CORE | F_RATIO: out->core = q[KG_DEV_GPU_CORE]; out->ratio = q[KG_DEV_GPU_MEMORY_RATIO]; break;
    default: out->error = 1; /* "invalid resource device requests" */
  }
  return 0;
}

int64_t or_ds_memory_bytes_to_ratio(int64_t bytes, int64_t total) {
  /* int64(float64(bytes.Value()) / float64(totalMemory.Value()) * 100): two roundings, no contraction */
  volatile double q = (double)bytes / (double)total;
  volatile double p = q * 100.0;
  return (int64_t)p;
}

int64_t or_ds_memory_ratio_to_bytes(int64_t ratio, int64_t total) { return ratio * total / 100; }

static int64_t sub0(int64_t a, int64_t b) { return a - b > 0 ? a - b : 0; }
static int64_t tot(const kg_node_device* d, int m, int r) {
  if (!d->present[m] || !d->healthy[m]) return 0; /* unhealthy: empty ResourceList (device_cache.go:513-515) */
  return r == 0 ? d->total_core[m] : (r == 1 ? d->total_memory[m] : d->total_ratio[m]);
}
static int64_t used(const kg_node_device* d, int m, int r) {
  return r == 0 ? d->used_core[m] : (r == 1 ? d->used_memory[m] : d->used_ratio[m]);
}
/* resetDeviceFree (device_cache.go:157-174): free = SubtractWithNonNegativeResult(total, used) */
static int64_t freev(const kg_node_device* d, int m, int r) { return sub0(tot(d, m, r), used(d, m, r)); }
static int free_zero(const kg_node_device* d, int m) {
  return freev(d, m, 0) == 0 && freev(d, m, 1) == 0 && freev(d, m, 2) == 0;
}

/* GPUHandler.CalcDesiredRequestsAndCount + fillGPUTotalMem (devicehandler_gpu.go:40-90) */
or_ds_inst or_ds_instance(const kg_node_device* d, const or_ds_pod* p) {
  or_ds_inst in;
  memset(&in, 0, sizeof(in));
  int any = 0, first = -1;
  for (int m = 0; m < KG_MAX_MINORS; m++) {
    if (!d->present[m]) continue;
    any = 1;
    if (first < 0 && (tot(d, m, 0) || tot(d, m, 1) || tot(d, m, 2))) first = m;
  }
  if (!any || first < 0) return in; /* "Insufficient gpu devices" / "no healthy GPU Devices" */
  const int64_t tmem = tot(d, first, 1);
  int64_t core = p->core, mem = p->mem, ratio = p->ratio;
  if (p->has_mem) ratio = or_ds_memory_bytes_to_ratio(mem, tmem);
  else mem = or_ds_memory_ratio_to_bytes(ratio, tmem);
  in.count = 1;
  if (ratio > 100 && ratio % 100 == 0) {
    const int64_t n = ratio / 100;
    in.count = (int)n;
    core /= n;
    mem /= n;
    ratio /= n;
  }
  in.ok = 1;
  in.core = core;
  in.mem = mem;
  in.ratio = ratio;
  return in;
}

static int fits(const kg_node_device* d, int m, const or_ds_inst* in) {
  /* quotav1.IsZero(free) skip + LessThanOrEqual(request, free) (device_allocator.go:412-421) */
  if (free_zero(d, m)) return 0;
  return in->core <= freev(d, m, 0) && in->mem <= freev(d, m, 1) && in->ratio <= freev(d, m, 2);
}

static int all_free_zero(const kg_node_device* d) {
  for (int m = 0; m < KG_MAX_MINORS; m++)
    if (d->present[m] && !free_zero(d, m)) return 0;
  return 1;
}

int or_ds_filter(const kg_node_device* d, const or_ds_pod* p) {
  if (p->skip) return 1;
  if (p->error) return 0;
  if (!d->has_device) return 0;
  if (!or_dsx_filter(d, p, NULL)) return 0; /* (ABI 17) every requested type must allocate */
  if (p->nogpu) return 1;
  const or_ds_inst in = or_ds_instance(d, p);
  if (!in.ok) return 0;
  if (all_free_zero(d)) return 0; /* nodeDevice.filter drops the type (device_cache.go:358-360) */
  int n = 0;
  for (int m = 0; m < KG_MAX_MINORS; m++)
    if (d->present[m] && fits(d, m, &in)) n++;
  return n >= in.count;
}

static int64_t least_requested(int64_t req, int64_t cap) {
  if (cap == 0 || req > cap) return 0;
  return (cap - req) * 100 / cap;
}
static int64_t most_requested(int64_t req, int64_t cap) {
  if (cap == 0) return 0;
  if (req > cap) req = cap;
  return req * 100 / cap;
}

/* resourceAllocationScorer over (requested, allocatable) per resource (scoring.go:183-243, 254-308) */
static int64_t scorer(int strategy, const int64_t w[3], const int64_t total[3], const int64_t free_[3],
                      const int64_t req[3]) {
  int64_t num = 0, ws = 0;
  for (int r = 0; r < 3; r++) {
    if (w[r] == 0 || total[r] == 0) continue;
    const int64_t rq = total[r] >= free_[r] ? total[r] - free_[r] + req[r] : total[r];
    const int64_t s = strategy == KG_STRATEGY_MOST_ALLOCATED ? most_requested(rq, total[r]) : least_requested(rq, total[r]);
    num += s * w[r];
    ws += w[r];
  }
  return ws == 0 ? 0 : num / ws;
}

int64_t or_ds_score(const kg_node_device* d, const or_ds_pod* p, int strategy, const int64_t w[3]) {
  if (p->skip || p->error || !d->has_device || p->nogpu) return 0;
  const or_ds_inst in = or_ds_instance(d, p);
  if (!in.ok || all_free_zero(d)) return 0;
  int64_t total[3] = {0, 0, 0}, free_[3] = {0, 0, 0};
  for (int m = 0; m < KG_MAX_MINORS; m++) {
    if (!d->present[m]) continue;
    for (int r = 0; r < 3; r++) {
      total[r] += tot(d, m, r);
      free_[r] += freev(d, m, r);
    }
  }
  const int64_t req[3] = {in.core, in.mem, in.ratio};
  return scorer(strategy, w, total, free_, req);
}

int64_t or_ds_score_minor(const kg_node_device* d, int m, const or_ds_pod* p, const or_ds_inst* in, int strategy,
                          const int64_t w[3]) {
  (void)p;
  const int64_t total[3] = {tot(d, m, 0), tot(d, m, 1), tot(d, m, 2)};
  const int64_t free_[3] = {freev(d, m, 0), freev(d, m, 1), freev(d, m, 2)};
  const int64_t req[3] = {in->core, in->mem, in->ratio};
  return scorer(strategy, w, total, free_, req);
}

int32_t or_ds_reserve(kg_node_device* d, const or_ds_pod* p, int strategy, const int64_t w[3]) {
  if (p->skip || !d->has_device) return 0;
  if (p->error) return -1;
  if (p->nogpu) return 0;
  const or_ds_inst in = or_ds_instance(d, p);
  if (!in.ok || all_free_zero(d)) return -1;
  /* scoreDevices → sortDeviceResourcesByMinor (score desc, minor asc) → first `count` that fit */
  int order[KG_MAX_MINORS], n = 0;
  int64_t sc[KG_MAX_MINORS];
  for (int m = 0; m < KG_MAX_MINORS; m++) {
    if (!d->present[m]) continue;
    sc[m] = or_ds_score_minor(d, m, p, &in, strategy, w);
    int k = n++;
    while (k > 0 && (sc[order[k - 1]] < sc[m])) { order[k] = order[k - 1]; k--; }
    order[k] = m;
  }
  int32_t mask = 0, got = 0;
  for (int k = 0; k < n && got < in.count; k++) {
    const int m = order[k];
    if (!fits(d, m, &in)) continue;
    mask |= 1 << m;
    got++;
  }
  if (got < in.count) return -1;
  for (int m = 0; m < KG_MAX_MINORS; m++) {
    if (!(mask >> m & 1)) continue;
    d->used_core[m] += in.core; /* updateDeviceUsed: quotav1.Add(used, allocation.Resources) */
    d->used_memory[m] += in.mem;
    d->used_ratio[m] += in.ratio;
  }
  return mask;
}

void or_ds_release(kg_node_device* d, const or_ds_pod* p, int32_t minors) {
  if (p->skip || !d->has_device || p->error) return;
  or_dsx_release(d, p, minors); /* (ABI 17) the RDMA / FPGA bytes of the packed mask */
  minors &= 0xFF;
  if (p->nogpu || !minors) return;
  const or_ds_inst in = or_ds_instance(d, p); /* the per-instance request Reserve added (node totals only) */
  for (int m = 0; m < KG_MAX_MINORS; m++) {
    if (!(minors >> m & 1)) continue;
    /* updateDeviceUsed(add=false): quotav1.SubtractWithNonNegativeResult(used, allocation.Resources) */
    d->used_core[m] = d->used_core[m] - in.core > 0 ? d->used_core[m] - in.core : 0;
    d->used_memory[m] = d->used_memory[m] - in.mem > 0 ? d->used_memory[m] - in.mem : 0;
    d->used_ratio[m] = d->used_ratio[m] - in.ratio > 0 ? d->used_ratio[m] - in.ratio : 0;
  }
}

void or_default_normalize(int64_t* s, int64_t n) {
  int64_t mx = 0;
  for (int64_t i = 0; i < n; i++)
    if (s[i] > mx) mx = s[i];
  if (mx == 0) return;
  for (int64_t i = 0; i < n; i++) s[i] = 100 * s[i] / mx;
}

/* ---- (ABI 17) RDMA / FPGA: DefaultDeviceHandler (devicehandler_default.go:45-92) without hints ------------------
 * CalcDesiredRequestsAndCount: a request q > 100 and a multiple of 100 is q / 100 instances of 100, else one of q;
 * "Insufficient %s devices" when the node lists no device of the type.  deviceTotal of an unhealthy device is an empty
 * ResourceList (device_cache.go:513-515); free = SubtractWithNonNegativeResult(total, used − preemptible). */
static void x_inst(int64_t q, int* count, int64_t* per) {
  const int multi = q > 100 && q % 100 == 0;
  *count = multi ? (int)(q / 100) : 1;
  *per = multi ? 100 : q;
}
static int64_t xtot(const kg_node_device* d, int t, int m) {
  return d->x_present[t][m] && d->x_healthy[t][m] ? d->x_total[t][m] : 0;
}
static int64_t xfree(const kg_node_device* d, int t, int m, const int64_t (*pre)[KG_MAX_MINORS]) {
  return sub0(xtot(d, t, m), sub0(d->x_used[t][m], pre ? pre[t][m] : 0));
}
static int x_listed(const kg_node_device* d, int t) {
  for (int m = 0; m < KG_MAX_MINORS; m++)
    if (d->x_present[t][m]) return 1;
  return 0;
}
/* the scorer over the type's one resource: the other configured resources see a zero total (skipped), so the weighted
 * mean is the resource's own least / most requested score when its weight is set, 0 otherwise (scoring.go:183-304) */
static int64_t x_scorer(int strategy, int64_t w, int64_t total, int64_t free_, int64_t req) {
  if (w == 0 || total == 0) return 0;
  const int64_t rq = total >= free_ ? total - free_ + req : total;
  const int64_t s = strategy == KG_STRATEGY_MOST_ALLOCATED ? most_requested(rq, total) : least_requested(rq, total);
  return s * w / w;
}

int or_dsx_filter(const kg_node_device* d, const or_ds_pod* p, const int64_t (*pre)[KG_MAX_MINORS]) {
  if (p->skip) return 1;
  if (p->error) return 0;
  for (int t = 0; t < KG_DEV_XTYPES; t++) {
    if (!p->xq[t]) continue;
    if (!d->has_device || !x_listed(d, t)) return 0;
    int count;
    int64_t per;
    x_inst(p->xq[t], &count, &per);
    int any = 0, n = 0;
    for (int m = 0; m < KG_MAX_MINORS; m++) {
      if (!d->x_present[t][m]) continue;
      const int64_t f = xfree(d, t, m, pre);
      any |= f != 0;
      n += f != 0 && per <= f; /* defaultAllocateDevices: skip zero free, LessThanOrEqual(request, free) */
    }
    if (!any || n < count) return 0; /* nodeDevice.filter drops an all-zero type; "Insufficient %s devices" */
  }
  return 1;
}

int64_t or_dsx_score(const kg_node_device* d, const or_ds_pod* p, int strategy, const int64_t w[KG_DEV_XTYPES]) {
  if (p->skip || p->error || !d->has_device) return 0;
  int64_t sum = 0;
  for (int t = 0; t < KG_DEV_XTYPES; t++) {
    if (!p->xq[t] || !x_listed(d, t)) continue;
    int count;
    int64_t per, T = 0, F = 0;
    x_inst(p->xq[t], &count, &per);
    for (int m = 0; m < KG_MAX_MINORS; m++) {
      if (!d->x_present[t][m]) continue;
      T += xtot(d, t, m);
      F += xfree(d, t, m, NULL);
    }
    sum += x_scorer(strategy, w[t], T, F, per); /* AutopilotAllocator.score: finalScore += per type */
  }
  return sum;
}

int32_t or_dsx_reserve(kg_node_device* d, const or_ds_pod* p, int strategy, const int64_t w[KG_DEV_XTYPES]) {
  if (p->skip || !d->has_device) return 0;
  if (p->error) return -1;
  int32_t taken[KG_DEV_XTYPES] = {0, 0};
  for (int t = 0; t < KG_DEV_XTYPES; t++) {
    if (!p->xq[t]) continue;
    if (!x_listed(d, t)) return -1;
    int count;
    int64_t per;
    x_inst(p->xq[t], &count, &per);
    /* scoreDevices → sortDeviceResourcesByMinor (score desc, minor asc) → the first `count` that fit */
    int order[KG_MAX_MINORS], n = 0, any = 0;
    int64_t sc[KG_MAX_MINORS];
    for (int m = 0; m < KG_MAX_MINORS; m++) {
      if (!d->x_present[t][m]) continue;
      const int64_t f = xfree(d, t, m, NULL);
      any |= f != 0;
      sc[m] = x_scorer(strategy, w[t], xtot(d, t, m), f, per);
      int k = n++;
      while (k > 0 && sc[order[k - 1]] < sc[m]) { order[k] = order[k - 1]; k--; }
      order[k] = m;
    }
    if (!any) return -1;
    int got = 0;
    for (int k = 0; k < n && got < count; k++) {
      const int m = order[k];
      const int64_t f = xfree(d, t, m, NULL);
      if (f == 0 || per > f) continue;
      taken[t] |= 1 << m;
      got++;
    }
    if (got < count) return -1;
  }
  int32_t out = 0;
  for (int t = 0; t < KG_DEV_XTYPES; t++) {
    if (!taken[t]) continue;
    int count;
    int64_t per;
    x_inst(p->xq[t], &count, &per);
    for (int m = 0; m < KG_MAX_MINORS; m++)
      if ((taken[t] >> m) & 1) d->x_used[t][m] += per; /* updateCacheUsed */
    out |= taken[t] << (8 * (t + 1));
  }
  return out;
}

void or_dsx_release(kg_node_device* d, const or_ds_pod* p, int32_t packed) {
  for (int t = 0; t < KG_DEV_XTYPES; t++) {
    const int32_t mk = (int32_t)(((uint32_t)packed >> (8 * (t + 1))) & 0xFFu);
    if (!mk || !p->xq[t]) continue;
    int count;
    int64_t per;
    x_inst(p->xq[t], &count, &per);
    for (int m = 0; m < KG_MAX_MINORS; m++)
      if ((mk >> m) & 1) d->x_used[t][m] = sub0(d->x_used[t][m], per);
  }
}

/* flat helper for the Python binding: CalcDesiredRequestsAndCount → out = {count, core, mem, ratio} */
int or_ds_instance_flat(const kg_node_device* d, const or_ds_pod* p, int64_t* out) {
  const or_ds_inst in = or_ds_instance(d, p);
  out[0] = in.count; out[1] = in.core; out[2] = in.mem; out[3] = in.ratio;
  return in.ok;
}

/* ===================================================================================================================
 * (ABI 13) Reservations that hold GPUs (deviceshare/reservation.go, plugin.go:280-459, scoring.go:34-160,
 * device_allocator.go:89-129, device_cache.go:314-391, device_resources.go:47-208).  Device resources are kept per minor
 * as {gpu-core, gpu-memory, gpu-memory-ratio}; a minor absent from a map holds zeros, which every formula below
 * treats exactly as the reference treats an absent key / minor (SubtractWithNonNegativeResult, appendAllocated,
 * calcFreeWithPreemptible's merge, LessThanOrEqual over the free resources' keys — all three keys are present on a
 * healthy GPU).
 * =================================================================================================================== */

static int64_t mn64(int64_t a, int64_t b) { return a < b ? a : b; }

/* RestoreReservation + mergeReservationAllocations (reservation.go:84-171) over the GPU-holding slots of the
 * Reservation restore's matched / unmatched lists: remained = SubtractWithNonNegativeResult(allocatable, allocated);
 * mergedUnmatchedUsed += allocatable − remained (= min(allocatable, allocated)); mergedMatchedAllocatable /
 * mergedMatchedAllocated += allocatable / allocated */
void or_ds_rsv_init(const kg_node_reservations* r, const int32_t* matched, int n_matched, const int32_t* unmatched,
                    int n_unmatched, or_ds_rsv* out) {
  memset(out, 0, sizeof(*out));
  if (!r) return;
  for (int k = 0; k < n_unmatched; k++) {
    const int s = unmatched[k];
    if (!r->gpu_minors[s]) continue;
    for (int m = 0; m < KG_MAX_MINORS; m++)
      for (int q = 0; q < 3; q++) out->unm_used[m][q] += mn64(r->gpu_alloc[s][m][q], r->gpu_allocated[s][m][q]);
  }
  for (int k = 0; k < n_matched; k++) {
    const int s = matched[k];
    if (!r->gpu_minors[s]) continue;
    out->matched[out->n_matched++] = s;
    for (int m = 0; m < KG_MAX_MINORS; m++)
      for (int q = 0; q < 3; q++) {
        out->mat_alloc[m][q] += r->gpu_alloc[s][m][q];
        out->mat_allocd[m][q] += r->gpu_allocated[s][m][q];
      }
  }
}

/* calcFreeWithPreemptible (device_cache.go:314-342): free = SubtractWithNonNegativeResult(total,
 * SubtractWithNonNegativeResult(used, preemptible)) on every minor (a minor without preemptible keeps total − used) */
static int64_t free_pre(const kg_node_device* d, int m, int q, const int64_t (*pre)[3]) {
  const int64_t u = sub0(used(d, m, q), pre ? pre[m][q] : 0);
  return sub0(tot(d, m, q), u);
}

/* AutopilotAllocator.Allocate / score over a filtered nodeDevice (device_allocator.go:89-155, 499-522): the minors and
 * free resources it sees — every listed minor with the preemptible-merged free, or, with requiredDeviceResources
 * (a Restricted reservation), only the reservation's minors with their remained resources.  Returns 0 when the GPU
 * type is dropped (nodeDevice.filter: free resources all zero). */
static int dsr_view(const kg_node_device* d, const int64_t (*pre)[3], uint32_t rr_minors, const int64_t (*rr)[3],
                    int64_t fr[KG_MAX_MINORS][3], uint32_t* minors) {
  *minors = 0;
  int any = 0;
  for (int m = 0; m < KG_MAX_MINORS; m++) {
    for (int q = 0; q < 3; q++) fr[m][q] = 0;
    if (!d->present[m]) continue;
    if (rr) {
      if (!((rr_minors >> m) & 1u)) continue;
      for (int q = 0; q < 3; q++) fr[m][q] = rr[m][q];
    } else {
      for (int q = 0; q < 3; q++) fr[m][q] = free_pre(d, m, q, pre);
    }
    *minors |= 1u << m;
    any |= fr[m][0] != 0 || fr[m][1] != 0 || fr[m][2] != 0;
  }
  return any;
}

/* Allocate(required, preferred, requiredDeviceResources, preemptible): defaultAllocateDevices over the view — pairs in
 * sortDeviceResourcesByMinor order (preferred first, then scoreDevice desc when a scorer is set — Reserve and Score,
 * not Filter —, then minor asc), skipping minors outside `required`, all-zero minors and minors the per-instance request
 * does not fit; the first desiredCount.  Returns the minor mask, -1 = Insufficient. */
int32_t or_ds_allocate(const kg_node_device* d, const or_ds_pod* p, uint32_t required, uint32_t preferred,
                       uint32_t rr_minors, const int64_t (*rr)[3], const int64_t (*pre)[3], int scored, int strategy,
                       const int64_t w[3]) {
  if (p->skip || !d->has_device) return 0;
  if (p->error) return -1;
  if (p->nogpu) return 0; /* (ABI 17) only RDMA / FPGA: no GPU minor */
  const or_ds_inst in = or_ds_instance(d, p);
  if (!in.ok) return -1;
  int64_t fr[KG_MAX_MINORS][3];
  uint32_t minors = 0;
  if (!dsr_view(d, pre, rr_minors, rr, fr, &minors)) return -1;
  int order[KG_MAX_MINORS], n = 0;
  int64_t sc[KG_MAX_MINORS] = {0};
  for (int m = 0; m < KG_MAX_MINORS; m++) {
    if (!((minors >> m) & 1u)) continue;
    if (scored) {
      const int64_t total[3] = {tot(d, m, 0), tot(d, m, 1), tot(d, m, 2)};
      const int64_t req[3] = {in.core, in.mem, in.ratio};
      sc[m] = scorer(strategy, w, total, fr[m], req);
    }
    const int pm = (preferred >> m) & 1;
    int k = n++;
    while (k > 0) {
      const int o = order[k - 1], po = (preferred >> o) & 1;
      if (po > pm || (po == pm && sc[o] >= sc[m])) break; /* earlier minors win ties (minor asc) */
      order[k] = o;
      k--;
    }
    order[k] = m;
  }
  int32_t mask = 0;
  int got = 0;
  for (int k = 0; k < n && got < in.count; k++) {
    const int m = order[k];
    if (required && !((required >> m) & 1u)) continue;
    if (fr[m][0] == 0 && fr[m][1] == 0 && fr[m][2] == 0) continue;
    if (!(in.core <= fr[m][0] && in.mem <= fr[m][1] && in.ratio <= fr[m][2])) continue;
    mask |= 1 << m;
    got++;
  }
  return got < in.count ? -1 : mask;
}

/* AutopilotAllocator.score over the view: scoreNode(request, Σ total, Σ free) of the minors it lists (0 when the type
 * is dropped) */
int64_t or_ds_score_view(const kg_node_device* d, const or_ds_pod* p, uint32_t rr_minors, const int64_t (*rr)[3],
                         const int64_t (*pre)[3], int strategy, const int64_t w[3]) {
  if (p->skip || p->error || !d->has_device || p->nogpu) return 0;
  const or_ds_inst in = or_ds_instance(d, p);
  if (!in.ok) return 0;
  int64_t fr[KG_MAX_MINORS][3];
  uint32_t minors = 0;
  if (!dsr_view(d, pre, rr_minors, rr, fr, &minors)) return 0;
  int64_t total[3] = {0, 0, 0}, free_[3] = {0, 0, 0};
  for (int m = 0; m < KG_MAX_MINORS; m++) {
    if (!((minors >> m) & 1u)) continue;
    for (int q = 0; q < 3; q++) {
      total[q] += tot(d, m, q);
      free_[q] += fr[m][q];
    }
  }
  const int64_t req[3] = {in.core, in.mem, in.ratio};
  return scorer(strategy, w, total, free_, req);
}

/* the preemptible map of one matched reservation s (tryAllocateFromReservation / scoreWithReservation):
 * mergedUnmatchedUsed + mergedMatchedAllocated + remained(s) (preemptibleInRR: no preemption here) */
static void dsr_pre_slot(const kg_node_reservations* r, const or_ds_rsv* st, int s, int64_t pre[KG_MAX_MINORS][3],
                         int64_t rem[KG_MAX_MINORS][3]) {
  for (int m = 0; m < KG_MAX_MINORS; m++)
    for (int q = 0; q < 3; q++) {
      rem[m][q] = sub0(r->gpu_alloc[s][m][q], r->gpu_allocated[s][m][q]);
      pre[m][q] = st->unm_used[m][q] + st->mat_allocd[m][q] + rem[m][q];
    }
}

/* tryAllocateFromReservation (reservation.go:173-244) over the given GPU-holding matched slots, in order:
 * Default / Aligned: Allocate(nil, preferred = the slot's minors, nil, preemptible); Restricted: the same with required =
 * preferred, and then once more with requiredDeviceResources = the slot's remained (calcRequiredDeviceResources: all
 * zero when nothing remains).  Returns the satisfied slot (its allocation in *mask), -1 none satisfied. */
int or_ds_try_rsv(const kg_node_device* d, const or_ds_pod* p, const kg_node_reservations* r, const or_ds_rsv* st,
                  const int32_t* slots, int n_slots, int scored, int strategy, const int64_t w[3], int32_t* mask) {
  for (int k = 0; k < n_slots; k++) {
    const int s = slots[k];
    int64_t pre[KG_MAX_MINORS][3], rem[KG_MAX_MINORS][3];
    dsr_pre_slot(r, st, s, pre, rem);
    const uint32_t pref = (uint32_t)r->gpu_minors[s];
    int32_t got;
    if (r->policy[s] == KG_RSV_POLICY_RESTRICTED) {
      if (or_ds_allocate(d, p, pref, pref, 0, NULL, (const int64_t(*)[3])pre, 0, strategy, w) < 0) continue;
      got = or_ds_allocate(d, p, pref, pref, pref, (const int64_t(*)[3])rem, (const int64_t(*)[3])pre, scored,
                           strategy, w);
    } else {
      got = or_ds_allocate(d, p, 0, pref, 0, NULL, (const int64_t(*)[3])pre, scored, strategy, w);
    }
    if (got >= 0) {
      if (mask) *mask = got;
      return s;
    }
  }
  return -1;
}

/* the preemptible map of the node-level fallback: mergedUnmatchedUsed + mergedMatchedAllocatable */
static void dsr_pre_node(const or_ds_rsv* st, int64_t pre[KG_MAX_MINORS][3]) {
  for (int m = 0; m < KG_MAX_MINORS; m++)
    for (int q = 0; q < 3; q++) pre[m][q] = st->unm_used[m][q] + st->mat_alloc[m][q];
}

/* Filter (plugin.go:280-330): tryAllocateFromReservation over every GPU-holding matched slot (requiredFromReservation =
 * the pod's required reservation affinity), else Allocate on the node with every matched reservation's allocatable
 * returned.  1 = pass. */
int or_ds_filter_rsv(const kg_node_device* d, const or_ds_pod* p, const kg_node_reservations* r, const or_ds_rsv* st,
                     int required_from_rsv) {
  if (p->skip) return 1;
  if (p->error || !d->has_device) return 0;
  if (!or_dsx_filter(d, p, NULL)) return 0; /* (ABI 17) the RDMA / FPGA types (no GPU-holding reservation with them) */
  if (p->nogpu) return 1;
  if (st->n_matched > 0) {
    int32_t mask = 0;
    if (or_ds_try_rsv(d, p, r, st, st->matched, st->n_matched, 0, 0, NULL, &mask) >= 0) return 1;
    if (required_from_rsv) return 0;
  }
  int64_t pre[KG_MAX_MINORS][3];
  dsr_pre_node(st, pre);
  return or_ds_allocate(d, p, 0, 0, 0, NULL, (const int64_t(*)[3])pre, 0, 0, NULL) >= 0;
}

/* FilterReservation (plugin.go:333-380) of slot s: a pod with device requests can use only a reservation the restore
 * holds GPUs for ("impossible, there is no relevant Reservation information" otherwise); tryAllocateFromReservation
 * with that slot alone, requiredFromReservation = true.  1 = pass. */
int or_ds_filter_reservation(const kg_node_device* d, const or_ds_pod* p, const kg_node_reservations* r,
                             const or_ds_rsv* st, int s) {
  if (p->skip) return 1;
  if (!d->has_device) return 1; /* nodeDeviceInfo == nil: nil */
  int in_state = 0;
  for (int k = 0; k < st->n_matched; k++) in_state |= st->matched[k] == s;
  if (!in_state) return 0;
  const int32_t one = s;
  return or_ds_try_rsv(d, p, r, st, &one, 1, 0, 0, NULL, NULL) >= 0;
}

/* scoreWithReservation (reservation.go:246-272) of slot s: score(requiredDeviceResources = remained for Restricted,
 * preemptible of the slot) — ScoreReservation, and Score for the nominated reservation */
int64_t or_ds_score_slot(const kg_node_device* d, const or_ds_pod* p, const kg_node_reservations* r,
                         const or_ds_rsv* st, int s, int strategy, const int64_t w[3]) {
  if (p->skip || !d->has_device) return 0;
  int in_state = 0;
  for (int k = 0; k < st->n_matched; k++) in_state |= st->matched[k] == s;
  if (!in_state) return 0;
  int64_t pre[KG_MAX_MINORS][3], rem[KG_MAX_MINORS][3];
  dsr_pre_slot(r, st, s, pre, rem);
  if (r->policy[s] == KG_RSV_POLICY_RESTRICTED)
    return or_ds_score_view(d, p, (uint32_t)r->gpu_minors[s], (const int64_t(*)[3])rem, (const int64_t(*)[3])pre,
                            strategy, w);
  return or_ds_score_view(d, p, 0, NULL, (const int64_t(*)[3])pre, strategy, w);
}

/* Score (scoring.go:34-89): the nominated reservation's score when one is nominated, else the node's with every
 * matched reservation's allocatable returned */
int64_t or_ds_score_rsv(const kg_node_device* d, const or_ds_pod* p, const kg_node_reservations* r,
                        const or_ds_rsv* st, int nominated, int strategy, const int64_t w[3]) {
  if (p->skip || p->error || !d->has_device || p->nogpu) return 0;
  if (nominated >= 0) {
    int in_state = 0;
    for (int k = 0; k < st->n_matched; k++) in_state |= st->matched[k] == nominated;
    if (in_state) return or_ds_score_slot(d, p, r, st, nominated, strategy, w);
  }
  int64_t pre[KG_MAX_MINORS][3];
  dsr_pre_node(st, pre);
  return or_ds_score_view(d, p, 0, NULL, (const int64_t(*)[3])pre, strategy, w);
}

/* Reserve (plugin.go:388-437): allocateWithNominatedReservation (the nominated slot alone, not required), else Allocate
 * on the node with the matched reservations' allocatable returned; updateCacheUsed adds the per-instance request to
 * every allocated minor.  Returns the minor mask (0: nothing to allocate), -1 on failure. */
int32_t or_ds_reserve_rsv(kg_node_device* d, const or_ds_pod* p, const kg_node_reservations* r, const or_ds_rsv* st,
                          int nominated, int strategy, const int64_t w[3]) {
  if (p->skip || !d->has_device) return 0;
  if (p->error) return -1;
  if (p->nogpu) return 0;
  int32_t mask = -1;
  if (nominated >= 0 && !(p->reserve)) {
    int in_state = 0;
    for (int k = 0; k < st->n_matched; k++) in_state |= st->matched[k] == nominated;
    if (in_state) {
      const int32_t one = nominated;
      if (or_ds_try_rsv(d, p, r, st, &one, 1, 1, strategy, w, &mask) < 0) mask = -1;
    }
  }
  if (mask < 0) {
    int64_t pre[KG_MAX_MINORS][3];
    dsr_pre_node(st, pre);
    mask = or_ds_allocate(d, p, 0, 0, 0, NULL, (const int64_t(*)[3])pre, 1, strategy, w);
  }
  if (mask <= 0) return mask;
  const or_ds_inst in = or_ds_instance(d, p);
  for (int m = 0; m < KG_MAX_MINORS; m++) {
    if (!((mask >> m) & 1)) continue;
    d->used_core[m] += in.core;
    d->used_memory[m] += in.mem;
    d->used_ratio[m] += in.ratio;
  }
  return mask;
}

/* the allocation of a pod assumed into slot s, on the reservation's minors (appendAllocatedByHints): sign ±1 */
void or_ds_rsv_assign(kg_node_reservations* r, int s, const kg_node_device* d, const or_ds_pod* p, int32_t mask,
                      int sign) {
  mask &= 0xFF; /* the GPU byte of a packed mask */
  if (s < 0 || !r->gpu_minors[s] || mask <= 0) return;
  const or_ds_inst in = or_ds_instance(d, p);
  const int64_t v[3] = {in.core, in.mem, in.ratio};
  for (int m = 0; m < KG_MAX_MINORS; m++) {
    if (!((mask >> m) & 1) || !((r->gpu_minors[s] >> m) & 1)) continue;
    for (int q = 0; q < 3; q++) {
      const int64_t x = r->gpu_allocated[s][m][q] + sign * v[q];
      r->gpu_allocated[s][m][q] = sign > 0 ? x : (x > 0 ? x : 0);
    }
  }
}
