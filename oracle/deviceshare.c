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
  const int64_t* q = pod->device_requests;
  for (int r = 0; r < KG_DEV_RES_MAX; r++)
    if (q[r] < 0) { out->error = 1; return 0; }
  if (q[KG_DEV_FPGA] != 0 || q[KG_DEV_RDMA] != 0) out->unsupported = 1;
  static const int flag_of[6] = {F_NVIDIA, F_DCU, F_KGPU, F_CORE, F_MEM, F_RATIO};
  unsigned comb = 0;
  for (int r = 0; r < 6; r++)
    if (q[r] != 0) comb |= (unsigned)flag_of[r]; /* quotav1.RemoveZeros */
  if (comb == 0) { out->skip = !out->unsupported; return 0; }
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
  if (p->skip || p->error || !d->has_device) return 0;
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

/* flat helper for the Python binding: CalcDesiredRequestsAndCount → out = {count, core, mem, ratio} */
int or_ds_instance_flat(const kg_node_device* d, const or_ds_pod* p, int64_t* out) {
  const or_ds_inst in = or_ds_instance(d, p);
  out[0] = in.count; out[1] = in.core; out[2] = in.mem; out[3] = in.ratio;
  return in.ok;
}
