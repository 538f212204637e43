/*
 * deviceshare.h — CPU restatement of the DeviceShare plugin's GPU path (Filter, Score, NormalizeScore, Reserve).
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h): the checker and CPU baseline, never linked by the engine.
 *
 * Restates (paths under /root/reference/pkg/scheduler/plugins/deviceshare):
 *   utils.go:37-216            GetPodDeviceRequests / ValidateDeviceRequest / ConvertDeviceRequest
 *   devicehandler_gpu.go:40-98 CalcDesiredRequestsAndCount, fillGPUTotalMem, memoryRatioToBytes/BytesToRatio
 *   device_allocator.go:70-129,131-155,333-454,499-522  Prepare/Allocate/filterNodeDevice/defaultAllocateDevices/score
 *   device_cache.go:124-174,314-391,505-523  updateCacheUsed/resetDeviceFree/calcFreeWithPreemptible/filter/build
 *   device_resources.go:164-208  scoreDevices + sortDeviceResourcesByMinor (score desc, minor asc)
 *   scoring.go:34-97,183-308   Score, NormalizeScore (DefaultNormalizeScore), scoreDevice/scoreNode, scorers
 * Scope: the GPU device type without hints, joint allocation, VFs, NUMA affinity, reservations or preemption.
 * Map-order pins: fillGPUTotalMem takes the lowest healthy minor (the reference iterates a Go map; every GPU of
 * a node is the same model, device_cache.go comment at devicehandler_gpu.go:69-70).
 */
#ifndef KOORD_ORACLE_DEVICESHARE_H_
#define KOORD_ORACLE_DEVICESHARE_H_
#include <stdint.h>
#include "../include/koordgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* DeviceShare preFilterState for the GPU device type (preparePod, utils.go:204-230) */
typedef struct or_ds_pod {
  int skip;          /* no device request: Filter passes, Score 0                         */
  int error;         /* PreFilter UnschedulableAndUnresolvable: invalid request           */
  int unsupported;   /* rdma / fpga requests: outside the restated scope                  */
  int has_mem;       /* the converted request names gpu-memory (else gpu-memory-ratio)   */
  int64_t core, mem, ratio;
} or_ds_pod;

/* per-instance request on one node (CalcDesiredRequestsAndCount) */
typedef struct or_ds_inst {
  int ok;            /* 0: Insufficient gpu devices / no healthy GPU (UnschedulableAndUnresolvable) */
  int count;         /* desiredCount                                                          */
  int64_t core, mem, ratio;
} or_ds_inst;

int or_ds_pod_init(const kg_pod* pod, or_ds_pod* out);
/* memoryBytesToRatio / memoryRatioToBytes (devicehandler_gpu.go:92-98) */
int64_t or_ds_memory_bytes_to_ratio(int64_t bytes, int64_t total_memory);
int64_t or_ds_memory_ratio_to_bytes(int64_t ratio, int64_t total_memory);
or_ds_inst or_ds_instance(const kg_node_device* d, const or_ds_pod* p);
/* Unreserve (plugin.go:440-455): each minor of `minors` gives the pod's per-instance request back */
void or_ds_release(kg_node_device* d, const or_ds_pod* p, int32_t minors);
/* Filter: 1 pass, 0 reject.  A node without a Device object rejects device pods (NodeResourcesFit on the device
 * extended resources, whose allocatable is then 0). */
int or_ds_filter(const kg_node_device* d, const or_ds_pod* p);
/* Score (raw, before NormalizeScore); strategy KG_STRATEGY_*, weights = gpu-core, gpu-memory, gpu-memory-ratio */
int64_t or_ds_score(const kg_node_device* d, const or_ds_pod* p, int strategy, const int64_t w[3]);
/* Reserve: allocates minors (defaultAllocateDevices order) and adds the per-instance request to their used
 * resources.  Returns the minor bitmask (0 = no allocation needed: skip / no Device object), -1 on failure. */
int32_t or_ds_reserve(kg_node_device* d, const or_ds_pod* p, int strategy, const int64_t w[3]);
/* scoreDevice for one minor (scoring.go:183-203) */
int64_t or_ds_score_minor(const kg_node_device* d, int minor, const or_ds_pod* p, const or_ds_inst* in,
                          int strategy, const int64_t w[3]);
/* DefaultNormalizeScore(MaxNodeScore, reverse=false) (upstream pluginhelper; frameworkext/normalize_score.go:24-52) */
void or_default_normalize(int64_t* scores, int64_t n);
/* Python binding helper: or_ds_instance → {count, core, mem, ratio}; returns ok */
int or_ds_instance_flat(const kg_node_device* d, const or_ds_pod* p, int64_t* out);

#ifdef __cplusplus
}
#endif
#endif
