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
 * Scope: the GPU device type without hints, joint allocation, VFs, NUMA affinity or preemption; (ABI 13) reservations
 * that hold GPUs (reservation.go RestoreReservation / tryAllocateFromReservation / scoreWithReservation); (ABI 17) the
 * RDMA / FPGA types of devicehandler_default.go (one percentage resource each, no hints), allocated alongside the GPU
 * type: Filter needs every requested type, Score sums the types (device_allocator.go:92-129, 333-454, 499-522).
 * Minor masks of a pod are packed: GPU bits 0-7, RDMA 8-15, FPGA 16-23.
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
  int skip;          /* no device request of any type (state.skip): Filter passes, Score 0 */
  int reserve;       /* (ABI 13) a reservation's reserve pod: allocateWithNominatedReservation skips it */
  int error;         /* PreFilter UnschedulableAndUnresolvable: invalid request           */
  int unsupported;   /* unused since ABI 17 (RDMA / FPGA are restated)                    */
  int has_mem;       /* the converted request names gpu-memory (else gpu-memory-ratio)   */
  int64_t core, mem, ratio;
  int nogpu;         /* (ABI 17) no GPU-type request (only RDMA / FPGA)                   */
  int64_t xq[KG_DEV_XTYPES]; /* (ABI 17) koordinator.sh/rdma, koordinator.sh/fpga (0 = none) */
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
/* (ABI 17) the RDMA / FPGA part alone: Filter (pre = the types' preemptible amounts per minor, NULL none), raw Score,
 * Reserve (the packed RDMA / FPGA masks, -1 = Insufficient; deviceUsed updated only on success) and Unreserve */
int or_dsx_filter(const kg_node_device* d, const or_ds_pod* p, const int64_t (*pre)[KG_MAX_MINORS]);
int64_t or_dsx_score(const kg_node_device* d, const or_ds_pod* p, int strategy, const int64_t w[KG_DEV_XTYPES]);
int32_t or_dsx_reserve(kg_node_device* d, const or_ds_pod* p, int strategy, const int64_t w[KG_DEV_XTYPES]);
void or_dsx_release(kg_node_device* d, const or_ds_pod* p, int32_t packed);
/* scoreDevice for one minor (scoring.go:183-203) */
int64_t or_ds_score_minor(const kg_node_device* d, int minor, const or_ds_pod* p, const or_ds_inst* in,
                          int strategy, const int64_t w[3]);
/* DefaultNormalizeScore(MaxNodeScore, reverse=false) (upstream pluginhelper; frameworkext/normalize_score.go:24-52) */
void or_default_normalize(int64_t* scores, int64_t n);
/* Python binding helper: or_ds_instance → {count, core, mem, ratio}; returns ok */
int or_ds_instance_flat(const kg_node_device* d, const or_ds_pod* p, int64_t* out);

/* (ABI 13) reservations holding GPUs: the DeviceShare restore of one node for one pod (reservation.go:84-171) */
typedef struct or_ds_rsv {
  int n_matched;
  int32_t matched[KG_MAX_RSV_SLOTS];        /* GPU-holding matched slots, in the Reservation restore's order */
  int64_t unm_used[KG_MAX_MINORS][3];       /* mergedUnmatchedUsed                                           */
  int64_t mat_allocd[KG_MAX_MINORS][3];     /* mergedMatchedAllocated                                        */
  int64_t mat_alloc[KG_MAX_MINORS][3];      /* mergedMatchedAllocatable                                      */
} or_ds_rsv;
void or_ds_rsv_init(const kg_node_reservations* r, const int32_t* matched, int n_matched, const int32_t* unmatched,
                    int n_unmatched, or_ds_rsv* out);
int32_t or_ds_allocate(const kg_node_device* d, const or_ds_pod* p, uint32_t required, uint32_t preferred,
                       uint32_t rr_minors, const int64_t (*rr)[3], const int64_t (*pre)[3], int scored, int strategy,
                       const int64_t w[3]);
int64_t or_ds_score_view(const kg_node_device* d, const or_ds_pod* p, uint32_t rr_minors, const int64_t (*rr)[3],
                         const int64_t (*pre)[3], int strategy, const int64_t w[3]);
int or_ds_try_rsv(const kg_node_device* d, const or_ds_pod* p, const kg_node_reservations* r, const or_ds_rsv* st,
                  const int32_t* slots, int n_slots, int scored, int strategy, const int64_t w[3], int32_t* mask);
int or_ds_filter_rsv(const kg_node_device* d, const or_ds_pod* p, const kg_node_reservations* r, const or_ds_rsv* st,
                     int required_from_rsv);
int or_ds_filter_reservation(const kg_node_device* d, const or_ds_pod* p, const kg_node_reservations* r,
                             const or_ds_rsv* st, int s);
int64_t or_ds_score_slot(const kg_node_device* d, const or_ds_pod* p, const kg_node_reservations* r,
                         const or_ds_rsv* st, int s, int strategy, const int64_t w[3]);
int64_t or_ds_score_rsv(const kg_node_device* d, const or_ds_pod* p, const kg_node_reservations* r,
                        const or_ds_rsv* st, int nominated, int strategy, const int64_t w[3]);
int32_t or_ds_reserve_rsv(kg_node_device* d, const or_ds_pod* p, const kg_node_reservations* r, const or_ds_rsv* st,
                          int nominated, int strategy, const int64_t w[3]);
void or_ds_rsv_assign(kg_node_reservations* r, int s, const kg_node_device* d, const or_ds_pod* p, int32_t mask,
                      int sign);

#ifdef __cplusplus
}
#endif
#endif
