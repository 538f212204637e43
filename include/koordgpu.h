/*
 * koordgpu.h — C ABI of the MI355X batch Filter/Score engine for koord-scheduler.
 *
 * This is the drop-in boundary. Everything that crosses it is a flat,
 * pointer-free struct of int64 fields (cgo rule: no Go pointers inside), a caller-owned
 * array, or an opaque engine handle. Device memory is owned by the engine.
 *
 * What each entry point replaces in the reference (all paths under /root/reference):
 *
 *   kg_engine_create        plugin construction: loadaware.New (pkg/scheduler/plugins/loadaware/load_aware.go:76-110)
 *                           with LoadAwareSchedulingArgs (pkg/scheduler/apis/config/types.go:30-76, defaults
 *                           v1beta2/defaults.go:76-99) + upstream NodeResourcesFit args + profile score weights
 *                           (config/manager/scheduler-config.yaml:82-91).
 *   kg_nodes_upsert         upstream scheduler-cache node add/update after the node transformer
 *                           (pkg/util/transformer/node_transformer.go:40-75); NodeInfo.Allocatable.
 *   kg_node_metrics_update  NodeMetric lister reads done per (pod,node) in LoadAware Filter/Score
 *                           (load_aware.go:133,278) — hoisted to ingest.
 *   kg_pods_add             assigned-pod informer add: upstream NodeInfo.AddPod + podAssignCache.OnAdd/assign
 *                           (pkg/scheduler/plugins/loadaware/pod_assign_cache.go:53-68,82-88).
 *   kg_pods_remove          pod delete / Unreserve / ForgetPod: NodeInfo.RemovePod + podAssignCache.unAssign
 *                           (pod_assign_cache.go:70-80,102-117; load_aware.go:265-267).
 *   kg_pods_schedule        the per-pod hot loop: upstream findNodesThatPassFilters + prioritizeNodes + selectHost +
 *                           assume, reached in koordinator through Scheduler.SchedulePod interception
 *                           (pkg/scheduler/frameworkext/framework_extender_factory.go:136-185) and
 *                           FrameworkExtender.RunFilterPluginsWithNominatedPods / RunScorePlugins
 *                           (framework_extender.go:204-258). Sequential FIFO semantics; assume applied on device.
 *   kg_pods_evaluate        one pod against every node WITHOUT assume: per-node Filter status and per-plugin Score,
 *                           i.e. RunFilterPlugins + RunScorePlugins for one pod (framework_extender.go:204-258) —
 *                           also what --debug-scores prints (frameworkext/debug.go:61-108).
 *   kg_nodes_device_upsert  DeviceShare nodeDeviceCache.updateNodeDevice (deviceshare/device_cache.go:485-523) + the
 *                           assigned-pod informer's updateCacheUsed (device_cache.go:124-135, eventhandler_pod.go).
 *   kg_pods_evaluate_device DeviceShare Filter + Score for one pod on every node (deviceshare/plugin.go:280-330,
 *                           scoring.go:34-89).
 *   kg_quotas_set           ElasticQuota PreFilter/Reserve state: per quota used / non-preemptible used (QuotaInfo,
 *                           elasticquota/core/quota_info.go) and usedLimit (getQuotaInfoUsedLimit: runtime or max,
 *                           elasticquota/plugin_helper.go:237-246) + min, as the Go GroupQuotaManager holds them.
 *   kg_last_error           error text for the last failing call on this thread (maps to framework.NewStatus(Error,…)).
 *
 * Units follow the reference's getResourceValue (load_aware/helper.go:146-151): cpu-like resources in
 * milli-units (Quantity.MilliValue), everything else in Quantity.Value.  Quantities must be integral.
 */
#ifndef KOORDGPU_H_
#define KOORDGPU_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KG_ABI_VERSION 17

/* ---- resource slots (fixed order) ------------------------------------------------------- */
enum {
  KG_RES_CPU = 0,          /* cpu, milli-cores                                   */
  KG_RES_MEMORY = 1,       /* memory, bytes                                      */
  KG_RES_EPHEMERAL = 2,    /* ephemeral-storage, bytes                           */
  KG_RES_BATCH_CPU = 3,    /* kubernetes.io/batch-cpu (Value)                    */
  KG_RES_BATCH_MEMORY = 4, /* kubernetes.io/batch-memory (Value)                 */
  KG_RES_MID_CPU = 5,      /* kubernetes.io/mid-cpu (Value)                      */
  KG_RES_MID_MEMORY = 6,   /* kubernetes.io/mid-memory (Value)                   */
  KG_RES_RESERVED7 = 7,
  KG_RES_MAX = 8
};

/* koordinator priority classes (apis/extension/priority.go:29-35); the caller passes the result of
 * extension.GetPodPriorityClassWithDefault (apis/extension/priority_utils.go:26-48). */
enum { KG_PRIO_NONE = 0, KG_PRIO_PROD = 1, KG_PRIO_MID = 2, KG_PRIO_BATCH = 3, KG_PRIO_FREE = 4 };

/* NodeNUMAResource vocabulary (apis/extension/numa_aware.go:89-144, apis/extension/qos.go:23-28) */
enum { KG_QOS_NONE = 0, KG_QOS_LSE = 1, KG_QOS_LSR = 2, KG_QOS_LS = 3, KG_QOS_BE = 4, KG_QOS_SYSTEM = 5 };
/* CPUBindPolicy: "" / Default / FullPCPUs / SpreadByPCPUs / ConstrainedBurst */
/* CPUExclusivePolicy (apis/scheduling/config types; ResourceSpec.PreferredCPUExclusivePolicy, plugin.go:261) */
enum { KG_EXCL_NONE = 0, KG_EXCL_PCPU_LEVEL = 1, KG_EXCL_NUMA_NODE_LEVEL = 2 };
enum { KG_BIND_NONE = 0, KG_BIND_DEFAULT = 1, KG_BIND_FULL_PCPUS = 2, KG_BIND_SPREAD_BY_PCPUS = 3,
       KG_BIND_CONSTRAINED_BURST = 4 };
/* NodeCPUBindPolicy label (or kubelet static policy with full-pcpus-only) */
enum { KG_NODE_BIND_NONE = 0, KG_NODE_BIND_FULL_PCPUS_ONLY = 1, KG_NODE_BIND_SPREAD_BY_PCPUS = 2 };
/* NUMATopologyPolicy (node label, else NodeResourceTopology) */
enum { KG_NUMA_POLICY_NONE = 0, KG_NUMA_POLICY_BEST_EFFORT = 1, KG_NUMA_POLICY_RESTRICTED = 2,
       KG_NUMA_POLICY_SINGLE_NUMA_NODE = 3 };
/* ScoringStrategy type / NUMAAllocateStrategy */
enum { KG_STRATEGY_LEAST_ALLOCATED = 0, KG_STRATEGY_MOST_ALLOCATED = 1 };
#define KG_MAX_NUMA 4
/* NodeMetric AggregatedNodeUsages (apis/slo/v1alpha1/nodemetric_types.go): ≤ KG_MAX_AGG durations, each with the
 * KG_AGG_TYPES percentile kinds of extension.AggregationType (apis/extension/constants.go:45-54) */
#define KG_MAX_AGG 4
#define KG_AGG_TYPES 5
enum { KG_AGG_NONE = 0, KG_AGG_AVG = 1, KG_AGG_P50 = 2, KG_AGG_P90 = 3, KG_AGG_P95 = 4, KG_AGG_P99 = 5 };
#define KG_MAX_CPUS 256

/* DeviceShare: device resources a pod may request (deviceshare/utils.go:46-56, apis/extension/resource.go) */
enum {
  KG_DEV_NVIDIA_GPU = 0,        /* nvidia.com/gpu (count)                              */
  KG_DEV_HYGON_DCU = 1,         /* dcu.com/gpu (count)                                 */
  KG_DEV_KOORD_GPU = 2,         /* koordinator.sh/gpu (percentage)                     */
  KG_DEV_GPU_CORE = 3,          /* koordinator.sh/gpu-core (percentage)                */
  KG_DEV_GPU_MEMORY = 4,        /* koordinator.sh/gpu-memory (bytes)                   */
  KG_DEV_GPU_MEMORY_RATIO = 5,  /* koordinator.sh/gpu-memory-ratio (percentage)        */
  KG_DEV_FPGA = 6,              /* koordinator.sh/fpga (percentage; (ABI 17) accelerated) */
  KG_DEV_RDMA = 7,              /* koordinator.sh/rdma (percentage; (ABI 17) accelerated) */
  KG_DEV_RES_MAX = 8
};
#define KG_MAX_MINORS 8         /* GPU minors per node */

/* status codes: 0 ok, <0 error class (framework.Error on the Go side) */
enum {
  KG_OK = 0,
  KG_E_INVALID = -1,     /* invalid argument / validation failure   */
  KG_E_DEVICE = -2,      /* HIP runtime error                       */
  KG_E_COLLECTIVE = -3,  /* RCCL error                              */
  KG_E_NOMEM = -4,       /* allocation failure                      */
  KG_E_UNSUPPORTED = -5  /* input outside the accelerated profile   */
};

/* per-node filter reasons written by kg_pods_evaluate (bit set = plugin rejected the node) */
enum {
  KG_REJECT_FIT_PODS = 1 << 0,      /* NodeResourcesFit: Too many pods                 */
  KG_REJECT_FIT_CPU = 1 << 1,       /* NodeResourcesFit: Insufficient cpu              */
  KG_REJECT_FIT_MEMORY = 1 << 2,    /* NodeResourcesFit: Insufficient memory           */
  KG_REJECT_LOADAWARE = 1 << 3,     /* LoadAwareScheduling: usage exceed threshold     */
  KG_REJECT_INVALID_NODE = 1 << 4,  /* deleted / never-upserted slot                   */
  KG_REJECT_NUMA = 1 << 5,          /* NodeNUMAResource (topology, cpuset, NUMA admit) */
  KG_REJECT_DEVICE = 1 << 6,        /* DeviceShare (Insufficient gpu devices)          */
  KG_REJECT_FIT_OTHER = 1 << 7,     /* NodeResourcesFit: Insufficient ephemeral-storage / a scalar resource
                                       (KG_RES_EPHEMERAL .. KG_RES_MID_MEMORY; reservation/plugin.go:469-479) */
  KG_REJECT_RESERVATION = 1 << 8,   /* (ABI 11) Reservation Filter (kg_pods_filter_preemption): preemption failed /
                                       no reservation meets the requirements / reservation affinity */
  KG_REJECT_SPREAD = 1 << 9,        /* (ABI 12) PodTopologySpread: DoNotSchedule constraint's skew exceeded   */
  KG_REJECT_INTERPOD = 1 << 10,     /* (ABI 12) InterPodAffinity: affinity / anti-affinity / existing pods'
                                       anti-affinity rules not matched                                          */
  KG_REJECT_NO_VICTIMS = 1 << 11,   /* (ABI 14) kg_pods_select_victims: the candidate has no potential victims
                                       ("No victims found on node": UnschedulableAndUnresolvable)              */
  KG_REJECT_TAINT = 1 << 12,        /* (ABI 16) TaintToleration (preemption dry run): an untolerated taint    */
  KG_REJECT_NODE_AFFINITY = 1 << 13 /* (ABI 16) NodeAffinity (preemption dry run): nodeSelector / required
                                       terms do not match                                                      */
};

/* node flags */
enum {
  KG_NODE_VALID = 1 << 0,
  KG_NODE_HAS_RAW_ALLOCATABLE = 1 << 1,   /* node.koordinator.sh/raw-allocatable annotation present */
  KG_NODE_HAS_CUSTOM_THRESHOLDS = 1 << 2  /* custom-usage-thresholds annotation parsed OK            */
};

/* pod flags */
enum {
  KG_POD_DAEMONSET = 1 << 0,
  KG_POD_NON_PREEMPTIBLE = 1 << 1,  /* extension.IsPodNonPreemptible (ElasticQuota min check) */
  KG_POD_RESERVE = 1 << 2,          /* a reservation's reserve pod (kg_pods_add): NodeInfo only — the LoadAware
                                       assign cache is fed by the pod informer, which never sees it */
  /* request-key presence (PodRequestsAndLimits keys, even when zero): with KG_POD_REQUEST_KEYS set the next two bits
   * say whether the cpu / memory keys exist; without it a key exists iff its request is non-zero.  Only
   * filterWithReservations looks at keys (Intersection(rInfo.ResourceNames, pod request names),
   * reservation/plugin.go:392-395). */
  KG_POD_REQUEST_KEYS = 1 << 3,
  KG_POD_CPU_KEY = 1 << 4,
  KG_POD_MEM_KEY = 1 << 5,
  /* (ABI 11) tolerated_taints was compiled against the first taint_count taints of the caller's taint table; without
   * it the mask does not depend on the table (no tolerations, or a toleration with no key, operator Exists and no
   * effect, for which the caller passes all ones) */
  KG_POD_TAINT_TABLE = 1 << 6
};
#define KG_MAX_QUOTAS 64

/* Engine configuration: plugin args + profile weights + engine tuning.  All int64 for a padding-free
 * layout.  A threshold/weight of 0 means "resource absent from the map". */
typedef struct kg_config {
  int64_t abi_version;                         /* must be KG_ABI_VERSION                              */
  /* LoadAwareSchedulingArgs (config/types.go:30-76) */
  int64_t la_filter_expired_node_metrics;      /* bool                                                */
  int64_t la_node_metric_expiration_seconds;   /* <0 = nil                                            */
  int64_t la_resource_weights[KG_RES_MAX];
  int64_t la_usage_thresholds[KG_RES_MAX];
  int64_t la_prod_usage_thresholds[KG_RES_MAX];
  int64_t la_estimated_scaling_factors[KG_RES_MAX];
  int64_t la_score_according_prod_usage;       /* bool                                                */
  /* NodeResourcesFit (upstream) LeastAllocated scoring strategy resources */
  int64_t fit_resource_weights[KG_RES_MAX];
  /* profile: plugins enabled at the Filter / Score extension points and their Score weights */
  int64_t fit_filter;                          /* NodeResourcesFit at Filter                          */
  int64_t fit_score;                           /* NodeResourcesFit at Score                           */
  int64_t la_filter;                           /* LoadAwareScheduling at Filter                       */
  int64_t la_score;                            /* LoadAwareScheduling at Score                        */
  int64_t weight_fit;
  int64_t weight_loadaware;
  /* NodeNUMAResourceArgs (config/types.go; defaults v1beta2/defaults.go:101-137) + profile */
  int64_t numa_filter;                         /* NodeNUMAResource at Filter                          */
  int64_t numa_score;                          /* NodeNUMAResource at Score                           */
  int64_t weight_numa;
  int64_t numa_default_cpu_bind_policy;        /* KG_BIND_* (default FullPCPUs)                       */
  int64_t numa_scoring_strategy;               /* ScoringStrategy.Type: KG_STRATEGY_*                 */
  int64_t numa_scoring_weights[2];             /* ScoringStrategy.Resources: cpu, memory              */
  int64_t numa_numa_scoring_strategy;          /* NUMAScoringStrategy.Type (also the default NUMA     */
  int64_t numa_numa_scoring_weights[2];        /* allocate strategy, util.go:26-32)                   */
  /* DeviceShareArgs (config/types.go; defaults v1beta2/defaults.go:187-208) + profile.  ScoringStrategy.Resources
   * weights over the GPU resources: gpu-core, gpu-memory, gpu-memory-ratio (default 0, 0, 1; rdma/fpga weights
   * only touch RDMA/FPGA devices, which are not accelerated). */
  int64_t ds_filter;                           /* DeviceShare at Filter                               */
  int64_t ds_score;                            /* DeviceShare at Score (NormalizeScore: DefaultNormalizeScore) */
  int64_t weight_deviceshare;
  int64_t ds_scoring_strategy;                 /* KG_STRATEGY_* (LeastAllocated only is accelerated)  */
  int64_t ds_scoring_weights[3];               /* gpu-core, gpu-memory, gpu-memory-ratio              */
  /* engine tuning (0 = default) */
  int64_t batch_pods;                          /* pods resolved per device round (B, 1..64)           */
  int64_t pods_per_wave;                       /* pods one eval wave scores per round (1..B)          */
  int64_t device_id;                           /* HIP device ordinal (-1 = current)                   */
  /* Reservation (reservation/plugin.go:318-559, scoring.go:42-203; weight scheduler-config.yaml:90-91) */
  int64_t reservation_filter;                  /* Reservation at Filter (+ BeforePreFilter restore)   */
  int64_t reservation_score;                   /* Reservation at PreScore/Score (NormalizeScore: DefaultNormalizeScore) */
  int64_t weight_reservation;
  int64_t pipeline_depth;                      /* rounds in flight (1..4; 0 = default 2) for monotone profiles  */
  /* LoadAwareSchedulingArgs.Aggregated (config/types.go:56-76): percentile usage for Filter / Score */
  int64_t la_agg_usage_thresholds[KG_RES_MAX]; /* Aggregated.UsageThresholds (0 = absent)            */
  int64_t la_agg_usage_type;                   /* UsageAggregationType KG_AGG_* (0 = "")              */
  int64_t la_agg_usage_duration_ns;            /* UsageAggregatedDuration (0 = the longest recorded) */
  int64_t la_agg_score_type;                   /* ScoreAggregationType KG_AGG_* (0 = "")              */
  int64_t la_agg_score_duration_ns;            /* ScoreAggregatedDuration (0 = the longest recorded) */
  /* upstream default plugins of a stock profile (k8s v1.24.15 pkg/scheduler/framework/plugins, not vendored; restated
   * as published — see DESIGN.md §3.13).  Evaluated on the exact per-pod pass.  Weights default 1 upstream. */
  int64_t taint_filter;                        /* TaintToleration at Filter (NoSchedule / NoExecute taints)      */
  int64_t taint_score;                         /* TaintToleration at Score (PreferNoSchedule; reverse-normalized) */
  int64_t weight_taint;
  int64_t affinity_filter;                     /* NodeAffinity at Filter (nodeSelector + required terms)         */
  int64_t affinity_score;                      /* NodeAffinity at Score (preferred terms; normalized)            */
  int64_t weight_affinity;
  int64_t balanced_score;                      /* NodeResourcesBalancedAllocation at Score                       */
  int64_t weight_balanced;
  int64_t balanced_resources;                  /* bit r: resource r (cpu 0, memory 1) is in its Resources list   */
  int64_t image_score;                         /* (ABI 10) ImageLocality at Score (no NormalizeScore)            */
  int64_t weight_image;
  /* (ABI 12) PodTopologySpread and InterPodAffinity with topologyKey kubernetes.io/hostname (k8s v1.24.15
   * podtopologyspread/{filtering,scoring}.go, interpodaffinity/{filtering,scoring}.go; not vendored — DESIGN.md §3.15).
   * Evaluated on the exact per-pod pass, one pod per pass.  Upstream default weights: 2 and 1. */
  int64_t spread_filter;                       /* PodTopologySpread at Filter (DoNotSchedule constraint)         */
  int64_t spread_score;                        /* PodTopologySpread at Score (ScheduleAnyway; its NormalizeScore) */
  int64_t weight_spread;
  int64_t interpod_filter;                     /* InterPodAffinity at Filter                                     */
  int64_t interpod_score;                      /* InterPodAffinity at Score (min-max NormalizeScore)             */
  int64_t weight_interpod;
  int64_t hard_pod_affinity_weight;            /* InterPodAffinityArgs.HardPodAffinityWeight (default 1)         */
  /* (ABI 15) several ranks (kg_engine_create n_ranks > 1): KG_MULTI_RANK_SHARD evaluates a node shard per rank and
   * exchanges each round's candidates; KG_MULTI_RANK_REPLICA makes every rank a replica of one GPU (the whole table, no
   * exchange, the same placements); AUTO shards only tables large enough for it to pay. */
  int64_t multi_rank_mode;
  /* (ABI 17) DeviceShareArgs.ScoringStrategy.Resources weights of koordinator.sh/rdma and koordinator.sh/fpga (the
   * scorer of the RDMA / FPGA device types; v1beta2 default 1 each) */
  int64_t ds_scoring_weights_x[2];
  int64_t reserved[1];
} kg_config;
enum { KG_MULTI_RANK_AUTO = 0, KG_MULTI_RANK_SHARD = 1, KG_MULTI_RANK_REPLICA = 2 };

/* One node (snapshot index = position given by the caller). */
typedef struct kg_node {
  int64_t allocatable[KG_RES_MAX];             /* NodeInfo.Allocatable                                */
  int64_t allowed_pods;                        /* Allocatable.AllowedPodNumber                        */
  int64_t flags;                               /* KG_NODE_*                                           */
  int64_t raw_allocatable[KG_RES_MAX];         /* extension.GetNodeRawAllocatable (EstimateNode)      */
  int64_t raw_allocatable_present[KG_RES_MAX]; /* key present in the annotation map                   */
  int64_t custom_usage_thresholds[KG_RES_MAX]; /* extension.GetCustomUsageThresholds; -1 = absent      */
  int64_t custom_prod_usage_thresholds[KG_RES_MAX];
  /* the annotation's CustomUsageThresholds.AggregatedUsage (apis/extension/load_aware.go:40-50) */
  int64_t custom_agg_thresholds[KG_RES_MAX];   /* UsageThresholds; -1 = absent                        */
  int64_t custom_agg_type;                     /* UsageAggregationType KG_AGG_* (0 = "")              */
  int64_t custom_agg_duration_ns;              /* UsageAggregatedDuration (0 = nil / the longest)    */
} kg_node;

/* NodeMetric status summary for one node (apis/slo/v1alpha1/nodemetric_types.go:107-122). */
typedef struct kg_node_metric {
  int64_t present;                             /* lister Get succeeded                                */
  int64_t has_node_metric;                     /* Status.NodeMetric != nil                            */
  int64_t has_update_time;                     /* Status.UpdateTime != nil                            */
  int64_t update_time_unix_nano;
  int64_t node_usage[KG_RES_MAX];              /* Status.NodeMetric.NodeUsage (cpu milli)             */
  int64_t node_usage_present[KG_RES_MAX];
  int64_t pods_metric_count;                   /* len(Status.PodsMetric)                              */
  int64_t prod_pods_usage[KG_RES_MAX];         /* Σ PodsMetric usage of prod pods (buildPodMetricMap  */
                                               /* filterProdPod=true + sumPodUsages, helper.go:153-186) */
  int64_t agg_count;                           /* len(Status.NodeMetric.AggregatedNodeUsages)         */
  int64_t agg_duration_ns[KG_MAX_AGG];         /* AggregatedUsage.Duration                            */
  int64_t agg_usage[KG_MAX_AGG][KG_AGG_TYPES][2];  /* Usage[type] cpu (milli) / memory (bytes)       */
  int64_t agg_present[KG_MAX_AGG][KG_AGG_TYPES];   /* bit r: resource r in that ResourceList (0 = empty) */
  int64_t report_interval_ns;                  /* Spec.CollectPolicy.ReportIntervalSeconds (0 = default 60 s,
                                                  getNodeMetricReportInterval, loadaware/helper.go:43-48) */
} kg_node_metric;

/* One entry of NodeMetric.Status.PodsMetric (PodMetricInfo) as buildPodMetricMap (loadaware/helper.go:153-170)
 * reads it: the pod's identity, its usage (cpu milli / memory bytes) and whether the pod is prod priority
 * (GetPodPriorityClassWithDefault == koord-prod, for the ScoreAccordingProdUsage view). */
typedef struct kg_pod_metric {
  int64_t uid;                                 /* the pod's identity (same value as kg_pod.uid)        */
  int64_t usage[2];                            /* PodUsage cpu (milli), memory (bytes)                 */
  int64_t usage_present;                       /* bit r: resource r is a key of PodUsage               */
  int64_t prod;                                /* the pod's priority class is koord-prod               */
} kg_pod_metric;

/* Node affinity terms a pod may carry (more: the pod stays on the Go path) */
#define KG_MAX_AFF_TERMS 4
/* Containers an ImageLocality pod may carry (more: the pod stays on the Go path) */
#define KG_MAX_CONTAINERS 8
#define KG_MAX_MATCH_GROUPS 16   /* (ABI 12) PodTopologySpread / InterPodAffinity match groups */
#define KG_MAX_POD_PREFERRED 4   /* (ABI 12) preferred pod (anti-)affinity terms per pod */
#define KG_MAX_SPREAD 4          /* (ABI 12) topology spread constraints per pod */
#define KG_MAX_ZONES 64          /* (ABI 12) topology.kubernetes.io/zone domains */
enum {
  KG_SPREAD_HARD = 1 << 0,       /* whenUnsatisfiable: DoNotSchedule (else ScheduleAnyway) */
  KG_SPREAD_ZONE = 1 << 1,       /* topologyKey topology.kubernetes.io/zone (else kubernetes.io/hostname) */
  /* (ABI 13) the constraint is one of the plugin's system defaults, applied because the pod has no constraints of its
   * own (podtopologyspread PreScore: requireAllTopologies = len(pod.Spec.TopologySpreadConstraints) > 0 ||
   * !systemDefaulted).  Set on every constraint of such a pod or on none; only with ScheduleAnyway.  Scoring then
   * ignores no node: a filtered node without the zone label skips that constraint's term and adds the empty zone value
   * to the constraint's topology size (scoring.go initPreScoreState, Score). */
  KG_SPREAD_SYSTEM_DEFAULT = 1 << 2
};

/* One pod, pre-decoded by the caller (PodRequestsAndLimits semantics, pkg/util/pod_resources_utils.go:48-64). */
typedef struct kg_pod {
  int64_t requests[KG_RES_MAX];
  int64_t limits[KG_RES_MAX];
  int64_t nonzero_requests[2];                 /* schedutil.GetNonzeroRequests: cpu milli, memory     */
  int64_t priority_class;                      /* KG_PRIO_*                                           */
  int64_t flags;                               /* KG_POD_*                                            */
  int64_t qos;                                 /* extension.GetPodQoSClassRaw: KG_QOS_*               */
  int64_t required_cpu_bind_policy;            /* ResourceSpec annotation: KG_BIND_*                  */
  int64_t preferred_cpu_bind_policy;           /* ResourceSpec annotation: KG_BIND_*                  */
  int64_t device_requests[KG_DEV_RES_MAX];     /* PodRequestsAndLimits of the device resources (KG_DEV_*) */
  int64_t quota_id;                            /* 1 + index into the kg_quotas_set table; 0 = no ElasticQuota */
  int64_t reservation_owner_mask;              /* bit g set: the pod matches the owners of reservation owner  */
                                               /* group g (kg_node_reservations.owner), as the caller decoded  */
                                               /* ReservationInfo.Match (reservation_info.go:231-236,          */
                                               /* MatchReservationOwners pkg/util/reservation:389-410) once per */
                                               /* distinct owner spec; 0 = matches none                         */
  int64_t reservation_flags;                   /* KG_POD_RSV_*                                        */
  int64_t uid;                                 /* the pod's identity (matches kg_pod_metric.uid; 0 = none)  */
  int64_t assign_time_unix_nano;               /* kg_pods_add: the podAssignCache timestamp of the pod  */
                                               /* (pod_assign_cache.go:62-66); scheduled pods take the engine clock */
  /* TaintToleration / NodeAffinity (ABI 8), over the caller's taint and predicate tables (kg_node_predicates): */
  uint64_t tolerated_taints;                   /* bit t: the pod's tolerations tolerate taint t                 */
  uint64_t node_selector;                      /* predicates pod.Spec.NodeSelector requires (all must hold)     */
  int64_t n_required_terms;                    /* required NodeSelectorTerms (0 = no required node affinity)   */
  uint64_t required_terms[KG_MAX_AFF_TERMS];   /* term k holds iff every listed predicate holds (0 = empty term: */
                                               /* matches no node)                                             */
  int64_t n_preferred_terms;                   /* preferred PreferredSchedulingTerms                            */
  uint64_t preferred_terms[KG_MAX_AFF_TERMS];
  int64_t preferred_weights[KG_MAX_AFF_TERMS];
  /* (ABI 9) ResourceSpec.PreferredCPUExclusivePolicy (KG_EXCL_*): cpuAccumulator's filterExclusive passes keep the
   * pod off the cores (PCPULevel) / NUMA nodes (NUMANodeLevel) that hold cpus of pods with the same policy
   * (cpu_accumulator.go:247-330), and Reserve records the pod's cpus with it (node_allocation.go:68-90) */
  int64_t preferred_cpu_exclusive_policy;
  /* (ABI 10) ImageLocality (k8s v1.24.15 imagelocality/image_locality.go, not vendored): the pod's containers
   * (pod.Spec.Containers, len ≤ KG_MAX_CONTAINERS) — per container the bit of its normalized image name in the caller's
   * image table (kg_node_predicates.images; -1: no node holds the image) and that image's scaledImageScore, which is
   * node-independent: int64(float64(ImageStateSummary.Size) * float64(NumNodes) / float64(totalNumNodes)) */
  int64_t n_containers;
  int64_t container_image_bit[KG_MAX_CONTAINERS];
  int64_t container_image_score[KG_MAX_CONTAINERS];
  /* (ABI 11) with KG_POD_TAINT_TABLE: the number of taints of the caller's taint table tolerated_taints was compiled
   * against (taint ids < taint_count are decided).  kg_pods_schedule* refuses a staged queue holding a pod compiled
   * against fewer taints than some valid node row carries (KG_E_INVALID: re-stage the pods). */
  int64_t taint_count;
  /* (ABI 12) PodTopologySpread / InterPodAffinity, topologyKey kubernetes.io/hostname only, over the caller's table of
   * match groups (≤ KG_MAX_MATCH_GROUPS).  A group is a label selector with its namespace set (a spread constraint's
   * selector in the pod's namespace; an affinity term's selector and namespaces), or the conjunction of a pod's
   * required pod-affinity terms.  Group ids below are 1 + index, 0 = none.  The same fields describe the pod both when
   * it is scheduled and when it sits on a node (kg_pods_add, or placed by the engine): the engine keeps per node the
   * number of pods matching each group, of required anti-affinity terms of each group, and the symmetric weights. */
  int64_t match_groups;                        /* bit k: the pod (labels, namespace) matches group k             */
  /* topology spread constraints in the pod's order (≤ KG_MAX_SPREAD; at most one per {key, whenUnsatisfiable}, as
   * the API validates): the selector's group, maxSkew and KG_SPREAD_* flags.  A pod without constraints passes the
   * system defaults here (hostname maxSkew 3 + zone maxSkew 5, ScheduleAnyway, with its owners' selector), each flagged
   * KG_SPREAD_SYSTEM_DEFAULT (ABI 13; before, such nodes were treated as if requireAllTopologies held). */
  int64_t n_spread;
  int64_t spread_group[KG_MAX_SPREAD];
  int64_t spread_max_skew[KG_MAX_SPREAD];
  int64_t spread_flags[KG_MAX_SPREAD];
  int64_t pod_affinity_group;                  /* the conjunction of its required pod-affinity terms (0 = none)  */
  int64_t pod_affinity_terms;                  /* bit k: a required pod-affinity term of group k (symmetric      */
                                               /* score of later pods: HardPodAffinityWeight)                    */
  int64_t pod_anti_affinity;                   /* bit k: a required pod-anti-affinity term of group k            */
  int64_t n_pod_preferred;                     /* preferred pod (anti-)affinity terms (≤ KG_MAX_POD_PREFERRED)   */
  int64_t pod_preferred_group[KG_MAX_POD_PREFERRED];
  int64_t pod_preferred_weight[KG_MAX_POD_PREFERRED];  /* + affinity weight, − anti-affinity weight           */
  /* InterPodAffinity terms with topologyKey topology.kubernetes.io/zone (the fields above are kubernetes.io/hostname
   * terms): required affinity terms (bit k: a term of group k; the conjunction stays pod_affinity_group), required
   * anti-affinity terms, and bit t: preferred term t is zone-keyed */
  int64_t pod_affinity_terms_zone;
  int64_t pod_anti_affinity_zone;
  int64_t pod_preferred_zone;
  /* (ABI 12) the required reservation affinity of a KG_POD_RSV_AFFINITY pod (GetRequiredReservationAffinity,
   * pkg/util/reservation/reservation.go:444-489), over the caller's predicate table evaluated on each slot's labels
   * (kg_node_reservations.predicates): matchReservation (reservation/transformer.go:348-372) also needs every
   * predicate of reservation_selector (ReservationSelector) and, when n_reservation_terms > 0, one of the
   * ReservationSelectorTerms (each: every listed predicate; 0 = an empty term, matching nothing).  All zero: the
   * owner groups alone decide, as before. */
  uint64_t reservation_selector;
  int64_t n_reservation_terms;
  uint64_t reservation_terms[KG_MAX_AFF_TERMS];
  /* (ABI 12) scheduling a Reservation: a staged pod with KG_POD_RESERVE is the reservation's reserve pod
   * (reservationutil.IsReservePod): it matches no reservation (transformer.go:112), and Reservation.Filter
   * (reservation/plugin.go:324-350) pins it to the reservation's node and rejects nodes holding an available
   * reservation whose allocate policy conflicts with its own (Default never coexists with another policy); a
   * KG_POD_RSV_OPERATING pod (IsReservationOperatingMode) takes that conflict check with the Aligned policy.
   * Its Reservation Score is MinNodeScore (scoring.go:104-106). */
  int64_t reserve_allocate_policy;             /* the reservation's Spec.AllocatePolicy: KG_RSV_POLICY_*          */
  int64_t reserve_node;                        /* 1 + index of GetReservePodNodeName's node; 0 = not pinned       */
} kg_pod;

/* pod reservation flags */
enum {
  KG_POD_RSV_AFFINITY = 1 << 0,  /* GetRequiredReservationAffinity != nil: must allocate from a reservation */
  KG_POD_RSV_OPERATING = 1 << 1  /* (ABI 12) apiext.IsReservationOperatingMode: Filter's allocate-policy check */
};

/* Reservation slots of one node as reservationCache holds them (frameworkext/reservation_info.go:79-99,
 * reservation/cache.go:56-61).  The reserve pods stay in NodeInfo (kg_pods_add: requests = allocatable, non-zero
 * requests = schedutil.GetNonzeroRequests of them, i.e. 100m / 200MiB for an absent key), as the reference's
 * scheduler cache keeps them.  Owners: reservations with the same owner spec (ObjectRef / Controller /
 * LabelSelector list) share an owner group 0..63; a pod carries the bitmask of the groups it matches.  An allocatable
 * of 0 = the resource is absent from ReservationInfo.Allocatable (cpu-only / memory-only reservations).  Policies:
 * reservation allocate policy (Default / Aligned / Restricted). */
#define KG_MAX_OWNER_GROUPS 64
#define KG_MAX_RSV_SLOTS 4
enum { KG_RSV_POLICY_DEFAULT = 0, KG_RSV_POLICY_ALIGNED = 1, KG_RSV_POLICY_RESTRICTED = 2 };
typedef struct kg_node_reservations {
  int64_t n;                                   /* slots in use (0..KG_MAX_RSV_SLOTS), by reservation index    */
  int64_t owner[KG_MAX_RSV_SLOTS];             /* owner group 0..63 (bit of kg_pod.reservation_owner_mask)    */
  int64_t allocatable_cpu[KG_MAX_RSV_SLOTS];   /* ReservationInfo.Allocatable (milli / bytes; 0 = absent)     */
  int64_t allocatable_mem[KG_MAX_RSV_SLOTS];
  int64_t allocated_cpu[KG_MAX_RSV_SLOTS];     /* ReservationInfo.Allocated (Σ assigned pods' requests)       */
  int64_t allocated_mem[KG_MAX_RSV_SLOTS];
  int64_t assigned[KG_MAX_RSV_SLOTS];          /* len(AssignedPods)                                            */
  int64_t order[KG_MAX_RSV_SLOTS];             /* LabelReservationOrder value (0 = absent; < 2^31)             */
  int64_t policy[KG_MAX_RSV_SLOTS];            /* KG_RSV_POLICY_*                                             */
  int64_t allocate_once[KG_MAX_RSV_SLOTS];     /* IsAllocateOnce                                               */
  int64_t available[KG_MAX_RSV_SLOTS];         /* IsAvailable && ParseError == nil                             */
  int64_t unschedulable[KG_MAX_RSV_SLOTS];     /* IsUnschedulable                                              */
  uint64_t predicates[KG_MAX_RSV_SLOTS];       /* (ABI 12) the caller's predicate bits over the node's labels  */
                                               /* overlaid with the reservation's (matchReservation's fakeNode, */
                                               /* transformer.go:357-369); read for reservation-affinity pods    */
  int64_t predicate_count;                     /* predicate ids decided in `predicates` (as node rows, ABI 11): */
                                               /* a queue using a later id is refused until the slots are re-sent */
  /* (ABI 13) DeviceShare: the GPUs each reservation holds.  gpu_alloc = nodeDevice.getUsed(reserve pod), the
   * reservation's allocatable per minor; gpu_allocated = the allocations of its assigned pods on those minors
   * (appendAllocatedByHints, deviceshare/reservation.go:133-160).  [slot][minor][0..2] = gpu-core, gpu-memory (bytes),
   * gpu-memory-ratio.  gpu_minors[s] = 0: the reservation holds no GPU (RestoreReservation drops it).  Both are in
   * kg_node_device.used already (the reserve pod and the assigned pods are bound pods of the node); Reserve / Unreserve
   * keep gpu_allocated current. */
  int64_t gpu_minors[KG_MAX_RSV_SLOTS];        /* bit m: minor m is in the reserve pod's allocation             */
  int64_t gpu_alloc[KG_MAX_RSV_SLOTS][KG_MAX_MINORS][3];
  int64_t gpu_allocated[KG_MAX_RSV_SLOTS][KG_MAX_MINORS][3];
  /* (ABI 15) NodeNUMAResource: the cpuset each reservation holds.  cpus = resourceManager.GetAllocatedCPUSet(node,
   * reservation UID), the reserve pod's allocation; cpus_assigned = the union of GetAllocatedCPUSet(node, pod.UID) over
   * the reservation's AssignedPods.  RestoreReservation (nodenumaresource/reservation.go:76-113) gives a pod matching
   * the reservation reservedCPUs = cpus − cpus_assigned, which getResourceOptions (plugin.go:482-505, 513-535) offers
   * to the pod nominated into it as preferredCPUs / reusable NUMA cpu at Score and Reserve.  Both sets are in
   * kg_node_numa.allocated_cpus already (the resource manager's allocatedCPUs); a cpu of cpus ∩ cpus_assigned has
   * RefCount 2 there (node_allocation.go:76-103).  Reserve / Unreserve keep cpus_assigned current.  All zero: the
   * reservation holds no cpuset. */
  uint64_t cpus[KG_MAX_RSV_SLOTS][KG_MAX_CPUS / 64];
  uint64_t cpus_assigned[KG_MAX_RSV_SLOTS][KG_MAX_CPUS / 64];
} kg_node_reservations;

/* One ElasticQuota as the plugin's PreFilter snapshot sees it (plugin.go:211-256) over KG_QUOTA_RES resources: cpu
 * (milli), memory (bytes), then the device resources of kg_pod.device_requests[0..5] (nvidia.com/gpu, dcu.com/gpu,
 * koordinator.sh/gpu, gpu-core, gpu-memory, gpu-memory-ratio) — the pod's quota request is PodRequestsAndLimits
 * over all of them.  used_limit = runtime when EnableRuntimeQuota else max (getQuotaInfoUsedLimit).  Runtime is
 * refreshed from the quota tree's requests, which Reserve does not change, so it is fixed for a batch.  A limit /
 * min of -1 = the resource is absent from that ResourceList: quotav1.LessThanOrEqual only compares keys of its
 * second argument, so an absent key does not constrain. */
#define KG_QUOTA_RES 8
typedef struct kg_quota {
  int64_t used[KG_QUOTA_RES];
  int64_t non_preemptible_used[KG_QUOTA_RES];
  int64_t used_limit[KG_QUOTA_RES];
  int64_t min[KG_QUOTA_RES];
} kg_quota;

/* DeviceShare view of one node's GPUs: the Device object's GPU entries (deviceshare/device_cache.go:505-523:
 * an unhealthy device has empty resources) + nodeDevice.deviceUsed from the pods already bound there.
 * has_device = 0: no Device object for the node (the plugin passes such nodes; NodeResourcesFit on the
 * device extended resources, whose allocatable is then 0, rejects device pods). */
/* (ABI 17) the device types of the default handler (deviceshare/devicehandler_default.go): RDMA, FPGA */
#define KG_DEV_XTYPES 2
enum { KG_XTYPE_RDMA = 0, KG_XTYPE_FPGA = 1 };
typedef struct kg_node_device {
  int64_t has_device;
  int64_t present[KG_MAX_MINORS];              /* a GPU DeviceInfo with this minor exists             */
  int64_t healthy[KG_MAX_MINORS];
  int64_t total_core[KG_MAX_MINORS], total_memory[KG_MAX_MINORS], total_ratio[KG_MAX_MINORS];
  int64_t used_core[KG_MAX_MINORS], used_memory[KG_MAX_MINORS], used_ratio[KG_MAX_MINORS];
  /* (ABI 17) RDMA / FPGA DeviceInfos (type KG_XTYPE_*): listed minors, health, the type's one resource
   * (koordinator.sh/rdma, koordinator.sh/fpga: percentage per device) and its deviceUsed */
  int64_t x_present[KG_DEV_XTYPES][KG_MAX_MINORS];
  int64_t x_healthy[KG_DEV_XTYPES][KG_MAX_MINORS];
  int64_t x_total[KG_DEV_XTYPES][KG_MAX_MINORS];
  int64_t x_used[KG_DEV_XTYPES][KG_MAX_MINORS];
} kg_node_device;

/* NodeNUMAResource view of one node: TopologyOptions (topology_options.go:40-48, from the
 * NodeResourceTopology) + the NodeAllocation built from already-bound pods (node_allocation.go:32-38).
 * The CPU topology is described in buildCPUTopology numbering (socket-major, then NUMA node, core, thread:
 * cpu = ((socket·nodes_per_socket + node)·cores_per_node + core)·cpus_per_core + thread) with ≤ 256 CPUs and
 * ≤ 4 NUMA nodes; NUMA zone i of the NRT is NUMA node i. */
typedef struct kg_node_numa {
  int64_t has_topology;                        /* CPUTopology reported                                */
  int64_t sockets, nodes_per_socket, cores_per_node, cpus_per_core;
  int64_t numa_policy;                         /* KG_NUMA_POLICY_* (label over NRT policy, util.go:51-57) */
  int64_t node_cpu_bind_policy;                /* KG_NODE_BIND_* (extension.GetNodeCPUBindPolicy)      */
  int64_t numa_allocate_strategy;              /* node label KG_STRATEGY_*, -1 = plugin default       */
  int64_t num_numa;                            /* NUMANodeResources zones (0 = none)                  */
  int64_t numa_cpu[KG_MAX_NUMA];               /* zone allocatable cpu (milli)                        */
  int64_t numa_mem[KG_MAX_NUMA];               /* zone allocatable memory (bytes)                     */
  uint64_t reserved_cpus[KG_MAX_CPUS / 64];    /* TopologyOptions.ReservedCPUs                        */
  uint64_t allocated_cpus[KG_MAX_CPUS / 64];   /* NodeAllocation.allocatedCPUs (maxRefCount 1)        */
  int64_t numa_alloc_cpu[KG_MAX_NUMA];         /* NodeAllocation.allocatedResources: cpu (milli)      */
  int64_t numa_alloc_mem[KG_MAX_NUMA];         /*                                   memory (bytes)    */
  /* node.koordinator.sh/resource-amplification-ratio cpu (extension.Ratio, ≤ 1 = none).  numa_cpu above is the
   * zone cpu AFTER amplifyNUMANodeResources (util.go:63-84), node allocatable cpu the amplified one. */
  double cpu_amplification_ratio;
  /* (ABI 9) NodeAllocation.allocatedCPUs whose CPUInfo.ExclusivePolicy is PCPULevel / NUMANodeLevel (the policy of
   * the pod holding them; subsets of allocated_cpus) */
  uint64_t exclusive_pcpu_cpus[KG_MAX_CPUS / 64];
  uint64_t exclusive_numa_cpus[KG_MAX_CPUS / 64];
} kg_node_numa;

/* Node-side view for TaintToleration / NodeAffinity (ABI 8).  The caller keeps two dense tables: up to 64 distinct
 * taints (key, value, effect) and up to 64 distinct node-selector predicates (a NodeSelectorRequirement — key, operator,
 * values — or a MatchFields requirement, or one nodeSelector key=value pair), and evaluates them on each node's
 * labels / name when the node or the tables change (label matching is string work; the device combines the bits). */
typedef struct kg_node_predicates {
  uint64_t predicates;                         /* bit k: predicate k holds on the node                          */
  uint64_t taints_hard;                        /* the node's taints with effect NoSchedule or NoExecute         */
  uint64_t taints_soft;                        /* the node's taints with effect PreferNoSchedule                */
  uint64_t images;                             /* (ABI 10) bit i: NodeInfo.ImageStates holds image i of the     */
                                               /* caller's image table (the ≤ 64 images queued pods reference) */
  /* (ABI 11) the sizes of the caller's predicate and image tables this row was compiled against: predicate ids <
   * predicate_count and image ids < image_count are decided.  kg_pods_schedule* refuses a staged queue that
   * references a predicate or image id some valid node row was not compiled for (KG_E_INVALID: re-send the rows). */
  int64_t predicate_count;
  int64_t image_count;
  /* (ABI 12) the node's topology.kubernetes.io/zone domain: 1 + the zone's index in the caller's zone table
   * (< KG_MAX_ZONES), 0 = the node has no zone label (PodTopologySpread zone constraints) */
  int64_t zone;
} kg_node_predicates;

typedef struct kg_stats {
  int64_t pods_scheduled;                      /* pods with a node                                    */
  int64_t pods_unschedulable;
  int64_t device_batches;                      /* eval+resolve rounds issued                          */
  int64_t node_evaluations;                    /* Σ pods × nodes evaluated                            */
  double seconds;                              /* wall time inside kg_pods_schedule                   */
  double reserved[3];
} kg_stats;

typedef struct kg_engine kg_engine;

/* Defaults: v1beta2.SetDefaults_LoadAwareSchedulingArgs (v1beta2/defaults.go:76-99), NodeResourcesFit
 * LeastAllocated cpu:1 memory:1, Fit and LoadAware enabled with weight 1. */
void kg_config_default(kg_config* cfg);

/* n_ranks>1: the engine shards node evaluation over ranks (one process per GPU) and exchanges candidates with
 * RCCL; `nccl_unique_id` is the 128-byte ncclUniqueId created on rank 0 and broadcast by the caller. */
/* ncclGetUniqueId (128 bytes) — call on rank 0, broadcast to the other ranks out of band. */
int kg_nccl_unique_id(void* out128);
int kg_engine_create(const kg_config* cfg, int64_t capacity_nodes, int rank, int n_ranks,
                     const void* nccl_unique_id, kg_engine** out);
void kg_engine_destroy(kg_engine* e);

/* Test hook (not a product path): n_ranks engines in ONE process, usually on one device, exchanging their
 * per-round candidate records (and DeviceShare's per-round maxima) by device copies ordered with HIP events
 * instead of RCCL, which runs one rank per device.  Every other step — the sharded wide pass, the rank-record
 * merge (merge_round over n_ranks records), the replicated resolver — is the multi-rank engine itself.  Each
 * rank's engine must be driven from its own host thread with the same calls in the same order (a host barrier
 * pairs the ranks' exchanges; it fails with KG_E_COLLECTIVE after 60 s without a peer). */
typedef struct kg_loopback kg_loopback;
int kg_loopback_create(int n_ranks, kg_loopback** out);
void kg_loopback_destroy(kg_loopback* lb);
int kg_engine_create_loopback(const kg_config* cfg, int64_t capacity_nodes, int rank, int n_ranks, kg_loopback* lb,
                              kg_engine** out);

/* Host-collective rank (test hook / RCCL-less deployments): a multi-rank engine whose per-round exchanges go through
 * the caller's all-gather instead of RCCL — e.g. torch.distributed gloo across processes.  `exchange` receives this
 * rank's `bytes` (host memory, already copied back from the device) and must fill `recv` with every rank's part in
 * rank order ([n_ranks][bytes]); it returns 0 on success.  The engine synchronises the round's stream around each
 * exchange, so this path is slow; every other step is the multi-rank engine itself.  Every rank must make the same
 * engine calls in the same order, as with RCCL. */
typedef int (*kg_exchange_fn)(void* user, const void* send, void* recv, int64_t bytes);
int kg_engine_create_hosted(const kg_config* cfg, int64_t capacity_nodes, int rank, int n_ranks,
                            kg_exchange_fn exchange, void* user, kg_engine** out);

int kg_nodes_upsert(kg_engine* e, const kg_node* nodes, const int32_t* idx, int64_t n);
int kg_nodes_delete(kg_engine* e, const int32_t* idx, int64_t n);
int kg_node_metrics_update(kg_engine* e, const kg_node_metric* m, const int32_t* idx, int64_t n, int64_t now_unix_nano);
/* NodeMetric.Status.PodsMetric of one node (replaces the node's list; informer delta, like kg_node_metrics_update).
 * LoadAware Score then follows estimatedAssignedPodUsed / sumPodUsages (load_aware.go:283-376): an assigned pod whose
 * usage is reported and who was assigned before the metric's update time (and not within the report interval) counts
 * through NodeUsage; the others are estimated as max(EstimatePod, reported usage), and their reported usage is taken
 * out of NodeUsage (or, for a prod pod under ScoreAccordingProdUsage, the prod pods' reported usages replace it). */
int kg_node_pods_metric_set(kg_engine* e, int32_t node_idx, const kg_pod_metric* m, int64_t n);

int kg_pods_add(kg_engine* e, const kg_pod* pods, const int32_t* node_idx, int64_t n);
int kg_pods_remove(kg_engine* e, const kg_pod* pods, const int32_t* node_idx, int64_t n);
/* The framework's Unreserve (RunReservePluginsUnreserve after a failed Permit / PreBind / Bind) of staged pods
 * [first, first+count) that kg_pods_schedule_staged placed, `mask` (nullable, count bytes) selecting them: every
 * enabled plugin releases what its Reserve took — NodeInfo.RemovePod + the LoadAware assign cache
 * (loadaware/pod_assign_cache.go:119-131), the NodeNUMAResource cpuset and NUMA resources
 * (nodenumaresource/plugin.go:417-425), the DeviceShare GPU minors (deviceshare/plugin.go:440-455), the
 * reservation assume (reservation/plugin.go:561-583) and the ElasticQuota charge (elasticquota/plugin.go:348-360).
 * The pods' decisions are cleared (fetch → -1); a pod is released at most once. */
int kg_pods_unreserve(kg_engine* e, int64_t first, int64_t count, const uint8_t* mask);
/* The scheduler clock isNodeMetricExpired reads (loadaware/helper.go:36-41, time.Since on every Filter/Score):
 * now_unix_nano > 0 fixes it; 0 = the host's real-time clock, read at every schedule / evaluate call; < 0 (the
 * default) = the newest now passed to kg_node_metrics_update.  Nodes whose metric expires or revives between calls
 * are re-flagged before the next call evaluates them. */
int kg_engine_set_clock(kg_engine* e, int64_t now_unix_nano);

/* Schedules `n` pods in FIFO order. out_node_idx[i] = chosen node (-1 = unschedulable), out_score[i] = the
 * weighted total score of that node. Each placement is assumed before the next pod is evaluated. */
int kg_pods_schedule(kg_engine* e, const kg_pod* pods, int64_t n, int32_t* out_node_idx, int64_t* out_score,
                     kg_stats* stats);

/* Evaluates one pod on every node slot [0, n_nodes): reject bits (KG_REJECT_*), NodeResourcesFit score and
 * LoadAwareScheduling score (unweighted, as the plugins' Score returns them). Any output may be NULL. */
int kg_pods_evaluate(kg_engine* e, const kg_pod* pod, int32_t* out_reject, int64_t* out_fit_score,
                     int64_t* out_loadaware_score);

/* Split form of kg_pods_schedule for callers that keep the pod queue resident on the device:
 * kg_pods_stage decodes + uploads a queue (replacing any staged queue); kg_pods_schedule_staged schedules
 * queue entries [first, first+count) (device only, blocks until done); kg_results_fetch copies decisions back. */
int kg_pods_stage(kg_engine* e, const kg_pod* pods, int64_t n);
int kg_pods_schedule_staged(kg_engine* e, int64_t first, int64_t count, kg_stats* stats);
int kg_results_fetch(kg_engine* e, int64_t first, int64_t count, int32_t* out_node_idx, int64_t* out_score);

int64_t kg_engine_num_nodes(const kg_engine* e);
/* (ABI 15) The ranks the engine shards node evaluation over (1 = unsharded) and, for a replica, the ranks of the
 * caller's group it replicates (1 otherwise): kg_config.multi_rank_mode resolved at kg_engine_create. */
int kg_engine_ranks(const kg_engine* e, int64_t* shard_ranks, int64_t* replica_ranks);
/* Reads the DEVICE copy of the mutable node state: NodeInfo.Requested{cpu,mem}, NonZeroRequested{cpu,mem},
 * pod count and the LoadAware estimated usage Σ EstimatePod over the assign cache (all pods / prod pods).
 * Any output may be NULL. */
int kg_nodes_read_state(kg_engine* e, int64_t* requested_cpu, int64_t* requested_mem, int64_t* nonzero_cpu,
                        int64_t* nonzero_mem, int64_t* num_pods, int64_t* la_est_cpu, int64_t* la_est_mem,
                        int64_t* la_est_prod_cpu, int64_t* la_est_prod_mem);

/* NodeNUMAResource (engines whose profile enables it): the TopologyOptions + NodeAllocation of nodes idx[0..n)
 * (replaces each node's NUMA state; node_allocation.go:32-38, topology_options.go:40-48 — fed by the NRT and
 * pod informers, topology_eventhandler.go:62-113 / pod_eventhandler.go:94-136). */
int kg_nodes_numa_upsert(kg_engine* e, const kg_node_numa* numa, const int32_t* idx, int64_t n);
/* Reads the DEVICE NodeAllocation: allocated cpus (4 words per node), per-NUMA allocated cpu / memory
 * (KG_MAX_NUMA per node). Any output may be NULL. */
int kg_nodes_read_numa(kg_engine* e, uint64_t* allocated_cpus, int64_t* numa_alloc_cpu, int64_t* numa_alloc_mem);
/* The cpuset NodeNUMAResource Reserve allocated to staged pods [first, first+count): 4 uint64 words per pod,
 * empty for pods without a cpuset (the resource-status annotation PreBind writes, plugin.go:427-463). */
int kg_results_fetch_cpusets(kg_engine* e, int64_t first, int64_t count, uint64_t* out_cpusets);
/* NodeNUMAResource Filter + Score of one pod on every node slot, the plugin alone: out_pass 1/0, the plugin's
 * unweighted score (0 where Filter rejects) and the affinity the topology manager stores (NUMA mask, -1 = nil).
 * Filter runs only when the profile enables the plugin at Filter; otherwise Score sees no stored affinity. */
int kg_pods_evaluate_numa(kg_engine* e, const kg_pod* pod, int32_t* out_pass, int64_t* out_score,
                          int64_t* out_affinity);

/* DeviceShare (engines whose profile enables it): the GPU devices of nodes idx[0..n) (replaces each node's
 * device state). */
int kg_nodes_device_upsert(kg_engine* e, const kg_node_device* dev, const int32_t* idx, int64_t n);
/* Reads the DEVICE nodeDevice.deviceUsed of every node: KG_MAX_MINORS values per node for each output. */
int kg_nodes_read_device(kg_engine* e, int64_t* used_core, int64_t* used_memory, int64_t* used_ratio);
/* The GPU minors DeviceShare Reserve allocated to staged pods [first, first+count): a bitmask per pod (0 = none);
 * every chosen minor received the pod's per-instance request (CalcDesiredRequestsAndCount). */
int kg_results_fetch_devices(kg_engine* e, int64_t first, int64_t count, int32_t* out_minor_mask);
/* (ABI 17) The RDMA / FPGA minors Reserve allocated to staged pods [first, first+count): out[k·KG_DEV_XTYPES + t] = the
 * bitmask of type t for pod first + k (the default handler's allocation: every chosen minor received the per-instance
 * request, devicehandler_default.go:45-92, device_allocator.go:384-454). */
int kg_results_fetch_devices_x(kg_engine* e, int64_t first, int64_t count, int32_t* out_minor_masks);
/* (ABI 17) Reads the device's RDMA / FPGA deviceUsed: [node][KG_DEV_XTYPES][KG_MAX_MINORS]. */
int kg_nodes_read_device_x(kg_engine* e, int64_t* x_used);
/* DeviceShare Filter + Score of one pod on every node slot, the plugin alone: out_pass 1/0 and the raw
 * (un-normalized) score, 0 where Filter rejects. */
int kg_pods_evaluate_device(kg_engine* e, const kg_pod* pod, int32_t* out_pass, int64_t* out_score);

/* Reservation (engines whose profile enables it): the reservation slots of nodes idx[0..n) (replaces each node's
 * slots; fed by the reservation informer, eventhandlers/reservation_handler.go).  The Reservation profile runs
 * one FIFO pod per device pass (BeforePreFilter restore + Filter + PreScore/nominate + Score + NormalizeScore). */
int kg_nodes_reservation_upsert(kg_engine* e, const kg_node_reservations* r, const int32_t* idx, int64_t n);
/* TaintToleration / NodeAffinity node view of nodes idx[0..n) (replaces each node's predicates and taints; fed by the
 * node informer after the caller re-evaluates its predicate / taint tables on the node's labels and taints). */
int kg_nodes_predicates_upsert(kg_engine* e, const kg_node_predicates* p, const int32_t* idx, int64_t n);
/* Reads the DEVICE reservation slots: allocated cpu / memory and assigned count, KG_MAX_RSV_SLOTS per node. */
int kg_nodes_read_reservations(kg_engine* e, int64_t* allocated_cpu, int64_t* allocated_mem, int64_t* assigned);
/* (ABI 13) Reads the DEVICE reservation slots' gpu_allocated, [n_nodes][KG_MAX_RSV_SLOTS][KG_MAX_MINORS][3] (zeros
 * for slots holding no GPU, or when DeviceShare is off; a re-upserted node's slots that no longer hold GPUs read zero).
 * KG_E_INVALID when the profile does not enable Reservation. */
int kg_nodes_read_reservation_gpus(kg_engine* e, int64_t* gpu_allocated);
/* (ABI 15) Reads the DEVICE reservation slots' cpus_assigned, [n_nodes][KG_MAX_RSV_SLOTS][KG_MAX_CPUS / 64] (zeros for
 * slots holding no cpuset, or when NodeNUMAResource is off); KG_E_INVALID when the profile does not enable Reservation.
 * Replaces the reference's read of reservationRestoreStateData through resourceManager.GetAllocatedCPUSet
 * (nodenumaresource/reservation.go:84-101). */
int kg_nodes_read_reservation_cpus(kg_engine* e, uint64_t* cpus_assigned);
/* The reservation slot Reserve assumed each staged pod [first, first+count) into (-1 = none). */
int kg_results_fetch_reservations(kg_engine* e, int64_t first, int64_t count, int32_t* out_slot);

/* The exact pass's evaluation of one pod on every node slot (profiles with Reservation, or NodeNUMAResource together
 * with DeviceShare): BeforePreFilter restore (reservation/transformer.go:49-346), every enabled Filter on the restored
 * NodeInfo, the nomination (nominator.go:76-134) and the raw Scores, exactly as kg_pods_schedule evaluates the pod —
 * what frameworkext's --debug-scores prints for it (frameworkext/debug.go:61-108).  KG_RSV_EVAL_WORDS int64 per node:
 * [0] pass, [1] nominated slot (-1 none), [2] raw Reservation score of it, [3] a nodeReservationState exists (the node
 * was restored), [4] the matched slots (bit s), [5..9] the restored NodeInfo Requested cpu / memory, NonZeroRequested
 * cpu / memory, pod count, [10..11] nodeReservationState.podRequested cpu / memory, [12] the weighted total of the
 * non-normalized plugins (Fit, LoadAware, NodeNUMAResource), [13] raw DeviceShare score, [14] the smallest
 * reservation-order label among the matched slots (0 none), [15] reserved. */
#define KG_RSV_EVAL_WORDS 16
int kg_pods_evaluate_reservation(kg_engine* e, const kg_pod* pod, int64_t* out);

/* (ABI 11) The preemption dry run's Filter of one pod on one node (PostFilter → defaultpreemption SelectVictimsOnNode
 * → RunFilterPluginsWithNominatedPods; replaces one Filter round of the Go dry run): the pod's Filters on node
 * node_idx of a NodeInfo copy with the n_victims pods `victims` removed (NodeInfo.RemovePod) and the Reservation
 * plugin's PreFilterExtensions.RemovePod applied (reservation/plugin.go:284-310: a victim's requests add to
 * state.preemptible[node], or to state.preemptibleInRRs[node][its reservation] when victim_slot[k] >= 0 names the
 * node's reservation slot it was allocated from; NULL = none).  The Reservation Filter then fits the pod against them
 * (plugin.go:357-428, fitsNode :433-482).  out_reject: 0 = every enabled Filter passes, else KG_REJECT_* bits.
 * Profiles with NodeResourcesFit / LoadAwareScheduling / Reservation; (ABI 14) pods and victims with ephemeral-storage
 * / scalar requests are accepted.  (ABI 16) The other accelerated Filters run in the dry run too:
 *   - NodeNUMAResource: no PreFilterExtensions (nodenumaresource/plugin.go:272-274), so the victims' cpusets stay
 *     allocated in the node's NodeAllocation; its Filter reads the victim-free NodeInfo.Requested (filterAmplifiedCPUs);
 *   - DeviceShare: AddPod / RemovePod (deviceshare/plugin.go:163-278) move a victim's device allocation (victim_minors[k]
 *     = the minors it holds on the node — GPU bits 0-7, (ABI 17) RDMA bits 8-15, FPGA bits 16-23 —, its per-instance
 *     share = its device request as Reserve allocated it; NULL or 0 = none) into state.preemptibleDevices[node] unless
 *     it is a reserve pod or was allocated from a reservation
 *     (victim_slot[k] >= 0); Filter allocates against free = total − max(0, used − preemptible)
 *     (calcFreeWithPreemptible, device_cache.go:314-342).  Engines whose reservations hold GPUs are refused;
 *   - TaintToleration / NodeAffinity: node-static (KG_REJECT_TAINT / KG_REJECT_NODE_AFFINITY).
 * PodTopologySpread / InterPodAffinity profiles are refused (KG_E_UNSUPPORTED). */
int kg_pods_filter_preemption(kg_engine* e, const kg_pod* pod, int32_t node_idx, const kg_pod* victims,
                              const int32_t* victim_slot, const int32_t* victim_minors, int64_t n_victims,
                              int32_t* out_reject);

/* (ABI 14) The preemption dry run over many candidate nodes in ONE launch: SelectVictimsOnNode for every candidate
 * (DryRunPreemption's per-node step: koordinator's elasticquota/preempt.go:111-215 and the k8s defaultpreemption
 * plugin run the same loop), one device thread per candidate c = node node_idx[c]:
 *   - its potential victims are victims[victim_offsets[c] .. victim_offsets[c + 1]) in the caller's reprieve order —
 *     the caller's canPreempt selection (priority, quota), util.MoreImportantPod sort and filterPodsWithPDBViolation
 *     split: PDB-violating victims first (pdb_violating[k] = 1; NULL = none), each group most important first;
 *     victim_slot[k] and victim_minors[k] as for kg_pods_filter_preemption (NULL = none);
 *   - the device removes them all (NodeInfo.RemovePod + the Reservation plugin's RemovePod) and runs the Filters:
 *     out_reject[c] = 0 or KG_REJECT_* bits (KG_REJECT_NO_VICTIMS for a candidate without potential victims);
 *   - when they pass, it reprieves each victim in order: adds it back (AddPodInfo + AddPod), re-runs the Filters and
 *     removes it again when the pod no longer fits: out_victim[k] = 1 for a victim kept, 0 for one reprieved (and for
 *     every entry of a candidate whose Filters failed); out_violating[c] = numViolatingVictim.
 * Nominated pods are not added (the engine holds no nominator).  Same profiles and refusals as
 * kg_pods_filter_preemption; ephemeral-storage and scalar requests are carried in NodeResourcesFit and in fitsNode's
 * EphemeralStorage / ScalarResources terms (reservation/plugin.go:471-479) by both entry points since ABI 14. */
int kg_pods_select_victims(kg_engine* e, const kg_pod* pod, int64_t n_candidates, const int32_t* node_idx,
                           const int64_t* victim_offsets, const kg_pod* victims, const int32_t* victim_slot,
                           const int32_t* victim_minors, const uint8_t* pdb_violating, int32_t* out_reject,
                           uint8_t* out_victim, int32_t* out_violating);

/* (ABI 12) PodTopologySpread / InterPodAffinity state (engines whose profile enables either): per node and match
 * group k, [n][k] layout of KG_MAX_MATCH_GROUPS int32 each — pods matching group k (countPodsMatchSelector),
 * required anti-affinity terms of group k held by the node's pods (existingAntiAffinityCounts), and the symmetric
 * score weight of the node's pods' terms of group k (processExistingPod: preferred ± weight, required affinity ×
 * HardPodAffinityWeight); anti_zone / sym_zone: the same for the node's pods' zone-keyed terms (NULL = skip).
 * Maintained from kg_pods_add / kg_pods_remove, Reserve and Unreserve. */
int kg_nodes_read_pod_groups(kg_engine* e, int32_t* match_count, int32_t* anti_count, int32_t* sym_weight,
                             int32_t* anti_zone, int32_t* sym_zone);

/* ElasticQuota admission (engines whose pods carry quota_id): replaces the quota table (n ≤ KG_MAX_QUOTAS).
 * Every scheduled pod runs PreFilter's check (used + request ≤ used_limit over the pod's cpu/memory requests; for
 * non-preemptible pods also non_preemptible_used + request ≤ min) before its node search, and a placed pod is
 * charged (ReservePod → updatePodUsedNoLock, core/group_quota_manager.go:613-648,791-797). */
int kg_quotas_set(kg_engine* e, const kg_quota* quotas, int64_t n);
/* Reads the DEVICE quota table back (used / non_preemptible_used after the batches so far). */
int kg_quotas_read(kg_engine* e, kg_quota* out, int64_t n);

/* Live kernel timing of the real (pipelined) round runners: with profiling on, every launch of kind k
 * (KG_PROF_*) is bracketed by HIP events on its own stream; kg_profile_read returns the summed event time (ms)
 * and the launch count per kind since kg_profile_enable.  Adds two event records per launch: not for the timed
 * region of a benchmark. */
enum {
  KG_PROF_EVAL = 0, KG_PROF_MERGE = 1, KG_PROF_RESOLVE = 2, KG_PROF_DS_MAX = 3, KG_PROF_DS_NORM = 4,
  KG_PROF_RSV_EVAL = 5, KG_PROF_RSV_SELECT = 6, KG_PROF_RSV_APPLY = 7, KG_PROF_KINDS = 16
};
int kg_profile_enable(kg_engine* e, int on);
int kg_profile_read(kg_engine* e, double* ms_total, int64_t* launches);

/* Measurement hooks (bench.py): replays one device round's kernel `which` (0 = eval, 1 = merge, 2 = resolve) `iters` times
 * on the engine stream between HIP events, restoring state, and returns the mean duration in ms plus the
 * algorithmic bytes that kernel must move per launch. Requires a staged queue. */
int kg_bench_kernel(kg_engine* e, int which, int iters, double* avg_ms, double* algo_bytes);
/* Debug: leastRequestedScore on the device for n (requested, capacity) pairs (exactness test of the
 * division-free path). */
int kg_debug_least_requested(kg_engine* e, const int64_t* requested, const int64_t* capacity, int64_t* out,
                             int64_t n);
/* Debug: the wide pass's division-free leastRequestedScore on n (requested, capacity) pairs — the 32-bit
 * cpu-term routine into out_cpu and the f64 memory-term routine into out_mem (-1 where a pair lies outside
 * that routine's exact domain; the engine sends such rows to the exact path). */
int kg_debug_fast_lrs(kg_engine* e, const int64_t* requested, const int64_t* capacity, int64_t* out_cpu,
                      int64_t* out_mem, int64_t n);

/* Debug: the device topology-manager policy merge — Policy.Merge + canAdmitPodResult over ≤ 2 filtered provider lists
 * (frameworkext/topologymanager/policy.go:127-185 mergeFilteredHints, policy_best_effort.go:43-48,
 * policy_restricted.go:41-46, policy_single_numa_node.go:38-77) — exactly the code NodeNUMAResource Filter runs, on n
 * caller-given cases of KG_DBG_MERGE_WORDS int64: policy (KG_NUMA_POLICY_*), NUMA node count (1..4), list count
 * (1..2), then per list {hint positions, preferred positions, nil, nil preferred, empty} (positions index the
 * IterateBitMasks order 1,2,4,8,3,5,9,6,10,12,7,11,13,14,15), then the hint score of each mask 0..15.
 * out: 8 int64 per case = admit, nil, mask, preferred, score. */
#define KG_DBG_MERGE_WORDS 32
int kg_debug_numa_merge(kg_engine* e, const int64_t* cases, int64_t n, int64_t* out);

/* Debug: evaluates every staged pod on every node with both device evaluation paths (the reference-shaped
 * one used for modified rows and per-plugin output, and the hoisted-term one of the wide pass) and returns
 * the number of (pod, node) pairs where feasibility or total score differ (must be 0). */
int kg_debug_eval_paths(kg_engine* e, int64_t* mismatches);

/* Diagnostic builds (-DKG_STAMPS) only: copies the in-kernel (s_memtime, s_memrealtime) stamps, uint64[4][32][2],
 * then the last resolver launch's per-pod (s_memtime, path bits, sub-phase stamps), uint64[64][6], then the NUMA
 * hint-merge counters (merges, all-permutation fallback passes), uint64[2]: 258 + 384 words in all. */
int kg_debug_stamps(kg_engine* e, uint64_t* out);

/* Debug: the RCCL calls a multi-rank engine makes (ncclGetUniqueId, ncclCommInitRank, ncclCommSplit, ncclAllGather on
 * a HIP stream), on a one-rank communicator of device `device_id`, gathering n uint64 words: 0 when the gathered
 * words equal the sent ones.  A one-GPU box cannot run two RCCL ranks; this checks the library path the driver's
 * multi-GPU run takes. */
int kg_debug_rccl_selftest(int device_id, int64_t n);

const char* kg_last_error(void);
int kg_abi_version(void);
/* sizeof of the ABI structs (0 kg_config, 1 kg_node, 2 kg_node_metric, 3 kg_pod, 4 kg_stats, 5 kg_node_numa,
 * 6 kg_node_device, 7 kg_quota, 8 kg_node_reservations, 9 kg_pod_metric, 10 kg_node_predicates) for
 * binding checks. */
int64_t kg_abi_struct_size(int which);

#ifdef __cplusplus
}
#endif
#endif /* KOORDGPU_H_ */
