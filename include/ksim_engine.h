/*
 * ksim_engine.h — C ABI of the MI355X scheduling-cycle engine (libksim_engine.so).
 *
 * This is the drop-in boundary described in SURVEY.md §8(b).  In the reference
 * (ThomasK33/kube-scheduler-simulator) the per-pod scheduling cycle runs the
 * in-tree plugins through the simulator's wrapper:
 *
 *   factory closure        simulator/scheduler/plugin/plugins.go:75-87
 *     r(configuration, f)  -> original in-tree plugin   (replaced by this engine)
 *     NewWrappedPlugin(..) -> result recording          (kept, unchanged)
 *   wrappedPlugin.PreFilter/Filter/PreScore/Score/NormalizeScore/Reserve
 *                          simulator/scheduler/plugin/wrappedplugin.go:356-516,583-612
 *
 * A cgo package would bind exactly these entry points.
 * All types are plain C: fixed-width integers, pointers and sizes.  No Go
 * pointer is retained after a call returns (cgo rule); every input is copied
 * during the call, every output is written into caller-provided memory.
 *
 * Semantics follow upstream k8s.io/kubernetes v1.26.2 (pinned in
 * simulator/go.mod:53) as restated in SURVEY.md Appendix A and in DESIGN.md.
 */
#ifndef KSIM_ENGINE_H
#define KSIM_ENGINE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KSIM_ABI_VERSION 11

/* ---- limits ------------------------------------------------------------ */
#define KSIM_KEY_NODE_MASK    ((1 << 18) - 1)  /* tie-break key: node field = mask - node (>= 1) */
#define KSIM_MAX_NODES        KSIM_KEY_NODE_MASK
#define KSIM_MAX_NODE_TAINTS  8          /* taints per node, node.Spec.Taints order */
#define KSIM_TAINT_WORDS      4          /* taint vocabulary <= 256 ids (id 0 = none) */
#define KSIM_MAX_SCALAR       8          /* scalar (extended) resource columns */
#define KSIM_MAX_LABEL_COLS   256        /* node label keys with a column (the keys pods reference) */
#define KSIM_EXPR_VALS        6          /* values per node-selector requirement */
#define KSIM_MAX_FILTER       16
#define KSIM_MAX_SCORE        8
#define KSIM_MAX_RES          4          /* resources in a scoring strategy */
#define KSIM_MAX_SHAPE        16         /* RequestedToCapacityRatio shape points */
#define KSIM_MAX_USES         16         /* topology uses per pod (PTS constraints + IPA terms) */
#define KSIM_MAX_CLASSES      4096       /* count classes (see ksim_topo_use) */
#define KSIM_COL_NONE         0xFFFF     /* topology key carried by no node */

/* ---- error codes (SURVEY §8(b) "Errors") -------------------------------- */
#define KSIM_OK            0
#define KSIM_E_INVALID    -1
#define KSIM_E_DEVICE     -2
#define KSIM_E_OOM        -3
#define KSIM_E_RCCL       -4
#define KSIM_E_UNSUPPORTED -5

/* ---- plugin ids.  Names are the upstream in-tree plugin names. ---------- */
enum ksim_plugin {
  KSIM_PL_NODE_UNSCHEDULABLE = 0,   /* NodeUnschedulable */
  KSIM_PL_NODE_NAME,                /* NodeName */
  KSIM_PL_TAINT_TOLERATION,         /* TaintToleration */
  KSIM_PL_NODE_AFFINITY,            /* NodeAffinity */
  KSIM_PL_NODE_PORTS,               /* NodePorts */
  KSIM_PL_NODE_RESOURCES_FIT,       /* NodeResourcesFit */
  KSIM_PL_VOLUME_RESTRICTIONS,      /* VolumeRestrictions */
  KSIM_PL_EBS_LIMITS,               /* EBSLimits */
  KSIM_PL_GCEPD_LIMITS,             /* GCEPDLimits */
  KSIM_PL_NODE_VOLUME_LIMITS,       /* NodeVolumeLimits */
  KSIM_PL_AZURE_DISK_LIMITS,        /* AzureDiskLimits */
  KSIM_PL_VOLUME_BINDING,           /* VolumeBinding */
  KSIM_PL_VOLUME_ZONE,              /* VolumeZone */
  KSIM_PL_POD_TOPOLOGY_SPREAD,      /* PodTopologySpread */
  KSIM_PL_INTER_POD_AFFINITY,       /* InterPodAffinity */
  KSIM_PL_BALANCED_ALLOCATION,      /* NodeResourcesBalancedAllocation */
  KSIM_PL_IMAGE_LOCALITY,           /* ImageLocality */
  KSIM_PL_NETWORK_BANDWIDTH,        /* NetworkBandwidth (the simulator's out-of-tree plugin,
                                       simulator/scheduler/plugin/networkbandwidth/plugin.go) */
  KSIM_PL_COUNT
};

/* taint effects */
#define KSIM_EFFECT_NONE               0
#define KSIM_EFFECT_NO_SCHEDULE        1
#define KSIM_EFFECT_PREFER_NO_SCHEDULE 2
#define KSIM_EFFECT_NO_EXECUTE         3

/* resources usable in scoring strategies (ScoringStrategy.Resources) */
#define KSIM_RES_CPU        0
#define KSIM_RES_MEMORY     1
#define KSIM_RES_EPHEMERAL  2
#define KSIM_RES_SCALAR0    3   /* KSIM_RES_SCALAR0 + k = scalar column k */

/* node flags */
#define KSIM_NODE_UNSCHEDULABLE  1u   /* node.Spec.Unschedulable */
#define KSIM_NODE_NB_LIMIT       2u   /* NetworkBandwidth: the node-limit annotation is present */
#define KSIM_NODE_NB_LIMIT_BAD   4u   /* ... and does not parse as a resource.Quantity */

/* pod flags */
#define KSIM_POD_TOLERATES_UNSCHEDULABLE 1u  /* tolerates node.kubernetes.io/unschedulable:NoSchedule */
#define KSIM_POD_HAS_REQUIRED_AFFINITY   2u  /* spec.affinity.nodeAffinity.required != nil */
#define KSIM_POD_HAS_SCALAR              4u  /* len(request.ScalarResources) > 0 */
#define KSIM_POD_HAS_HOST_PORTS          8u  /* ports not compiled to KSIM_USE_NODE_PORT uses -> KSIM_E_UNSUPPORTED */
#define KSIM_POD_HAS_VOLUMES            16u  /* unsupported by the engine -> KSIM_E_UNSUPPORTED */
/* NodeAffinity's PreFilterResult (nodeaffinity.PreFilter: the union over the
 * required terms of the intersection of each term's metadata.name In
 * matchFields; a term without one means all nodes, i.e. no flag).  The cycle
 * scans only those nodes: nn[nn_first .. nn_first + nn_count) of the pod set,
 * node positions in increasing (nodeTree) order, from nextStartNodeIndex mod
 * nn_count (schedule_one.go findNodesThatFitPod / findNodesThatPassFilters,
 * where upstream visits the set in Go map order).  nn_count == 0: the terms
 * conflict, the pod is unschedulable without any Filter call ("pod affinity
 * terms conflict"); nextStartNodeIndex stays. */
#define KSIM_POD_NODE_NAMES             32u
/* ... and a listed name is not a node of the snapshot: NodeInfos().Get fails
 * and the cycle fails with framework.Error before any Filter call. */
#define KSIM_POD_NODE_NAMES_UNKNOWN     64u
/* NodeAffinityArgs.addedAffinity.requiredDuringSchedulingIgnoredDuringExecution
 * (the profile's scheduler-enforced node selector) applies: terms
 * [added_term_first, +added_term_count) of the pod set, OR-ed.  NodeAffinity's
 * Filter checks them before the pod's own selector and terms and fails with
 * fail_detail KSIM_NA_ENFORCED (nodeaffinity.go errReasonEnforced).  The
 * added PREFERRED terms are scored exactly like the pod's own preferred terms,
 * so the host appends them to pref_term_* instead.  PodTopologySpread's
 * nodeAffinityPolicy reads the pod's own affinity only (GetRequiredNodeAffinity). */
#define KSIM_POD_ADDED_AFFINITY        128u

/* pod nb_flags (NetworkBandwidth request annotations) */
#define KSIM_POD_NB_INGRESS_BAD 1u   /* the ingress request annotation does not parse */
#define KSIM_POD_NB_EGRESS_BAD  2u   /* the egress request annotation does not parse */

/* pod topo_flags */
#define KSIM_POD_IPA_SELF_AFFINITY 1u  /* podMatchesAllAffinityTerms(required affinity terms, pod) */
/* The pod's PodTopologySpread constraints are the system defaults
 * (PodTopologySpreadArgs defaultingType System, the pod has no constraints of
 * its own and a Service / ReplicaSet / ReplicationController / StatefulSet
 * selects it: buildDefaultConstraints with helper.DefaultSelector).  PreScore
 * then runs with requireAllTopologies = false (podtopologyspread.PreScore): no
 * IgnoredNodes, and a node lacking a key registers and counts toward the pair
 * (key, "") -- value id 0 of the use's column -- while Score credits only the
 * keys the node has. */
#define KSIM_POD_PTS_SYSTEM_DEFAULT 2u

/* node-selector requirement operators (k8s NodeSelectorOperator + matchFields) */
#define KSIM_OP_IN            0
#define KSIM_OP_NOT_IN        1
#define KSIM_OP_EXISTS        2
#define KSIM_OP_DOES_NOT_EXIST 3
#define KSIM_OP_GT            4
#define KSIM_OP_LT            5
#define KSIM_OP_FIELD_IN      6  /* matchFields metadata.name In   (vals = node positions) */
#define KSIM_OP_FIELD_NOT_IN  7  /* matchFields metadata.name NotIn */
#define KSIM_OP_FALSE         8  /* requirement that can never match (e.g. unknown value) */
#define KSIM_OP_TRUE          9  /* requirement that always matches (e.g. NotIn of unknown values) */

/* Filter outcome per node (ksim_eval_out.fail_plugin) */
#define KSIM_PASSED        0xFF
#define KSIM_NOT_EVALUATED 0xFE
#define KSIM_FAIL_EXTENDER 0xFD  /* passed the plugins, filtered out by an extender (findNodesThatPassExtenders) */

/* NodeResourcesFit failure reason bits (ksim_eval_out.fail_detail) */
#define KSIM_FIT_TOO_MANY_PODS   1u
#define KSIM_FIT_CPU             2u
#define KSIM_FIT_MEMORY          4u
#define KSIM_FIT_EPHEMERAL       8u
#define KSIM_FIT_SCALAR0        16u   /* << k for scalar column k */

/* PodTopologySpread / InterPodAffinity failure details (ksim_eval_out.fail_detail) */
#define KSIM_PTS_MISSING_LABEL   1u   /* ErrReasonNodeLabelNotMatch (UnschedulableAndUnresolvable) */
#define KSIM_PTS_SKEW            2u   /* ErrReasonConstraintsNotMatch */
#define KSIM_IPA_AFFINITY        1u   /* ErrReasonAffinityRulesNotMatch (UnschedulableAndUnresolvable) */
#define KSIM_IPA_ANTI_AFFINITY   2u   /* ErrReasonAntiAffinityRulesNotMatch */
#define KSIM_IPA_EXISTING_ANTI   3u   /* ErrReasonExistingAntiAffinityRulesNotMatch */
/* NodeAffinity failure detail: 0 = the pod's selector / required terms
 * (ErrReasonPod), KSIM_NA_ENFORCED = the profile's addedAffinity (errReasonEnforced) */
#define KSIM_NA_ENFORCED         1u
/* VolumeBinding failure detail: the reasons FindPodVolumes gives the node */
#define KSIM_VB_NODE_CONFLICT    1u   /* a bound PV's node affinity (ErrReasonNodeConflict) */
#define KSIM_VB_BIND_CONFLICT    2u   /* an unbound claim: no PV, no provisioning (ErrReasonBindConflict) */

/* per-pod cycle status */
#define KSIM_STATUS_SCHEDULED      0
#define KSIM_STATUS_UNSCHEDULABLE  1   /* FitError: no feasible node */
#define KSIM_STATUS_ERROR          2   /* a plugin returned a status other than Success /
                                          Unschedulable: the cycle fails with framework.Error,
                                          no node is chosen (chosen[] = KSIM_CHOSEN_ERROR) */
#define KSIM_CHOSEN_ERROR         -2

/* NetworkBandwidth fail_detail (plugin.go:52-102, in the order Filter checks) */
#define KSIM_NB_INSUFFICIENT   1u   /* Unschedulable: allocated + request > limit */
#define KSIM_NB_NO_LIMIT       2u   /* Skip: node has no limit annotation       -> Error */
#define KSIM_NB_LIMIT_BAD      3u   /* Error: node limit does not parse */
#define KSIM_NB_INGRESS_BAD    4u   /* Error: pod ingress request does not parse */
#define KSIM_NB_EGRESS_BAD     5u   /* Error: pod egress request does not parse */
#define KSIM_NB_NO_REQUEST     6u   /* Skip: pod requests no bandwidth          -> Error */

/* ---- cluster snapshot (SoA; one entry per node in nodeTree order) -------- */
/* Mirrors [upstream] framework.NodeInfo: Allocatable, Requested,
 * NonZeroRequested, len(Pods); node.Spec.{Unschedulable,Taints}; node labels. */
typedef struct ksim_node_table {
  int32_t n_nodes;
  int32_t n_scalar;               /* <= KSIM_MAX_SCALAR */
  int32_t n_label_cols;           /* <= KSIM_MAX_LABEL_COLS */
  int32_t _pad0;
  const int64_t*  alloc_cpu;      /* Allocatable.MilliCPU */
  const int64_t*  alloc_mem;      /* Allocatable.Memory */
  const int64_t*  alloc_eph;      /* Allocatable.EphemeralStorage */
  const int32_t*  alloc_pods;     /* Allocatable.AllowedPodNumber */
  const int64_t*  alloc_scalar;   /* [n_scalar][n_nodes] */
  const int64_t*  req_cpu;        /* Requested.* */
  const int64_t*  req_mem;
  const int64_t*  req_eph;
  const int64_t*  req_scalar;     /* [n_scalar][n_nodes] */
  const int64_t*  nz_cpu;         /* NonZeroRequested.MilliCPU */
  const int64_t*  nz_mem;         /* NonZeroRequested.Memory */
  const int32_t*  num_pods;       /* len(NodeInfo.Pods) */
  const uint32_t* flags;          /* KSIM_NODE_* */
  const uint16_t* taints;         /* [KSIM_MAX_NODE_TAINTS][n_nodes]; taint vocab id, 0 terminates */
  const uint32_t* labels;         /* [n_label_cols][n_nodes]; label value id, 0 = key absent */
  int32_t n_classes;              /* <= KSIM_MAX_CLASSES */
  int32_t _pad1;
  const int32_t* class_count;     /* [n_classes][n_nodes]: pods (or term weights) of each count
                                     class on each node, from the pods already bound */
  /* NetworkBandwidth (NULL when no node carries the limit annotation), milli-units */
  const int64_t* nb_limit;        /* the node-limit annotation's quantity */
  const int64_t* nb_alloc;        /* getNodeAllocatedAmount over the pods already bound */
} ksim_node_table;

/* Vocabularies the host interned (strings stay on the host). */
typedef struct ksim_vocab {
  int32_t n_taints;               /* taint vocabulary size incl. id 0 (<= 64*KSIM_TAINT_WORDS) */
  int32_t n_label_values;         /* entries of label_num / label_num_ok */
  const uint8_t* taint_effect;    /* [n_taints] KSIM_EFFECT_* */
  const int32_t* label_col_offset;/* [n_label_cols]: base index of the column's value ids */
  const int64_t* label_num;       /* strconv.ParseInt(value,10,64) per (col, value id) */
  const uint8_t* label_num_ok;    /* 1 if that parse succeeded */
  int32_t n_topo_log;             /* >= n_nodes + 1 when any pod spreads with ScheduleAnyway */
  int32_t _pad;
  const double* topo_log;         /* [size] = math.Log(float64(size + 2)) (PTS topologyNormalizingWeight),
                                     computed by the host so the device never evaluates log */
} ksim_vocab;

/* One NodeSelectorRequirement compiled against the vocabulary. */
typedef struct ksim_label_expr {
  int64_t  num;                     /* Gt/Lt operand */
  uint32_t vals[KSIM_EXPR_VALS];    /* value ids (In/NotIn) or node positions (FIELD_*) */
  uint16_t col;                     /* node label column */
  uint8_t  op;                      /* KSIM_OP_* */
  uint8_t  nvals;
  uint32_t _pad;
} ksim_label_expr;                  /* 40 bytes */

/* NodeSelectorTerm = AND of exprs[first .. first+n_expr); n_expr == 0 -> empty
 * term, which matches nothing (component-helpers nodeSelectorTerm.match). */
typedef struct ksim_term {
  int32_t first_expr;
  int32_t n_expr;
  int32_t weight;                   /* PreferredSchedulingTerm.Weight (preferred terms only) */
  int32_t _pad;
} ksim_term;                        /* 16 bytes */

/* A pod compiled by the host (resources already summed per Fit PreFilter
 * computePodResourceRequest / NodeInfo calculateResource). */
typedef struct ksim_pod {
  int64_t  req_cpu, req_mem, req_eph;        /* requests: max(sum containers, any init) + overhead */
  int64_t  nz_cpu, nz_mem;                   /* non-zero requests (100m / 200Mi defaults) */
  int64_t  scalar_req[KSIM_MAX_SCALAR];      /* per node scalar column; 0 = not requested */
  uint64_t tol_filter[KSIM_TAINT_WORDS];     /* bit t: taint t tolerated by pod.Spec.Tolerations */
  uint64_t tol_prefer[KSIM_TAINT_WORDS];     /* bit t: tolerated by tolerations with effect "" or PreferNoSchedule */
  int32_t  node_name;                        /* -1: spec.nodeName empty; -2: unknown node; else node position */
  uint32_t flags;                            /* KSIM_POD_* */
  int32_t  sel_first, sel_count;             /* spec.nodeSelector as In{value} exprs (AND) */
  int32_t  req_term_first, req_term_count;   /* required node affinity terms (OR) */
  int32_t  pref_term_first, pref_term_count; /* preferred node affinity terms */
  int32_t  use_first, use_count;             /* topology uses (PodTopologySpread / InterPodAffinity) */
  int32_t  add_first, add_count;             /* count-class contributions once bound (NodeInfo.AddPod) */
  uint32_t topo_flags;                       /* KSIM_POD_IPA_* */
  uint32_t nb_flags;                         /* KSIM_POD_NB_* */
  int32_t  nn_first, nn_count;               /* PreFilterResult.NodeNames (KSIM_POD_NODE_NAMES) */
  /* Bound PersistentVolumeClaims (see "volume groups" below): VolumeBinding's
   * PV node affinity and VolumeZone's PV topology labels as groups of terms. */
  int32_t  vb_first, vb_count;               /* VolumeBinding groups: terms [vb_first, +vb_count) */
  int32_t  vz_first, vz_count;               /* VolumeZone groups: terms [vz_first, +vz_count) */
  int64_t  nb_req;                           /* NetworkBandwidth Filter request (milli): ingress
                                                + egress request annotations, each falling back
                                                to the *-bandwidth annotation */
  int64_t  nb_add;                           /* added to the node's allocated amount once bound
                                                (request annotations only, unparsable ones skipped) */
  int32_t  added_term_first, added_term_count;/* NodeAffinityArgs.addedAffinity required terms
                                                (KSIM_POD_ADDED_AFFINITY) */
} ksim_pod;

/* Volume groups.  A pod's PersistentVolumeClaims bound to PersistentVolumes
 * become node-label requirements (host compile, ksim/encode.py):
 *   VolumeBinding  (binder.go checkBoundClaims -> volumeutil.CheckNodeAffinity)
 *                  one group per PV with spec.nodeAffinity.required: its
 *                  NodeSelectorTerms (OR), evaluated on a node that has only
 *                  labels (a matchFields metadata.name requirement sees "");
 *   VolumeZone     (volume_zone.go Filter) one group per PV topology label
 *                  (topology.kubernetes.io/zone|region and the beta
 *                  failure-domain keys): the terms {key In LabelZonesToSet(v)}
 *                  and {every topology key DoesNotExist} (a node without any
 *                  topology label passes).
 *   VolumeBinding, unbound WaitForFirstConsumer claims (binder.go
 *                  FindPodVolumes): groups of node-name / label terms the host
 *                  derives from the matching PVs and the class's provisioning,
 *                  their group index or-ed with KSIM_VB_UNBOUND_GROUP, after
 *                  the bound-PV groups.
 * Terms of a list are consecutive ksim_term entries of the pod set; a term's
 * `weight` is its group index (0, 0, 1, 2, 2, ... non-decreasing).  The filter
 * passes iff every group has a matching term.  VolumeBinding's failure detail
 * is KSIM_VB_NODE_CONFLICT if a bound-PV group failed, | KSIM_VB_BIND_CONFLICT
 * if an unbound-claim group failed ("node(s) had volume node affinity
 * conflict", "node(s) didn't find available persistent volumes to bind",
 * joined in that order); VolumeZone's is 0 ("node(s) had no available volume
 * zone"). */
#define KSIM_VB_UNBOUND_GROUP    (1 << 30)

/* Count classes.  The host evaluates every label selector / affinity term
 * against pod namespaces and labels once (that string work does not depend
 * on placement) and hands the device integer classes:
 *   class_count[c][node] = sum over pods bound to node of their multiplicity in c.
 * A "use" tells the device which class to aggregate over which topology key
 * and in which role ([upstream] podtopologyspread / interpodaffinity):
 *   PTS_HARD           DoNotSchedule constraint: TpPairToMatchNum over eligible nodes,
 *                      skew vs the critical-path minimum (Filter)
 *   PTS_SOFT           ScheduleAnyway constraint: TopologyPairToPodCounts (PreScore/Score)
 *   IPA_EXISTING_ANTI  existingAntiAffinityCounts of a carried required anti-affinity term
 *   IPA_AFFINITY       affinityCounts of one incoming required affinity term
 *   IPA_ANTI           antiAffinityCounts of one incoming required anti-affinity term
 *   IPA_SCORE          topologyScore += arg x domain count
 *   IPA_SCORE_HARD     topologyScore += hardPodAffinityWeight x domain count */
#define KSIM_USE_PTS_HARD           0
#define KSIM_USE_PTS_SOFT           1
#define KSIM_USE_IPA_EXISTING_ANTI  2
#define KSIM_USE_IPA_AFFINITY       3
#define KSIM_USE_IPA_ANTI           4
#define KSIM_USE_IPA_SCORE          5
#define KSIM_USE_IPA_SCORE_HARD     6
#define KSIM_USE_NODE_PORT          7   /* NodePorts: the node must hold no pod of class cls (col unused) */
#define KSIM_USE_IMAGE              8   /* ImageLocality: raw score = class count (per node, static) */
#define KSIM_USEF_SELF_MATCH        1u   /* PTS: constraint selector matches the pod itself */
#define KSIM_USEF_HONOR_AFFINITY    2u   /* PTS: nodeAffinityPolicy Honor (default) */
#define KSIM_USEF_HONOR_TAINTS      4u   /* PTS: nodeTaintsPolicy Honor (default Ignore) */
#define KSIM_USEF_HOSTNAME          8u   /* PTS: topologyKey == kubernetes.io/hostname */

typedef struct ksim_topo_use {
  int32_t  cls;                     /* count class; -1 = counts no pod */
  int32_t  arg;                     /* PTS: maxSkew; IPA_SCORE: signed weight */
  uint16_t col;                     /* topology key label column, KSIM_COL_NONE if no node has it */
  uint8_t  kind;                    /* KSIM_USE_* */
  uint8_t  flags;                   /* KSIM_USEF_* */
  int32_t  _pad;
} ksim_topo_use;                    /* 16 bytes */

typedef struct ksim_class_add {
  int32_t cls;
  int32_t count;
} ksim_class_add;

typedef struct ksim_pod_set {
  int32_t n_pods;
  int32_t n_exprs;
  int32_t n_terms;
  int32_t _pad;
  const ksim_pod* pods;
  const ksim_label_expr* exprs;
  const ksim_term* terms;
  int32_t n_uses;
  int32_t n_adds;
  const ksim_topo_use* uses;
  const ksim_class_add* adds;
  int32_t n_nn;                     /* entries of nn */
  int32_t _pad2;
  const int32_t* nn;                /* PreFilterResult node positions (see KSIM_POD_NODE_NAMES) */
} ksim_pod_set;

/* NodeResourcesFit ScoringStrategy types (NodeResourcesFitArgs.scoringStrategy.type) */
#define KSIM_FIT_LEAST_ALLOCATED              0   /* least_allocated.go leastResourceScorer */
#define KSIM_FIT_MOST_ALLOCATED               1   /* most_allocated.go mostResourceScorer */
#define KSIM_FIT_REQUESTED_TO_CAPACITY_RATIO  2   /* requested_to_capacity_ratio.go (broken-linear shape) */

/* Profile: the converted KubeSchedulerProfile (simulator/scheduler/scheduler.go:199-249,
 * plugins.go:185-220) restricted to what the cycle needs, with the plugin args
 * NewPluginConfig merges over the defaults (plugins.go:103-179).  An arg the
 * engine does not implement is refused by the host compile (ksim/profile.py),
 * never dropped. */
typedef struct ksim_profile {
  int32_t n_filter;
  int32_t n_score;
  uint8_t filter[KSIM_MAX_FILTER];     /* ksim_plugin ids, profile Filter order */
  uint8_t score[KSIM_MAX_SCORE];       /* ksim_plugin ids, profile Score order */
  int32_t score_weight[KSIM_MAX_SCORE];/* profile weights; 0 is treated as 1 (framework) */
  int32_t percentage_of_nodes_to_score;/* 0 = adaptive (simulator default), 100 = all */
  /* NodeResourcesFit ScoringStrategy: resources and weights (weight 0 defaulted to 1) */
  int32_t fit_n_res;
  int32_t fit_res[KSIM_MAX_RES];       /* KSIM_RES_* */
  int64_t fit_res_weight[KSIM_MAX_RES];
  /* NodeResourcesBalancedAllocation resources */
  int32_t ba_n_res;
  int32_t ba_res[KSIM_MAX_RES];
  int64_t ba_res_weight[KSIM_MAX_RES];
  int32_t hard_pod_affinity_weight;    /* InterPodAffinityArgs (default 1) */
  uint32_t fit_ignored_scalar;         /* NodeResourcesFitArgs ignoredResources / ignoredResourceGroups:
                                          bit k = Fit's Filter skips scalar column k (extended resources
                                          only; the scores and the binds still count it) */
  uint64_t tiebreak_seed;              /* selectHost fixed-seed tie-break TB(seed) */
  /* ABI 8: the rest of NodeResourcesFitArgs.scoringStrategy and DefaultPreemptionArgs */
  int32_t fit_strategy;                /* KSIM_FIT_* */
  int32_t fit_n_shape;                 /* RequestedToCapacityRatio: shape points (1..KSIM_MAX_SHAPE) */
  int32_t fit_shape_util[KSIM_MAX_SHAPE];  /* utilization, strictly increasing in [0, 100] */
  int32_t fit_shape_score[KSIM_MAX_SHAPE]; /* score already scaled to [0, 100]
                                              (x MaxNodeScore / MaxCustomPriorityScore = x 10) */
  int32_t preempt_min_pct;             /* DefaultPreemptionArgs.minCandidateNodesPercentage (default 10) */
  int32_t preempt_min_abs;             /* ... minCandidateNodesAbsolute (default 100) */
} ksim_profile;

/* Full per-node outputs of one scheduling cycle (compat mode: what the
 * wrapper records into the result store).  Any pointer may be NULL. */
typedef struct ksim_eval_out {
  uint8_t*  fail_plugin;   /* [n_nodes] filter-order index of the first failing plugin,
                              KSIM_PASSED, or KSIM_NOT_EVALUATED (ADAPT scan never reached it) */
  uint32_t* fail_detail;   /* [n_nodes] reason detail (Fit bits, taint id, ...) */
  uint8_t*  scored;        /* [n_nodes] 1 if the node was in the list passed to Score */
  int64_t*  raw;           /* [n_score][n_nodes] Score() result for scored nodes */
  int64_t*  norm;          /* [n_score][n_nodes] after NormalizeScore (raw if the plugin has none) */
  int64_t*  total;         /* [n_nodes] sum of norm * profile weight */
  int32_t chosen;          /* node position, -1 if unschedulable */
  int32_t status;          /* KSIM_STATUS_* */
  int32_t n_feasible;      /* feasible nodes kept (<= K) */
  int32_t n_evaluated;     /* nodes whose filter chain ran */
  int32_t n_processed;     /* feasible + failed (nextStartNodeIndex advance) */
  int32_t k_to_find;       /* numFeasibleNodesToFind */
  int32_t next_start;      /* nextStartNodeIndex after this cycle */
  int32_t _pad;
} ksim_eval_out;

typedef struct ksim_batch_stats {
  int64_t pods;            /* cycles run */
  int64_t scheduled;
  int64_t unschedulable;
  int64_t evals;           /* pod x node filter evaluations (SURVEY §8(d) definition) */
  double  device_ms;       /* device time of the batch (HIP events) */
  int64_t batches;         /* speculative batches run (batch path) */
  int64_t truncations;     /* batches cut short by an exhausted candidate list */
  int64_t perpod_cycles;   /* cycles run on the per-pod path */
} ksim_batch_stats;

typedef struct ksim_handle ksim_handle;

/* ---- lifecycle ----------------------------------------------------------- */
int  ksim_abi_version(void);
/* sizeof() of the ABI structs, for binding-layout checks: which = 0 node_table,
 * 1 vocab, 2 label_expr, 3 term, 4 pod, 5 pod_set, 6 profile, 7 eval_out, 8 batch_stats,
 * 9 topo_use, 10 class_add */
size_t ksim_abi_sizeof(int which);
int  ksim_create(int device, ksim_handle** out);
void ksim_destroy(ksim_handle* h);
const char* ksim_last_error(const ksim_handle* h);

/* ---- configuration / snapshot ------------------------------------------- */
/* The compiled profile: plugin order and enable bits, score weights, plugin
 * args.  Replaces what the simulator hands upstream scheduler.New after
 * convertConfigurationForSimulator (simulator/scheduler/scheduler.go:199-249),
 * ConvertForSimulator (scheduler/plugin/plugins.go:185-288) and NewPluginConfig
 * (plugins.go:103-179). */
int ksim_set_profile(ksim_handle* h, const ksim_profile* p);
/* Replace the whole snapshot (nodes already in nodeTree order). Resets
 * nextStartNodeIndex.  The device-side counterpart of the scheduler cache's
 * Snapshot / UpdateSnapshot that the wrapped plugins read through
 * framework.NodeInfo (scheduler/plugin/wrappedplugin.go:491, 388). */
int ksim_set_cluster(ksim_handle* h, const ksim_node_table* nodes, const ksim_vocab* vocab);
/* Node informer deltas (the scheduler cache's AddNode / UpdateNode /
 * RemoveNode, then UpdateSnapshot) without losing the binds
 * the cycles made.  `nodes` is the new snapshot in nodeTree order (static
 * columns, vocabulary, and the dynamic columns of the pods bound in it);
 * old_pos[i] is the current position of new node i, or -1 for an added node.
 * On a kept node the binds made since the last snapshot (the device's dynamic
 * column minus the snapshot's, at old_pos) are replayed on top of the table,
 * for the scalar columns and count classes the handle already has; added
 * nodes, appended scalar columns and appended classes take the table as is.
 * The table becomes the ksim_reset_cluster snapshot.  Label columns may be
 * added or dropped (the vocabulary is replaced).  nextStartNodeIndex carries
 * over mod the new node count ([upstream] the scheduler keeps the index and
 * scans nodes[(index + i) % numAllNodes]); the pod sequence carries over.
 * Loaded pods and the bound-pod table refer to node positions and are
 * dropped.  Unsharded handles only. */
int ksim_upsert_nodes(ksim_handle* h, const ksim_node_table* nodes, const ksim_vocab* vocab, const int32_t* old_pos);
/* RemoveNode of the node at position `pos` (later nodes move down by one),
 * from the device-resident snapshot alone. */
int ksim_remove_node(ksim_handle* h, int32_t pos);
/* UpdateNode in place (ABI 11): the static columns of the nodes at positions
 * rows[0..n_rows) -- allocatable (and its reciprocals), scalar allocatable,
 * flags, taints, label value ids, the NetworkBandwidth limit -- taken from
 * `nodes` at those positions.  `nodes` / `vocab` must have the handle's node
 * count, scalar columns, label columns and count classes and the same taint
 * and label-value vocabulary sizes; anything else is KSIM_E_INVALID (send the
 * table with ksim_upsert_nodes).  Dynamic columns, count classes and
 * nextStartNodeIndex are kept; loaded pods are dropped (their filter plans
 * read the cluster's taint and unschedulable facts).  The encoder's
 * ksim_encoder_changed_rows names the rows when a delta moved no node. */
int ksim_update_node_rows(ksim_handle* h, const ksim_node_table* nodes, const ksim_vocab* vocab, const int32_t* rows,
                          int32_t n_rows);
/* Read back the dynamic node state (Requested/NonZeroRequested/len(Pods)). NULL skips a field. */
int ksim_get_node_state(ksim_handle* h, int64_t* req_cpu, int64_t* req_mem, int64_t* req_eph,
                        int64_t* nz_cpu, int64_t* nz_mem, int32_t* num_pods);
/* Read back NetworkBandwidth's allocated amount per node (milli-units). */
int ksim_get_nb_alloc(ksim_handle* h, int64_t* out);
/* Read back the count classes [n_classes][n_nodes] (PodTopologySpread / InterPodAffinity state). */
int ksim_get_class_count(ksim_handle* h, int32_t* out);
int ksim_get_next_start(ksim_handle* h, int32_t* next_start);
int ksim_set_next_start(ksim_handle* h, int32_t next_start);
/* Pod sequence number used by the tie-break (advances once per cycle). */
int ksim_set_pod_seq(ksim_handle* h, int64_t seq);

/* ---- scheduling cycles --------------------------------------------------- */
/* One full cycle for pod `pod_index` of `pods` (compat mode) incl. assume/bind.
 * It replaces the original-plugin calls inside the wrapped plugins: PreFilter
 * (scheduler/plugin/wrappedplugin.go:459-486), Filter (:491-516), PreScore
 * (:427-454), Score (:388-413), NormalizeScore (:346-383), and the selected
 * node that Reserve records (:583-612).  fail_plugin / fail_detail, raw /
 * norm and total are what those wrappers pass to Store.AddFilterResult,
 * AddScoreResult and AddNormalizedScoreResult
 * (scheduler/plugin/resultstore/store.go:418-502). */
int ksim_eval_pod(ksim_handle* h, const ksim_pod_set* pods, int32_t pod_index, ksim_eval_out* out);

/* The same cycle around the host's extender round trip (SURVEY §8(f) 4;
 * schedule_one.go findNodesThatPassExtenders / prioritizeNodes):
 *   ksim_eval_pod_filter  PreFilter, Filter and the numFeasibleNodesToFind
 *                         window.  fail_plugin / fail_detail and the scalars
 *                         (n_feasible, n_evaluated, n_processed, k_to_find,
 *                         next_start) are filled; the kept nodes are the ones
 *                         with fail_plugin == KSIM_PASSED.  The host sends them
 *                         to its extenders.
 *   ksim_eval_pod_finish  ext_fail[n] nonzero: an extender filtered the kept
 *                         node out (fail_plugin = KSIM_FAIL_EXTENDER).
 *                         ext_score[n]: the extenders' combined weighted scores,
 *                         added to the plugin totals.  Either may be NULL.
 *                         Score, NormalizeScore over the remaining nodes,
 *                         selectHost and the bind; every output as ksim_eval_pod.
 * nextStartNodeIndex advances by the filter pass, as upstream (before the
 * extenders).  Unsharded handles only. */
/* The simulator's extender service forwards these calls to the extenders
 * (scheduler/extender/extender.go:122-148, Filter and Prioritize). */
int ksim_eval_pod_filter(ksim_handle* h, const ksim_pod_set* pods, int32_t pod_index, ksim_eval_out* out);
int ksim_eval_pod_finish(ksim_handle* h, const uint8_t* ext_fail, const int64_t* ext_score, ksim_eval_out* out);
/* Assume/forget a pod on a node (NodeInfo.AddPod / RemovePod): the state change
 * behind Reserve / Unreserve (scheduler/plugin/wrappedplugin.go:583, 617). */
int ksim_assume(ksim_handle* h, const ksim_pod_set* pods, int32_t pod_index, int32_t node);
int ksim_forget(ksim_handle* h, const ksim_pod_set* pods, int32_t pod_index, int32_t node);

/* ---- framework-driven compat mode ---------------------------------------------
 * The simulator runs upstream's framework with parallelism 16 and
 * percentageOfNodesToScore 0 (simulator/scheduler/scheduler.go:149,153, re-
 * defaulted at :231-241).  The FRAMEWORK then decides which nodes Filter runs
 * on (16 racing Parallelizer workers stop after numFeasibleNodesToFind feasible
 * nodes), which feasible list PreScore / Score / NormalizeScore see, and which
 * tied node selectHost's reservoir hands to Reserve.  ksim_eval_pod makes those
 * choices itself (sequential scan, TB tie-break); these calls answer the
 * engine-backed plugins under the framework's own choices instead:
 *
 *   ksim_fw_prefilter  PreFilter, then Filter of EVERY node of the pod's scan
 *                      set (all nodes, or PreFilterResult.NodeNames), so a
 *                      worker reaching any node finds its answer: fail_plugin
 *                      / fail_detail for every node (KSIM_NOT_EVALUATED only
 *                      for nodes outside PreFilterResult.NodeNames, which the
 *                      framework never hands to Filter).  n_feasible = nodes
 *                      passing, n_evaluated = scan-set size, k_to_find =
 *                      numFeasibleNodesToFind(scan-set size) for the
 *                      framework's scan.  nextStartNodeIndex and the tie-break
 *                      sequence are the framework's: untouched.  status
 *                      KSIM_STATUS_ERROR: a PreFilterResult name is not a node
 *                      (the framework fails the cycle; no Filter runs).  A
 *                      NetworkBandwidth Filter Skip / Error shows as its
 *                      fail_detail (KSIM_NB_NO_LIMIT and above): the framework
 *                      turns it into framework.Error.
 *                      Replaces the original plugins' PreFilter and Filter
 *                      behind wrappedPlugin.PreFilter / Filter
 *                      (wrappedplugin.go:459-486, 491-516).
 *   ksim_fw_score      PreScore, Score and NormalizeScore over exactly the
 *                      framework's feasible list nodes[0..n) (any order; each a
 *                      node that passed the filter pass, once):
 *                      PodTopologySpread's IgnoredNodes, pair registration and
 *                      topologyNormalizingWeight over the list, raw / norm /
 *                      total / scored for the listed nodes (the same layout as
 *                      ksim_eval_out; the entries of unlisted nodes are left
 *                      as the caller had them).  No selectHost, no bind: chosen = -1
 *                      (KSIM_CHOSEN_ERROR with status KSIM_STATUS_ERROR when a
 *                      listed node's NetworkBandwidth Score fails).
 *                      Replaces PreScore / Score (wrappedplugin.go:427-454,
 *                      388-413).
 *   ksim_fw_normalize  NormalizeScore of the plugin at profile score slot
 *                      `score_slot` over an explicit (node, score) list, e.g.
 *                      the NodeScoreList the wrapper passes
 *                      (wrappedplugin.go:356-375), with the PreScore state of
 *                      the last ksim_fw_score (IgnoredNodes, topologyScore
 *                      emptiness).  out[j] = normalized score of entry j;
 *                      plugins without NormalizeScore copy the scores.
 *   Reserve / Unreserve with the framework's node: ksim_assume / ksim_forget
 *                      (wrappedplugin.go:583-584, 617); they return once the
 *                      update is queued on the handle's stream (every later
 *                      call on the handle sees it; a device error shows at the
 *                      next call that synchronizes).
 * Any other cycle or snapshot call on the handle ends a framework cycle in
 * flight.  Unsharded handles only. */
int ksim_fw_prefilter(ksim_handle* h, const ksim_pod_set* pods, int32_t pod_index, ksim_eval_out* out);
int ksim_fw_score(ksim_handle* h, const int32_t* nodes, int32_t n, ksim_eval_out* out);
int ksim_fw_normalize(ksim_handle* h, int32_t score_slot, const int32_t* nodes, const int64_t* scores, int32_t n,
                      int64_t* out);
/* Nominated pods (ABI 8).  After a preemption the framework keeps the
 * preemptor nominated to a node (PostFilter's result, handleSchedulingFailure
 * -> SchedulingQueue.AddNominatedPod) and later cycles run
 * RunFilterPluginsWithNominatedPods (framework/runtime/framework.go): on a node
 * with nominated pods of equal or higher priority, Filter first runs on a
 * clone of the NodeInfo with those pods added and a clone of the cycle state
 * after the PreFilterExtensions' AddPod (addNominatedPods), then -- if that
 * passed -- on the plain NodeInfo; the wrapper records both passes.
 *   ksim_fw_filter_nominated  the first pass, for the cycle in flight
 *                             (ksim_fw_prefilter): group k is node nodes[k]
 *                             with pods [first[k], first[k] + count[k]) of
 *                             `nominated` added.  fail_plugin[k] /
 *                             fail_detail[k] are the filter outcome there
 *                             (KSIM_PASSED or the failing plugin's filter
 *                             index).  The second pass is ksim_fw_prefilter's
 *                             answer for the node; the framework (the host)
 *                             combines them.  The cycle's own PreFilter state
 *                             is unchanged afterwards.  Replaces the
 *                             original plugins' AddPod (PreFilterExtensions)
 *                             and Filter behind wrappedplugin.go:491-516. */
int ksim_fw_filter_nominated(ksim_handle* h, const ksim_pod_set* nominated, int32_t n_nodes, const int32_t* nodes,
                             const int32_t* first, const int32_t* count, uint8_t* fail_plugin,
                             uint32_t* fail_detail);

/* Batch mode: upload a pod set once (device-resident), then schedule a range
 * of it in queue order; chosen[i] = node position or -1.  The whole-cycle
 * entry point of SURVEY §8(b) (ksim_schedule_batch): the same placements as
 * running the wrapped plugins pod by pod, without a Go call per node. */
int ksim_load_pods(ksim_handle* h, const ksim_pod_set* pods);
int ksim_schedule_loaded(ksim_handle* h, int32_t first, int32_t count,
                         int32_t* chosen, ksim_batch_stats* stats);
/* Convenience: load + schedule all. */
int ksim_schedule_batch(ksim_handle* h, const ksim_pod_set* pods, int32_t* chosen,
                        ksim_batch_stats* stats);

/* Restore the dynamic node state (Requested / NonZeroRequested / len(Pods)) to
 * the snapshot given at ksim_set_cluster, and nextStartNodeIndex / pod
 * sequence to 0 (device-side copy; used by sweeps and the bench). */
int ksim_reset_cluster(ksim_handle* h);

/* ---- node sharding (multi-GPU) -------------------------------
 * A cluster of n_total nodes (nodeTree order) is split into contiguous shards.
 * A shard handle holds global positions [node_base, node_base + n_nodes) of
 * the table given to ksim_set_cluster; tie-break keys, spec.nodeName,
 * metadata.name selectors and chosen[] use GLOBAL positions.  Sharded runs
 * take batchable pods (P100, no topology uses) and exchange, per batch of 256
 * pods, one all-gather of the shards' candidate records (18 KB per shard)
 * and one all-reduce (max) of 256 pair keys. */
#define KSIM_COMM_ID_BYTES 128
/* Must precede ksim_set_cluster. */
int ksim_set_shard(ksim_handle* h, int32_t node_base, int32_t n_total);
/* One process per GPU over RCCL: rank 0 creates the id (ncclGetUniqueId),
 * every rank passes the same bytes; ksim_schedule_loaded then runs sharded. */
/* Replicated node sharding (an alternative to ksim_set_shard for the P100
 * batch path): the handle holds EVERY node (ksim_set_cluster with the whole
 * snapshot) and its batch top-T evaluates only local positions [eval_lo,
 * eval_hi); the ranks' ranges tile the cluster in rank order.  Each batch then
 * needs one exchange (the all-gather of the per-rank candidate records): the
 * pair keys of every guess are computed locally and every rank binds every
 * placement, so the replicas stay equal.  Other runs (per-pod cycles, ADAPT)
 * execute whole on every replica.  Call after ksim_set_cluster (a new
 * snapshot clears it) and before ksim_comm_init / the group call. */
int ksim_set_eval_range(ksim_handle* h, int32_t eval_lo, int32_t eval_hi);
int ksim_comm_unique_id(uint8_t* id /* [KSIM_COMM_ID_BYTES] */);
int ksim_comm_init(ksim_handle* h, int32_t rank, int32_t world, const uint8_t* id);
/* An in-process group of shard handles on one device (exchanges by device
 * copies): the same protocol without a communicator.  hs[i] must tile the
 * cluster in order; chosen / stats as ksim_schedule_loaded (evals summed). */
int ksim_group_schedule_loaded(ksim_handle** hs, int32_t n, int32_t first, int32_t count,
                               int32_t* chosen, ksim_batch_stats* stats);

/* ---- measurement ----------------------------------------------------------- */
/* Schedule loaded pods [first, first+count) exactly as ksim_schedule_loaded
 * would, with a HIP event between every kernel on the engine's stream.
 * avg_ms[k] = mean duration of kernel k over its launches that did work
 * (0 if never launched); launches[k] = that count.  Kernel k is named by
 * ksim_kernel_name(k).  Returns the number of kernel kinds (<= cap). */
int ksim_time_kernels(ksim_handle* h, int32_t first, int32_t count, double* avg_ms,
                      int64_t* launches, int32_t cap);
const char* ksim_kernel_name(int32_t k);
/* The evaluation kernel of the path pod `first` takes (P100 batch path:
 * k_batch_eval over the batch starting at `first`; per-pod path:
 * k_filter_score of pod `first`), launched `reps` times back to back on the
 * engine's stream between two HIP events, against the current snapshot
 * (the kernel only writes scratch).  *avg_ms = elapsed / reps; the kernel's
 * ksim_kernel_name index goes to *kernel.  KSIM_E_UNSUPPORTED for the ADAPT
 * batch path (its evaluations span two kernels). */
int ksim_time_eval(ksim_handle* h, int32_t first, int32_t reps, double* avg_ms, int32_t* kernel);
/* Batch-path diagnostics of the last ksim_schedule_loaded: out[0] batches,
 * out[1] truncations (an exhausted candidate list ended a batch), out[2] cuts
 * (a pod's exact choice was a node bound earlier in its batch, ending it);
 * out[3..18] device phase-clock accumulators since ksim_set_cluster (100 MHz
 * ticks: [3] chain prologue, [4] chain loop, [5] chain epilogue, [6] chain
 * launches); out[19] hipGraphs captured since ksim_create (a weight sweep that
 * keeps its graphs across ksim_set_profile captures none); out[20] device
 * time of the last ksim_match_terms in ns (HIP events); out[21..24] framework-
 * driven calls since ksim_create: ksim_fw_score answered on the host / on the
 * device, ksim_fw_normalize answered from ksim_fw_score's list / on the device;
 * out[25] the batch evaluation launches' instantiations launched or captured
 * by this process (a bitmask: bits 0..9 k_batch_top_commit -- flush direct /
 * overlay-indexed, node-stationary direct / indexed, KEEP default-shape /
 * generic, direct default-shape / generic, indexed default-shape / generic --
 * bits 16..21 k_batch_top -- static-class default-shape KEEP, static-class
 * default-shape, static-class, FAST default-shape, FAST, generic keys);
 * out[26] topology batch pods committed on a zone variant (their batch moved
 * their DoNotSchedule domain verdicts; ksim_tbatch.hip TbVar), cumulative.
 * Returns the number of values written (<= n). */
int ksim_get_diag(ksim_handle* h, int64_t* out, int32_t n);
/* Batch-path geometry compiled into the library: out[0] pods per batch (B),
 * out[1] candidate keys kept per pod (T), out[2] nodes per wave tile,
 * out[3] keys a tile keeps per pod.  Returns the number written (<= n). */
int ksim_batch_geometry(int32_t* out, int32_t n);

/* ---- PostFilter: DefaultPreemption ----------------------- */
/* The bound pods preemption may evict: per pod its node, priority, start
 * time (any monotone unit) and the requests it holds on the node
 * (cpu, memory, ephemeral-storage, then the scalar columns). */
#define KSIM_PREEMPT_REQ (3 + KSIM_MAX_SCALAR)
typedef struct ksim_bound_pods {
  int32_t n, _pad;
  const int32_t* node;        /* [n] node position */
  const int32_t* priority;    /* [n] .spec.priority */
  const int64_t* start_time;  /* [n] status.startTime */
  const int64_t* req;         /* [n][KSIM_PREEMPT_REQ] */
} ksim_bound_pods;

typedef struct ksim_preempt_out {
  int32_t nominated;          /* node position; -1: preemption cannot help */
  int32_t n_victims;          /* victims on the nominated node (may exceed victims_cap) */
  int32_t n_potential;        /* nodesWherePreemptionMightHelp */
  int32_t n_candidates;       /* candidates the dry run kept (<= numCandidates) */
  int32_t* victims;           /* [victims_cap] bound-pod indices, reprieve (importance) order */
  int32_t victims_cap, _pad;
} ksim_preempt_out;

/* Replace the bound-pod table (copied; the engine orders it per node by
 * importance: priority desc, start time asc). */
int ksim_set_bound_pods(ksim_handle* h, const ksim_bound_pods* b);
/* DefaultPreemption's PostFilter for an unschedulable pod of `priority`
 * (default_preemption.go / preemption.go, v1.26) on the current snapshot,
 * without changing it.  It replaces the original plugin's PostFilter that the
 * wrapper calls and records (scheduler/plugin/wrappedplugin.go:518-544,
 * Store.AddPostFilterResult store.go:437):
 *   potential nodes  the nodes whose filter status is Unschedulable, i.e. the
 *                    ones that failed NodeResourcesFit (the plugins before it
 *                    return UnschedulableAndUnresolvable);
 *   dry run          SelectVictimsOnNode on each, in nodeTree order from
 *                    offset 0 (upstream draws a random offset), keeping the
 *                    first numCandidates = max(minCandidateNodesPercentage %
 *                    of them, minCandidateNodesAbsolute) candidates (the
 *                    profile's DefaultPreemptionArgs; 10 % and 100 default);
 *   selection        pickOneNodeForPreemption: lowest highest-victim
 *                    priority, lowest sum of (priority + 2^31), fewest
 *                    victims, latest earliest start among the highest-
 *                    priority victims, then the first candidate (no PDBs).
 * The pod must carry no topology / port / image uses (KSIM_E_UNSUPPORTED). */
int ksim_preempt(ksim_handle* h, const ksim_pod_set* pods, int32_t pod_index, int32_t priority,
                 ksim_preempt_out* out);
/* ksim_preempt with the PodNominator's pods (replaces the same PostFilter;
 * upstream SelectVictimsOnNode filters through RunFilterPluginsWithNominatedPods,
 * framework.go:764-800 v1.26).  Group k = the pods [first[k], first[k] +
 * count[k]) of `nominated`, nominated on node nodes[k] with priority >=
 * `priority`, the preemptor excluded (the caller selects them, as for
 * ksim_fw_filter_nominated; nodes distinct).  A grouped node's status is the
 * two-pass one (pass 1 with the group's pods added; pass 2 as is only if pass
 * 1 passed) and its dry run keeps the group's requests and pod count on the
 * node.  n_groups = 0 is ksim_preempt. */
int ksim_preempt_nominated(ksim_handle* h, const ksim_pod_set* pods, int32_t pod_index, int32_t priority,
                           const ksim_pod_set* nominated, int32_t n_groups, const int32_t* nodes,
                           const int32_t* first, const int32_t* count, ksim_preempt_out* out);

/* ---- selector / affinity-term matching -------------------- */
/* The pod-matching half of PodTopologySpread's and InterPodAffinity's
 * PreFilter / PreScore: upstream countPodsMatchSelector,
 * getExistingAntiAffinityCounts, getIncomingAffinityAntiAffinityCounts and
 * processExistingPod run every selector / term against every existing pod,
 * reached per pod through the wrapped plugins' PreFilter / PreScore
 * (scheduler/plugin/wrappedplugin.go:427-486).  The engine keeps the answers
 * as count classes (ksim_node_table.class_count); this call computes them.
 *
 * The host reduces each matcher to requirements over a feature vocabulary
 * (a namespace, a label key=value pair, a label key): In / Exists name the
 * features that satisfy them, NotIn / DoesNotExist (neg = 1) the features
 * that break them; a namespace predicate is an In over namespaces; a nil
 * selector is a positive requirement naming no feature.  A signature is the
 * feature set of a (namespace, labels) pair.  On the device:
 *   hits[s][r]  = |features(s) & features(r)|   (int8 MFMA contraction)
 *   match[s][m] = AND over r in m of (hits > 0) != neg[r]
 *   counts[c][node] = #{bound pods p on node : match[sig(p)][class_matcher[c]]}
 * Limits: n_reqs <= 4096, n_feat <= 65536 (KSIM_E_UNSUPPORTED beyond). */
typedef struct ksim_match_problem {
  int32_t n_sigs, n_feat, n_reqs, n_matchers;
  const int32_t* sig_feat_off;     /* [n_sigs + 1] CSR over sig_feat */
  const int32_t* sig_feat;         /* feature ids < n_feat */
  const int32_t* req_feat_off;     /* [n_reqs + 1] CSR over req_feat */
  const int32_t* req_feat;
  const uint8_t* req_neg;          /* [n_reqs] */
  const int32_t* m_req_off;        /* [n_matchers + 1] CSR over m_req (requirement ids, AND) */
  const int32_t* m_req;
  int32_t n_pods, n_nodes, n_classes, _pad;
  const int32_t* pod_sig;          /* [n_pods] signature of each bound pod */
  const int32_t* pod_node;         /* [n_pods] its node position */
  const int32_t* class_matcher;    /* [n_classes] matcher of each output class */
} ksim_match_problem;

/* match_bits: [n_sigs][ceil(n_matchers / 32)] (bit m of row s: signature s
 * matches matcher m); counts (may be NULL when n_classes == 0):
 * [n_classes][n_nodes].  Needs no cluster or profile on the handle. */
int ksim_match_terms(ksim_handle* h, const ksim_match_problem* mp, uint32_t* match_bits, int32_t* counts);

/* ---- result emission ------------------------------------- */
/* One cycle's outputs (ksim_eval_out or the oracle's) plus the names the
 * annotations use.  messages[msg_id[i]] is the failure reason of node i when
 * fail_plugin[i] is a filter index (the host builds the few distinct reasons,
 * e.g. ksim/wrapped.py filter_message). */
typedef struct ksim_emit_input {
  int32_t n_nodes, n_filter, n_score, n_messages;
  const char* const* node_names;       /* [n_nodes] nodeTree order */
  const char* const* filter_names;     /* [n_filter] profile order, original plugin names */
  const char* const* score_names;      /* [n_score] profile order, original plugin names */
  const int32_t* score_weight;         /* [n_score] the store's scorePluginWeight (registry default) */
  const uint8_t* has_normalize;        /* [n_score] plugin has a NormalizeScore extension */
  const uint8_t* fail_plugin;          /* [n_nodes] KSIM_PASSED / KSIM_NOT_EVALUATED / filter index */
  const int32_t* msg_id;               /* [n_nodes] index into messages (failed nodes) */
  const char* const* messages;         /* [n_messages] */
  const uint8_t* scored;               /* [n_nodes] */
  const int64_t* raw;                  /* [n_score][n_nodes] */
  const int64_t* norm;                 /* [n_score][n_nodes] */
} ksim_emit_input;

/* The filter-result, score-result and finalscore-result annotation values
 * (annotation.go:3-30) of the cycle, exactly as resultstore.AddStoredResultToPod
 * encodes the maps the wrapped plugins fill (store.go:129-190, 418-502): Go
 * encoding/json text, NUL-terminated, into the three caller buffers.  lens[3]
 * receives the lengths; a buffer smaller than its length + 1 gets nothing
 * and the call returns KSIM_E_INVALID (retry with lens[k] + 1 bytes).  Host
 * code only: no device, no handle. */
int ksim_emit_cycle_json(const ksim_emit_input* in, char* filter_json, int64_t filter_cap, char* score_json,
                         int64_t score_cap, char* final_json, int64_t final_cap, int64_t* lens);

/* ---- native snapshot encoder (ABI 10; SURVEY §2.3 "Host snapshot encoder") ----
 * Replaces the host compile a simulator host runs before the engine sees a
 * snapshot: v1.Node / v1.Pod objects -> ksim_node_table / ksim_vocab (nodeTree
 * order, NodeInfo aggregates of the bound pods, taint and label vocabularies)
 * and the pending queue -> ksim_pod_set (request sums, toleration bitsets,
 * compiled node-selector terms, PodTopologySpread / InterPodAffinity count
 * classes, NodePorts / ImageLocality classes, NetworkBandwidth quantities).
 * It is the restatement of ksim/encode.py + ksim/topology.py in C++ and its
 * outputs are byte-equal to theirs (tests/test_native_encode.py).  Host code
 * only: no device, no engine handle.
 *
 * The reference hands the plugins these objects through the scheduler cache
 * (simulator/scheduler/plugin/plugins.go:75-87 builds the plugins the engine
 * replaces; integration/go/engine/plugins.go implements its Encoder over this
 * API).  Input objects live in one flat pool: every string is an id into one
 * string table, every list a (first, count) range into a typed array of the
 * pool.  A Go caller builds the pool from v1 objects with no Go pointer inside
 * C memory (cgo rule): one byte blob, offsets and arrays of plain structs.
 * Where nil and empty differ in Kubernetes (label selectors, nodeAffinity
 * required terms) first = -1 (or id -1) is nil. */
typedef struct ksim_k8s_kv {              /* map entry: labels, annotations, resource lists */
  int32_t key, value;                     /* string ids; resource lists carry Quantity strings */
} ksim_k8s_kv;

typedef struct ksim_k8s_taint {
  int32_t key, value, effect;             /* string ids */
} ksim_k8s_taint;

typedef struct ksim_k8s_toleration {
  int32_t key, op, value, effect;         /* string ids; op "" = Equal */
} ksim_k8s_toleration;

typedef struct ksim_k8s_requirement {     /* NodeSelectorRequirement / LabelSelectorRequirement */
  int32_t key, op;                        /* string ids */
  int32_t values_first, values_count;     /* range of ksim_k8s_pool.str_list */
} ksim_k8s_requirement;

typedef struct ksim_k8s_selector_term {   /* NodeSelectorTerm */
  int32_t exprs_first, exprs_count;       /* matchExpressions: ksim_k8s_pool.reqs */
  int32_t fields_first, fields_count;     /* matchFields: ksim_k8s_pool.reqs */
} ksim_k8s_selector_term;

typedef struct ksim_k8s_preferred_term {  /* PreferredSchedulingTerm */
  int32_t weight, term;                   /* term: index into ksim_k8s_pool.terms */
} ksim_k8s_preferred_term;

typedef struct ksim_k8s_label_selector {  /* metav1.LabelSelector */
  int32_t labels_first, labels_count;     /* matchLabels: ksim_k8s_pool.kv */
  int32_t exprs_first, exprs_count;       /* matchExpressions: ksim_k8s_pool.reqs */
} ksim_k8s_label_selector;

typedef struct ksim_k8s_pod_term {        /* PodAffinityTerm (weight: WeightedPodAffinityTerm) */
  int32_t topology_key;                   /* string id */
  int32_t selector;                       /* ksim_k8s_pool.selectors index, -1 = nil */
  int32_t ns_first, ns_count;             /* namespaces: ksim_k8s_pool.str_list */
  int32_t ns_selector;                    /* namespaceSelector, -1 = nil */
  int32_t weight;
} ksim_k8s_pod_term;

typedef struct ksim_k8s_spread {          /* TopologySpreadConstraint */
  int32_t max_skew;
  int32_t topology_key, when_unsatisfiable;   /* string ids */
  int32_t selector;                       /* -1 = nil */
  int32_t node_affinity_policy;           /* string id, -1 = nil (Honor) */
  int32_t node_taints_policy;             /* string id, -1 = nil (Ignore) */
} ksim_k8s_spread;

typedef struct ksim_k8s_port {            /* ContainerPort: hostPort 0 = none */
  int32_t host_port, protocol, host_ip;   /* protocol / host_ip: string ids ("" = TCP / 0.0.0.0) */
} ksim_k8s_port;

typedef struct ksim_k8s_container {
  int32_t requests_first, requests_count; /* resources.requests: ksim_k8s_pool.kv */
  int32_t ports_first, ports_count;
  int32_t image;                          /* string id */
} ksim_k8s_container;

typedef struct ksim_k8s_image {           /* node status.images entry */
  int32_t names_first, names_count;       /* ksim_k8s_pool.str_list */
  int64_t size_bytes;
} ksim_k8s_image;

typedef struct ksim_k8s_volume_group {    /* one VolumeBinding / VolumeZone group (see "volume groups") */
  int32_t terms_first, terms_count;       /* ksim_k8s_pool.terms; match_fields ops "__true__" /
                                             "__false__" are decided by the host's binder */
} ksim_k8s_volume_group;

typedef struct ksim_k8s_node {
  int32_t name, unschedulable;
  int32_t labels_first, labels_count;
  int32_t taints_first, taints_count;
  int32_t alloc_first, alloc_count;       /* status.allocatable: kv of Quantity strings */
  int32_t annotations_first, annotations_count;
  int32_t images_first, images_count;
} ksim_k8s_node;

#define KSIM_K8S_VOLUMES_NONE   0         /* no persistentVolumeClaim volume */
#define KSIM_K8S_VOLUMES_REFUSE 1         /* a volume the engine does not model (KSIM_POD_HAS_VOLUMES) */
#define KSIM_K8S_VOLUMES_GROUPS 2         /* claims compiled by the host's binder into groups */

typedef struct ksim_k8s_pod {
  int32_t name, namespace_;
  int32_t labels_first, labels_count;
  int32_t annotations_first, annotations_count;
  int32_t containers_first, containers_count;
  int32_t init_first, init_count;         /* initContainers */
  int32_t overhead_first, overhead_count; /* kv */
  int32_t selector_first, selector_count; /* spec.nodeSelector: kv */
  int32_t required_first, required_count; /* nodeAffinity required terms; first = -1: nil */
  int32_t preferred_first, preferred_count;
  int32_t tolerations_first, tolerations_count;
  int32_t spread_first, spread_count;
  int32_t aff_req_first, aff_req_count;   /* podAffinity required: ksim_k8s_pool.pod_terms */
  int32_t aff_pref_first, aff_pref_count; /* podAffinity preferred (weighted) */
  int32_t anti_req_first, anti_req_count; /* podAntiAffinity required */
  int32_t anti_pref_first, anti_pref_count;
  int32_t node_name;                      /* string id ("" = unbound) */
  int32_t owner_api_version, owner_kind, owner_name;   /* controller ownerReference; -1 = none */
  int32_t volumes;                        /* KSIM_K8S_VOLUMES_* */
  int32_t vb_first, vb_count, vb_bound;   /* VolumeBinding groups; the first vb_bound are bound PVs */
  int32_t vz_first, vz_count;             /* VolumeZone groups */
  int32_t _pad;
} ksim_k8s_pod;

typedef struct ksim_k8s_namespace {
  int32_t name, labels_first, labels_count, _pad;
} ksim_k8s_namespace;

typedef struct ksim_k8s_service {         /* v1.Service: spec.selector (first = -1: nil) */
  int32_t namespace_, selector_first, selector_count, _pad;
} ksim_k8s_service;

typedef struct ksim_k8s_controller {      /* ReplicationController / ReplicaSet / StatefulSet */
  int32_t kind, namespace_, name;         /* string ids */
  int32_t rc_selector_first, rc_selector_count;   /* ReplicationController spec.selector (kv, -1: nil) */
  int32_t selector;                       /* ReplicaSet / StatefulSet spec.selector (-1: nil) */
} ksim_k8s_controller;

typedef struct ksim_k8s_pool {
  const char* strings;                    /* string i = strings[str_off[i] .. str_off[i+1]) */
  const int64_t* str_off;                 /* [n_strings + 1] */
  int64_t n_strings;
  const int32_t* str_list;   int64_t n_str_list;   /* string-id lists */
  const ksim_k8s_kv* kv;     int64_t n_kv;
  const ksim_k8s_taint* taints;           int64_t n_taints;
  const ksim_k8s_toleration* tolerations; int64_t n_tolerations;
  const ksim_k8s_requirement* reqs;       int64_t n_reqs;
  const ksim_k8s_selector_term* terms;    int64_t n_terms;
  const ksim_k8s_preferred_term* preferred; int64_t n_preferred;
  const ksim_k8s_label_selector* selectors; int64_t n_selectors;
  const ksim_k8s_pod_term* pod_terms;     int64_t n_pod_terms;
  const ksim_k8s_spread* spread;          int64_t n_spread;
  const ksim_k8s_port* ports;             int64_t n_ports;
  const ksim_k8s_container* containers;   int64_t n_containers;
  const ksim_k8s_image* images;           int64_t n_images;
  const ksim_k8s_volume_group* volume_groups; int64_t n_volume_groups;
  const ksim_k8s_node* nodes;             int64_t n_nodes;
  const ksim_k8s_pod* pods;               int64_t n_pods;
  const ksim_k8s_namespace* namespaces;   int64_t n_namespaces;
  const ksim_k8s_service* services;       int64_t n_services;
  const ksim_k8s_controller* controllers; int64_t n_controllers;
} ksim_k8s_pool;

typedef struct ksim_encode_nodes_opts {
  /* NetworkBandwidthArgs annotation names (string ids of the pool; -1 = the
     plugin's default, networkbandwidth/plugin.go:200-204) */
  int32_t nb_node_limit, nb_ingress_request, nb_egress_request;
  int32_t keep_previous;                  /* 1: the previous snapshot's scalar columns first and its
                                             count classes registered first, with their ids (the
                                             scheduler cache after node deltas, ksim/ingest.py NodeCache) */
  int32_t extra_scalar_first, extra_scalar_count;  /* str_list: scalar columns no node offers yet */
} ksim_encode_nodes_opts;

#define KSIM_SPREAD_DEFAULTS_NONE   0     /* no profile defaults: only the pods' own constraints */
#define KSIM_SPREAD_DEFAULTS_SYSTEM 1     /* PodTopologySpreadArgs defaultingType System */
#define KSIM_SPREAD_DEFAULTS_LIST   2     /* defaultingType List: spread_first/count */

typedef struct ksim_encode_pods_opts {
  /* NodeAffinityArgs.addedAffinity: required terms (first = -1: nil) and preferred terms */
  int32_t added_required_first, added_required_count;
  int32_t added_preferred_first, added_preferred_count;
  /* PodTopologySpreadArgs: the defaults a pod without constraints takes, with
     the selector helper.DefaultSelector builds from the pool's services and
     controllers */
  int32_t spread_defaults;                /* KSIM_SPREAD_DEFAULTS_* */
  int32_t spread_first, spread_count;     /* List defaults (ksim_k8s_pool.spread) */
  int32_t _pad;
} ksim_encode_pods_opts;

typedef struct ksim_encoder ksim_encoder;

typedef struct ksim_encoder_info {
  int32_t n_nodes, n_scalar, n_label_cols, n_taints;
  int32_t n_classes, n_pods, n_exprs, n_terms;
  int32_t n_uses, n_adds, n_nn, n_members;   /* n_members: bound pods in the snapshot (ABI 11) */
} ksim_encoder_info;

int  ksim_encoder_create(ksim_encoder** out);
void ksim_encoder_destroy(ksim_encoder* e);
const char* ksim_encoder_last_error(const ksim_encoder* e);
/* A snapshot: pool.nodes (any order; encoded in nodeTree order) and pool.pods,
 * the pods already bound (spec.nodeName; a pod naming no node of the pool is
 * skipped), pool.namespaces for namespaceSelector terms.  Replaces the
 * encoder's snapshot; label columns start empty. */
int ksim_encode_nodes(ksim_encoder* e, const ksim_k8s_pool* pool, const ksim_encode_nodes_opts* opts);
/* The queue pool.pods against the current snapshot: label columns and count
 * classes the pods reference are added to the snapshot (the node table's
 * labels / class_count change), the pod set is replaced. */
int ksim_encode_pods(ksim_encoder* e, const ksim_k8s_pool* pool, const ksim_encode_pods_opts* opts);
/* Views of the encoder's buffers, valid until its next encode call. */
int ksim_encoder_cluster(const ksim_encoder* e, ksim_node_table* nodes, ksim_vocab* vocab);
int ksim_encoder_pods(const ksim_encoder* e, ksim_pod_set* pods);
int ksim_encoder_get_info(const ksim_encoder* e, ksim_encoder_info* out);
/* order[position] = index into the snapshot pool's nodes */
int ksim_encoder_node_order(const ksim_encoder* e, int32_t* order);
/* Host metadata (strings never cross to the device): what = KSIM_ENC_STR_*,
 * i / j as listed; NULL when out of range.  Valid until the next encode call. */
#define KSIM_ENC_STR_LABEL_KEY    0       /* i: label column */
#define KSIM_ENC_STR_LABEL_VALUE  1       /* i: label column, j: value id */
#define KSIM_ENC_STR_SCALAR       2       /* i: scalar column */
#define KSIM_ENC_STR_TAINT_KEY    3       /* i: taint vocabulary id (>= 1) */
#define KSIM_ENC_STR_TAINT_VALUE  4
#define KSIM_ENC_STR_TAINT_EFFECT 5
#define KSIM_ENC_STR_NODE_NAME    6       /* i: node position */
const char* ksim_encoder_string(const ksim_encoder* e, int32_t what, int32_t i, int32_t j);

/* ---- snapshot deltas (ABI 11) ----------------------------------------------------
 * The scheduler cache between two snapshots, without re-encoding the cluster:
 * the simulator's scheduler runs off informers
 * (simulator/scheduler/scheduler.go:160-167) and upstream's UpdateSnapshot
 * copies only the NodeInfos whose generation moved.  The host diffs the
 * framework's snapshot by NodeInfo generation (integration/go/engine/
 * encoder.go NativeEncoder.Snapshot, ksim/fwsnapshot.py SnapshotSync) and
 * feeds the changes here and to the engine:
 *
 *   a node added / updated / removed   ksim_encoder_update_nodes, then
 *                                      ksim_encoder_cluster + ksim_encoder_old_pos
 *                                      into ksim_upsert_nodes (the engine replays
 *                                      its binds on the kept nodes);
 *   a bound pod added (an informer     ksim_encode_pods of the pod, the table
 *   event, or the framework's Reserve) re-sent if the compile added label
 *                                      columns or count classes (ksim_upsert_nodes
 *                                      with every node kept), ksim_assume,
 *                                      ksim_encoder_bind;
 *   a bound pod deleted / Unreserve    ksim_encode_pods of the pod (same re-send
 *                                      rule), ksim_forget, ksim_encoder_unbind.
 *
 * The encoder keeps the snapshot's node rows and class rows as the engine last
 * received them (the rows ksim_upsert_nodes replays onto) and the membership
 * of every bound pod (its signature and host ports per node), so a count class
 * a later pod registers counts every pod bound so far.  Re-send a grown table
 * before the next ksim_assume / ksim_forget, so that a new class row reaches
 * the engine before any bind it does not count.
 *
 * ksim_encoder_update_nodes: pool.nodes are added (new name) or updated
 * (known name) nodes, removed[0..n_removed) string ids of the pool naming the
 * nodes that leave (their bound pods leave the snapshot).  Nodes keep informer
 * add order; an update that changes a node's zone re-adds it at the end
 * (nodeTree.updateNode).  Scalar columns, taint ids, label columns and count
 * class ids are kept; the pod set is cleared (its positions are stale).
 * ksim_encoder_old_pos: old_pos[i] = the previous position of node i of the
 * new snapshot, -1 for an added node (KSIM_E_INVALID before any delta).
 * Updates that move no node and add no vocabulary are applied in place
 * (ksim_encoder_changed_rows, then ksim_update_node_rows on the engine).
 * ksim_encoder_bind: pod `pod_index` of the current pod set (the last
 * ksim_encode_pods) is bound at node position `node`, under its
 * namespace / name; binding a pod already bound is KSIM_E_INVALID.
 * ksim_encoder_unbind: the bound pod namespace/name leaves (its position in
 * *node); KSIM_E_INVALID when it is not bound.
 * ksim_encoder_bound_node: the pod's position, or -1 when not bound. */
int ksim_encoder_update_nodes(ksim_encoder* e, const ksim_k8s_pool* pool, const int32_t* removed,
                              int32_t n_removed);
int ksim_encoder_old_pos(const ksim_encoder* e, int32_t* old_pos);
/* The last ksim_encoder_update_nodes, when it only updated nodes in place
 * (no node added, removed or moved to another zone; no new scalar column,
 * taint or label value; images unchanged): the number of updated positions,
 * written to rows[0..min(count, cap)); the table then differs from the
 * previous one only in those rows' static columns (ksim_update_node_rows).
 * -1 when the delta needs ksim_upsert_nodes with ksim_encoder_old_pos. */
int ksim_encoder_changed_rows(const ksim_encoder* e, int32_t* rows, int32_t cap);
int ksim_encoder_bind(ksim_encoder* e, int32_t pod_index, int32_t node);
int ksim_encoder_unbind(ksim_encoder* e, const char* namespace_, const char* name, int32_t* node);
int ksim_encoder_bound_node(const ksim_encoder* e, const char* namespace_, const char* name, int32_t* node);

#ifdef __cplusplus
}
#endif
#endif /* KSIM_ENGINE_H */
