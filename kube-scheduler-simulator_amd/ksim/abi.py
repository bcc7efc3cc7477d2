"""ctypes / numpy mirror of include/ksim_engine.h (the C-ABI boundary).

The structs are the ones a cgo package would pass across the boundary
(SURVEY.md §8(b)); tests check every size against ``ksim_abi_sizeof``.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

ABI_VERSION = 11

MAX_NODES = (1 << 18) - 1
MAX_NODE_TAINTS = 8
TAINT_WORDS = 4
MAX_SCALAR = 8
MAX_LABEL_COLS = 256
EXPR_VALS = 6
MAX_FILTER = 16
MAX_SCORE = 8
MAX_RES = 4
MAX_SHAPE = 16
MAX_USES = 16
MAX_CLASSES = 4096
COL_NONE = 0xFFFF

OK = 0
E_INVALID = -1
E_DEVICE = -2
E_OOM = -3
E_RCCL = -4
E_UNSUPPORTED = -5

# plugin ids (enum ksim_plugin); names are the upstream in-tree plugin names
PLUGINS = [
    "NodeUnschedulable",
    "NodeName",
    "TaintToleration",
    "NodeAffinity",
    "NodePorts",
    "NodeResourcesFit",
    "VolumeRestrictions",
    "EBSLimits",
    "GCEPDLimits",
    "NodeVolumeLimits",
    "AzureDiskLimits",
    "VolumeBinding",
    "VolumeZone",
    "PodTopologySpread",
    "InterPodAffinity",
    "NodeResourcesBalancedAllocation",
    "ImageLocality",
    "NetworkBandwidth",
]
PLUGIN_ID = {n: i for i, n in enumerate(PLUGINS)}
PL_NODE_UNSCHEDULABLE = 0
PL_NODE_NAME = 1
PL_TAINT_TOLERATION = 2
PL_NODE_AFFINITY = 3
PL_NODE_PORTS = 4
PL_NODE_RESOURCES_FIT = 5
PL_POD_TOPOLOGY_SPREAD = 13
PL_INTER_POD_AFFINITY = 14
PL_BALANCED_ALLOCATION = 15
PL_IMAGE_LOCALITY = 16
PL_NETWORK_BANDWIDTH = 17

EFFECT_NONE = 0
EFFECT_NO_SCHEDULE = 1
EFFECT_PREFER_NO_SCHEDULE = 2
EFFECT_NO_EXECUTE = 3
EFFECT_ID = {"": EFFECT_NONE, "NoSchedule": EFFECT_NO_SCHEDULE,
             "PreferNoSchedule": EFFECT_PREFER_NO_SCHEDULE, "NoExecute": EFFECT_NO_EXECUTE}

RES_CPU = 0
RES_MEMORY = 1
RES_EPHEMERAL = 2
RES_SCALAR0 = 3

NODE_UNSCHEDULABLE = 1
NODE_NB_LIMIT = 2
NODE_NB_LIMIT_BAD = 4

POD_TOLERATES_UNSCHEDULABLE = 1
POD_HAS_REQUIRED_AFFINITY = 2
POD_HAS_SCALAR = 4
POD_HAS_HOST_PORTS = 8
POD_HAS_VOLUMES = 16
POD_NODE_NAMES = 32            # NodeAffinity PreFilterResult restricts the scan (nn_first, nn_count)
POD_NODE_NAMES_UNKNOWN = 64    # ... and names a node the snapshot lacks: the cycle errors
POD_ADDED_AFFINITY = 128       # NodeAffinityArgs.addedAffinity required terms (added_term_first, added_term_count)

# pod nb_flags
POD_NB_INGRESS_BAD = 1
POD_NB_EGRESS_BAD = 2

# pod topo_flags
POD_IPA_SELF_AFFINITY = 1
POD_PTS_SYSTEM_DEFAULT = 2     # system-defaulted spread constraints: PreScore's requireAllTopologies = false

# topology uses (ksim_topo_use.kind)
USE_PTS_HARD = 0
USE_PTS_SOFT = 1
USE_IPA_EXISTING_ANTI = 2
USE_IPA_AFFINITY = 3
USE_IPA_ANTI = 4
USE_IPA_SCORE = 5
USE_IPA_SCORE_HARD = 6
USE_NODE_PORT = 7
USE_IMAGE = 8
USEF_SELF_MATCH = 1
USEF_HONOR_AFFINITY = 2
USEF_HONOR_TAINTS = 4
USEF_HOSTNAME = 8

# PodTopologySpread / InterPodAffinity filter failure details
PTS_MISSING_LABEL = 1
PTS_SKEW = 2
IPA_AFFINITY = 1
IPA_ANTI_AFFINITY = 2
IPA_EXISTING_ANTI = 3
NA_ENFORCED = 1                # NodeAffinity failed the scheduler-enforced addedAffinity
VB_NODE_CONFLICT = 1           # VolumeBinding detail: a bound PV's node affinity
VB_BIND_CONFLICT = 2           # VolumeBinding detail: an unbound claim found no PV / provisioning
VB_UNBOUND_GROUP = 1 << 30     # group-index flag of an unbound-claim VolumeBinding group

# NodeResourcesFit scoring strategies
FIT_LEAST_ALLOCATED = 0
FIT_MOST_ALLOCATED = 1
FIT_REQUESTED_TO_CAPACITY_RATIO = 2
FIT_STRATEGY_ID = {"LeastAllocated": FIT_LEAST_ALLOCATED, "MostAllocated": FIT_MOST_ALLOCATED,
                   "RequestedToCapacityRatio": FIT_REQUESTED_TO_CAPACITY_RATIO}

OP_IN = 0
OP_NOT_IN = 1
OP_EXISTS = 2
OP_DOES_NOT_EXIST = 3
OP_GT = 4
OP_LT = 5
OP_FIELD_IN = 6
OP_FIELD_NOT_IN = 7
OP_FALSE = 8
OP_TRUE = 9

PASSED = 0xFF
NOT_EVALUATED = 0xFE
FAIL_EXTENDER = 0xFD

FIT_TOO_MANY_PODS = 1
FIT_CPU = 2
FIT_MEMORY = 4
FIT_EPHEMERAL = 8
FIT_SCALAR0 = 16

STATUS_SCHEDULED = 0
STATUS_UNSCHEDULABLE = 1
STATUS_ERROR = 2
CHOSEN_ERROR = -2

# NetworkBandwidth fail details
NB_INSUFFICIENT = 1
NB_NO_LIMIT = 2
NB_LIMIT_BAD = 3
NB_INGRESS_BAD = 4
NB_EGRESS_BAD = 5
NB_NO_REQUEST = 6

# ---- numpy dtypes (align=True reproduces the C layout) -------------------
LABEL_EXPR_DTYPE = np.dtype(
    [("num", "<i8"), ("vals", "<u4", (EXPR_VALS,)), ("col", "<u2"), ("op", "u1"),
     ("nvals", "u1"), ("_pad", "<u4")], align=True)
TERM_DTYPE = np.dtype(
    [("first_expr", "<i4"), ("n_expr", "<i4"), ("weight", "<i4"), ("_pad", "<i4")], align=True)
POD_DTYPE = np.dtype(
    [("req_cpu", "<i8"), ("req_mem", "<i8"), ("req_eph", "<i8"),
     ("nz_cpu", "<i8"), ("nz_mem", "<i8"),
     ("scalar_req", "<i8", (MAX_SCALAR,)),
     ("tol_filter", "<u8", (TAINT_WORDS,)), ("tol_prefer", "<u8", (TAINT_WORDS,)),
     ("node_name", "<i4"), ("flags", "<u4"),
     ("sel_first", "<i4"), ("sel_count", "<i4"),
     ("req_term_first", "<i4"), ("req_term_count", "<i4"),
     ("pref_term_first", "<i4"), ("pref_term_count", "<i4"),
     ("use_first", "<i4"), ("use_count", "<i4"), ("add_first", "<i4"), ("add_count", "<i4"),
     ("topo_flags", "<u4"), ("nb_flags", "<u4"), ("nn_first", "<i4"), ("nn_count", "<i4"),
     ("vb_first", "<i4"), ("vb_count", "<i4"), ("vz_first", "<i4"), ("vz_count", "<i4"),
     ("nb_req", "<i8"), ("nb_add", "<i8"), ("added_term_first", "<i4"), ("added_term_count", "<i4")],
    align=True)
TOPO_USE_DTYPE = np.dtype(
    [("cls", "<i4"), ("arg", "<i4"), ("col", "<u2"), ("kind", "u1"), ("flags", "u1"), ("_pad", "<i4")],
    align=True)
CLASS_ADD_DTYPE = np.dtype([("cls", "<i4"), ("count", "<i4")], align=True)


def _p(arr):
    """Pointer to a numpy array's data (None for None / empty)."""
    if arr is None:
        return None
    return ctypes.c_void_p(arr.ctypes.data) if arr.size else None


class NodeTable(ctypes.Structure):
    _fields_ = [
        ("n_nodes", ctypes.c_int32), ("n_scalar", ctypes.c_int32),
        ("n_label_cols", ctypes.c_int32), ("_pad0", ctypes.c_int32),
        ("alloc_cpu", ctypes.c_void_p), ("alloc_mem", ctypes.c_void_p),
        ("alloc_eph", ctypes.c_void_p), ("alloc_pods", ctypes.c_void_p),
        ("alloc_scalar", ctypes.c_void_p),
        ("req_cpu", ctypes.c_void_p), ("req_mem", ctypes.c_void_p),
        ("req_eph", ctypes.c_void_p), ("req_scalar", ctypes.c_void_p),
        ("nz_cpu", ctypes.c_void_p), ("nz_mem", ctypes.c_void_p),
        ("num_pods", ctypes.c_void_p), ("flags", ctypes.c_void_p),
        ("taints", ctypes.c_void_p), ("labels", ctypes.c_void_p),
        ("n_classes", ctypes.c_int32), ("_pad1", ctypes.c_int32),
        ("class_count", ctypes.c_void_p),
        ("nb_limit", ctypes.c_void_p), ("nb_alloc", ctypes.c_void_p),
    ]


class Vocab(ctypes.Structure):
    _fields_ = [
        ("n_taints", ctypes.c_int32), ("n_label_values", ctypes.c_int32),
        ("taint_effect", ctypes.c_void_p), ("label_col_offset", ctypes.c_void_p),
        ("label_num", ctypes.c_void_p), ("label_num_ok", ctypes.c_void_p),
        ("n_topo_log", ctypes.c_int32), ("_pad", ctypes.c_int32),
        ("topo_log", ctypes.c_void_p),
    ]


class PodSet(ctypes.Structure):
    _fields_ = [
        ("n_pods", ctypes.c_int32), ("n_exprs", ctypes.c_int32),
        ("n_terms", ctypes.c_int32), ("_pad", ctypes.c_int32),
        ("pods", ctypes.c_void_p), ("exprs", ctypes.c_void_p), ("terms", ctypes.c_void_p),
        ("n_uses", ctypes.c_int32), ("n_adds", ctypes.c_int32),
        ("uses", ctypes.c_void_p), ("adds", ctypes.c_void_p),
        ("n_nn", ctypes.c_int32), ("_pad2", ctypes.c_int32), ("nn", ctypes.c_void_p),
    ]


class Profile(ctypes.Structure):
    _fields_ = [
        ("n_filter", ctypes.c_int32), ("n_score", ctypes.c_int32),
        ("filter", ctypes.c_uint8 * MAX_FILTER), ("score", ctypes.c_uint8 * MAX_SCORE),
        ("score_weight", ctypes.c_int32 * MAX_SCORE),
        ("percentage_of_nodes_to_score", ctypes.c_int32),
        ("fit_n_res", ctypes.c_int32), ("fit_res", ctypes.c_int32 * MAX_RES),
        ("fit_res_weight", ctypes.c_int64 * MAX_RES),
        ("ba_n_res", ctypes.c_int32), ("ba_res", ctypes.c_int32 * MAX_RES),
        ("ba_res_weight", ctypes.c_int64 * MAX_RES),
        ("hard_pod_affinity_weight", ctypes.c_int32), ("fit_ignored_scalar", ctypes.c_uint32),
        ("tiebreak_seed", ctypes.c_uint64),
        ("fit_strategy", ctypes.c_int32), ("fit_n_shape", ctypes.c_int32),
        ("fit_shape_util", ctypes.c_int32 * MAX_SHAPE), ("fit_shape_score", ctypes.c_int32 * MAX_SHAPE),
        ("preempt_min_pct", ctypes.c_int32), ("preempt_min_abs", ctypes.c_int32),
    ]


class EvalOut(ctypes.Structure):
    _fields_ = [
        ("fail_plugin", ctypes.c_void_p), ("fail_detail", ctypes.c_void_p),
        ("scored", ctypes.c_void_p), ("raw", ctypes.c_void_p), ("norm", ctypes.c_void_p),
        ("total", ctypes.c_void_p),
        ("chosen", ctypes.c_int32), ("status", ctypes.c_int32),
        ("n_feasible", ctypes.c_int32), ("n_evaluated", ctypes.c_int32),
        ("n_processed", ctypes.c_int32), ("k_to_find", ctypes.c_int32),
        ("next_start", ctypes.c_int32), ("_pad", ctypes.c_int32),
    ]


class BatchStats(ctypes.Structure):
    _fields_ = [
        ("pods", ctypes.c_int64), ("scheduled", ctypes.c_int64),
        ("unschedulable", ctypes.c_int64), ("evals", ctypes.c_int64),
        ("device_ms", ctypes.c_double), ("batches", ctypes.c_int64),
        ("truncations", ctypes.c_int64), ("perpod_cycles", ctypes.c_int64),
    ]


class MatchProblem(ctypes.Structure):
    """ksim_match_problem: selectors / terms as requirements over a feature
    vocabulary, signatures as feature sets (ksim/termmatch.py)."""
    _fields_ = [
        ("n_sigs", ctypes.c_int32), ("n_feat", ctypes.c_int32),
        ("n_reqs", ctypes.c_int32), ("n_matchers", ctypes.c_int32),
        ("sig_feat_off", ctypes.c_void_p), ("sig_feat", ctypes.c_void_p),
        ("req_feat_off", ctypes.c_void_p), ("req_feat", ctypes.c_void_p),
        ("req_neg", ctypes.c_void_p), ("m_req_off", ctypes.c_void_p), ("m_req", ctypes.c_void_p),
        ("n_pods", ctypes.c_int32), ("n_nodes", ctypes.c_int32),
        ("n_classes", ctypes.c_int32), ("_pad", ctypes.c_int32),
        ("pod_sig", ctypes.c_void_p), ("pod_node", ctypes.c_void_p), ("class_matcher", ctypes.c_void_p),
    ]


# ---- native snapshot encoder input pool (ksim_k8s_*; ksim/nativeenc.py) ------
def _i32s(*names):
    return np.dtype([(n, "<i4") for n in names], align=True)


K8S_KV_DTYPE = _i32s("key", "value")
K8S_TAINT_DTYPE = _i32s("key", "value", "effect")
K8S_TOLERATION_DTYPE = _i32s("key", "op", "value", "effect")
K8S_REQ_DTYPE = _i32s("key", "op", "values_first", "values_count")
K8S_TERM_DTYPE = _i32s("exprs_first", "exprs_count", "fields_first", "fields_count")
K8S_PREF_DTYPE = _i32s("weight", "term")
K8S_SELECTOR_DTYPE = _i32s("labels_first", "labels_count", "exprs_first", "exprs_count")
K8S_POD_TERM_DTYPE = _i32s("topology_key", "selector", "ns_first", "ns_count", "ns_selector", "weight")
K8S_SPREAD_DTYPE = _i32s("max_skew", "topology_key", "when_unsatisfiable", "selector", "node_affinity_policy",
                         "node_taints_policy")
K8S_PORT_DTYPE = _i32s("host_port", "protocol", "host_ip")
K8S_CONTAINER_DTYPE = _i32s("requests_first", "requests_count", "ports_first", "ports_count", "image")
K8S_IMAGE_DTYPE = np.dtype([("names_first", "<i4"), ("names_count", "<i4"), ("size_bytes", "<i8")], align=True)
K8S_GROUP_DTYPE = _i32s("terms_first", "terms_count")
K8S_NODE_DTYPE = _i32s("name", "unschedulable", "labels_first", "labels_count", "taints_first", "taints_count",
                       "alloc_first", "alloc_count", "annotations_first", "annotations_count", "images_first",
                       "images_count")
K8S_POD_DTYPE = _i32s("name", "namespace", "labels_first", "labels_count", "annotations_first",
                      "annotations_count", "containers_first", "containers_count", "init_first", "init_count",
                      "overhead_first", "overhead_count", "selector_first", "selector_count", "required_first",
                      "required_count", "preferred_first", "preferred_count", "tolerations_first",
                      "tolerations_count", "spread_first", "spread_count", "aff_req_first", "aff_req_count",
                      "aff_pref_first", "aff_pref_count", "anti_req_first", "anti_req_count", "anti_pref_first",
                      "anti_pref_count", "node_name", "owner_api_version", "owner_kind", "owner_name", "volumes",
                      "vb_first", "vb_count", "vb_bound", "vz_first", "vz_count", "_pad")
K8S_NAMESPACE_DTYPE = _i32s("name", "labels_first", "labels_count", "_pad")
K8S_SERVICE_DTYPE = _i32s("namespace", "selector_first", "selector_count", "_pad")
K8S_CONTROLLER_DTYPE = _i32s("kind", "namespace", "name", "rc_selector_first", "rc_selector_count", "selector")
K8S_VOLUMES_NONE = 0
K8S_VOLUMES_REFUSE = 1
K8S_VOLUMES_GROUPS = 2
SPREAD_DEFAULTS_NONE = 0
SPREAD_DEFAULTS_SYSTEM = 1
SPREAD_DEFAULTS_LIST = 2
ENC_STR_LABEL_KEY = 0
ENC_STR_LABEL_VALUE = 1
ENC_STR_SCALAR = 2
ENC_STR_TAINT_KEY = 3
ENC_STR_TAINT_VALUE = 4
ENC_STR_TAINT_EFFECT = 5
ENC_STR_NODE_NAME = 6

# ksim_k8s_pool: (field, element dtype or None for raw pointers) in C order
POOL_ARRAYS = [("str_list", np.dtype("<i4")), ("kv", K8S_KV_DTYPE), ("taints", K8S_TAINT_DTYPE),
               ("tolerations", K8S_TOLERATION_DTYPE), ("reqs", K8S_REQ_DTYPE), ("terms", K8S_TERM_DTYPE),
               ("preferred", K8S_PREF_DTYPE), ("selectors", K8S_SELECTOR_DTYPE), ("pod_terms", K8S_POD_TERM_DTYPE),
               ("spread", K8S_SPREAD_DTYPE), ("ports", K8S_PORT_DTYPE), ("containers", K8S_CONTAINER_DTYPE),
               ("images", K8S_IMAGE_DTYPE), ("volume_groups", K8S_GROUP_DTYPE), ("nodes", K8S_NODE_DTYPE),
               ("pods", K8S_POD_DTYPE), ("namespaces", K8S_NAMESPACE_DTYPE), ("services", K8S_SERVICE_DTYPE),
               ("controllers", K8S_CONTROLLER_DTYPE)]


class K8sPool(ctypes.Structure):
    _fields_ = ([("strings", ctypes.c_void_p), ("str_off", ctypes.c_void_p), ("n_strings", ctypes.c_int64)] +
                [f for name, _ in POOL_ARRAYS for f in ((name, ctypes.c_void_p), ("n_" + name, ctypes.c_int64))])


class EncodeNodesOpts(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("nb_node_limit", "nb_ingress_request", "nb_egress_request",
                                              "keep_previous", "extra_scalar_first", "extra_scalar_count")]


class EncodePodsOpts(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("added_required_first", "added_required_count",
                                              "added_preferred_first", "added_preferred_count", "spread_defaults",
                                              "spread_first", "spread_count", "_pad")]


class EncoderInfo(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("n_nodes", "n_scalar", "n_label_cols", "n_taints", "n_classes",
                                              "n_pods", "n_exprs", "n_terms", "n_uses", "n_adds", "n_nn", "n_members")]


STRUCT_ORDER = [NodeTable, Vocab, LABEL_EXPR_DTYPE, TERM_DTYPE, POD_DTYPE, PodSet, Profile,
                EvalOut, BatchStats, TOPO_USE_DTYPE, CLASS_ADD_DTYPE, MatchProblem,
                K8S_KV_DTYPE, K8S_TAINT_DTYPE, K8S_TOLERATION_DTYPE, K8S_REQ_DTYPE, K8S_TERM_DTYPE,
                K8S_PREF_DTYPE, K8S_SELECTOR_DTYPE, K8S_POD_TERM_DTYPE, K8S_SPREAD_DTYPE, K8S_PORT_DTYPE,
                K8S_CONTAINER_DTYPE, K8S_IMAGE_DTYPE, K8S_GROUP_DTYPE, K8S_NODE_DTYPE, K8S_POD_DTYPE,
                K8S_NAMESPACE_DTYPE, K8S_SERVICE_DTYPE, K8S_CONTROLLER_DTYPE, K8sPool, EncodeNodesOpts,
                EncodePodsOpts, EncoderInfo]


def struct_size(s) -> int:
    return s.itemsize if isinstance(s, np.dtype) else ctypes.sizeof(s)


class EvalBuffers:
    """Caller-owned output arrays for one compat-mode cycle (ksim_eval_out)."""

    def __init__(self, n_nodes: int, n_score: int):
        self.fail_plugin = np.zeros(n_nodes, np.uint8)
        self.fail_detail = np.zeros(n_nodes, np.uint32)
        self.scored = np.zeros(n_nodes, np.uint8)
        self.raw = np.zeros((max(n_score, 1), n_nodes), np.int64)
        self.norm = np.zeros((max(n_score, 1), n_nodes), np.int64)
        self.total = np.zeros(n_nodes, np.int64)
        self.out = EvalOut()
        self.out.fail_plugin = _p(self.fail_plugin)
        self.out.fail_detail = _p(self.fail_detail)
        self.out.scored = _p(self.scored)
        self.out.raw = _p(self.raw)
        self.out.norm = _p(self.norm)
        self.out.total = _p(self.total)

    def result(self) -> dict:
        o = self.out
        return dict(chosen=o.chosen, status=o.status, n_feasible=o.n_feasible,
                    n_evaluated=o.n_evaluated, n_processed=o.n_processed,
                    k_to_find=o.k_to_find, next_start=o.next_start,
                    fail_plugin=self.fail_plugin.copy(), fail_detail=self.fail_detail.copy(),
                    scored=self.scored.copy(), raw=self.raw.copy(), norm=self.norm.copy(),
                    total=self.total.copy())


# ---- PostFilter: DefaultPreemption ----------------------------------------------
PREEMPT_REQ = 3 + MAX_SCALAR


class _BoundPodsC(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("_pad", ctypes.c_int32), ("node", ctypes.c_void_p),
                ("priority", ctypes.c_void_p), ("start_time", ctypes.c_void_p), ("req", ctypes.c_void_p)]


class BoundPods:
    """ksim_bound_pods over numpy arrays (kept alive by this object)."""

    def __init__(self, node, priority, start_time, req):
        self.node = np.ascontiguousarray(node, np.int32)
        self.priority = np.ascontiguousarray(priority, np.int32)
        self.start_time = np.ascontiguousarray(start_time, np.int64)
        self.req = np.ascontiguousarray(np.asarray(req, np.int64).reshape(-1, PREEMPT_REQ))
        self.n = int(self.node.size)
        self.c = _BoundPodsC(self.n, 0, _p(self.node), _p(self.priority), _p(self.start_time), _p(self.req))


class _PreemptOutC(ctypes.Structure):
    _fields_ = [("nominated", ctypes.c_int32), ("n_victims", ctypes.c_int32), ("n_potential", ctypes.c_int32),
                ("n_candidates", ctypes.c_int32), ("victims", ctypes.c_void_p), ("victims_cap", ctypes.c_int32),
                ("_pad", ctypes.c_int32)]


class PreemptOut:
    def __init__(self, cap: int):
        self.victims = np.zeros(max(cap, 1), np.int32)
        self.c = _PreemptOutC(-1, 0, 0, 0, _p(self.victims), int(self.victims.size), 0)

    def result(self) -> tuple:
        n = min(self.c.n_victims, self.c.victims_cap)
        return self.c.nominated, [int(v) for v in self.victims[:n]], self.c.n_potential, self.c.n_candidates


def repo_root() -> str:
    return os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
