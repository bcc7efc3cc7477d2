"""Host snapshot encoder: Node/Pod objects -> the engine's SoA buffers.

Mirrors what [upstream] internal/cache does before each cycle (snapshot in
nodeTree order, NodeInfo aggregates) and what each plugin's PreFilter/PreScore
precomputes per pod (request sums, toleration sets, compiled affinity), so
the device only sees integer ids (SURVEY.md §2.3 "Host snapshot encoder").
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import abi, netbw
from .model import (Node, Pod, Taint, Toleration, quantity_milli_value, quantity_value)
from .topology import TopologyError, TopologyIndex, pod_uses, register_pod_classes, topo_log_table
from .volumes import VolumeUnsupported

LABEL_HOSTNAME = "kubernetes.io/hostname"
LABEL_ZONE = "topology.kubernetes.io/zone"
LABEL_REGION = "topology.kubernetes.io/region"
LABEL_ZONE_BETA = "failure-domain.beta.kubernetes.io/zone"
LABEL_REGION_BETA = "failure-domain.beta.kubernetes.io/region"
TAINT_NODE_UNSCHEDULABLE = "node.kubernetes.io/unschedulable"

DEFAULT_MILLI_CPU_REQUEST = 100                 # schedutil.DefaultMilliCPURequest
DEFAULT_MEMORY_REQUEST = 200 * 1024 * 1024      # schedutil.DefaultMemoryRequest
_NATIVE = ("cpu", "memory", "ephemeral-storage", "pods")


class EncodeError(ValueError):
    pass


def zone_key(labels: Dict[str, str]) -> str:
    """component-helpers node/topology GetZoneKey."""
    zone = labels.get(LABEL_ZONE, labels.get(LABEL_ZONE_BETA, ""))
    region = labels.get(LABEL_REGION, labels.get(LABEL_REGION_BETA, ""))
    if region == "" and zone == "":
        return ""
    return region + ":\x00:" + zone


def node_tree_order(zone_keys: Sequence[str]) -> List[int]:
    """[upstream] internal/cache/node_tree.go nodeTree.list(): round-robin over
    zones (zone insertion order), insertion order inside each zone."""
    zones: List[str] = []
    tree: Dict[str, List[int]] = {}
    for i, z in enumerate(zone_keys):
        if z not in tree:
            zones.append(z)
            tree[z] = []
        tree[z].append(i)
    out: List[int] = []
    idx = 0
    n = len(zone_keys)
    while len(out) < n:
        for z in zones:
            lst = tree[z]
            if idx < len(lst):
                out.append(lst[idx])
        idx += 1
    return out


# ---- pod resource sums ------------------------------------------------------
def _res(requests: Dict[str, str], name: str) -> int:
    q = requests.get(name)
    if q is None:
        return 0
    return quantity_milli_value(q) if name == "cpu" else quantity_value(q)


def pod_requests(pod: Pod) -> Dict[str, int]:
    """computePodResourceRequest ([upstream] noderesources/fit.go) ==
    NodeInfo calculateResource 'res': sum containers, max init, + overhead."""
    names = set()
    for c in pod.containers + pod.init_containers:
        names.update(c.requests)
    names.update(pod.overhead)
    out = {}
    for n in names:
        if n == "pods":
            continue
        v = sum(_res(c.requests, n) for c in pod.containers)
        for ic in pod.init_containers:
            v = max(v, _res(ic.requests, n))
        v += _res(pod.overhead, n)
        out[n] = v
    return out


def _nonzero(requests: Dict[str, str]) -> Tuple[int, int]:
    """schedutil.GetNonzeroRequests."""
    cpu = DEFAULT_MILLI_CPU_REQUEST if "cpu" not in requests else _res(requests, "cpu")
    mem = DEFAULT_MEMORY_REQUEST if "memory" not in requests else _res(requests, "memory")
    return cpu, mem


def pod_nonzero_requests(pod: Pod) -> Tuple[int, int]:
    """NodeInfo calculateResource non0CPU/non0Mem (== the LeastAllocated pod
    request computed with nonZero=true)."""
    cpu = mem = 0
    for c in pod.containers:
        a, b = _nonzero(c.requests)
        cpu += a
        mem += b
    for ic in pod.init_containers:
        a, b = _nonzero(ic.requests)
        cpu = max(cpu, a)
        mem = max(mem, b)
    if "cpu" in pod.overhead:
        cpu += _res(pod.overhead, "cpu")
    if "memory" in pod.overhead:
        mem += _res(pod.overhead, "memory")
    return cpu, mem


# ---- encoded buffers --------------------------------------------------------
@dataclass
class EncodedCluster:
    n_nodes: int
    n_scalar: int
    alloc_cpu: np.ndarray
    alloc_mem: np.ndarray
    alloc_eph: np.ndarray
    alloc_pods: np.ndarray
    alloc_scalar: np.ndarray          # [n_scalar][N]
    req_cpu: np.ndarray
    req_mem: np.ndarray
    req_eph: np.ndarray
    req_scalar: np.ndarray            # [n_scalar][N]
    nz_cpu: np.ndarray
    nz_mem: np.ndarray
    num_pods: np.ndarray
    flags: np.ndarray
    taints: np.ndarray                # [MAX_NODE_TAINTS][N] uint16
    labels: np.ndarray                # [L][N] uint32
    taint_effect: np.ndarray          # [V] uint8
    label_col_offset: np.ndarray      # [L] int32
    label_num: np.ndarray             # int64
    label_num_ok: np.ndarray          # uint8
    # host metadata (strings never cross the boundary)
    node_names: List[str] = field(default_factory=list)
    label_keys: List[str] = field(default_factory=list)
    label_values: List[List[str]] = field(default_factory=list)   # per col: [vid] -> value
    taint_vocab: List[Taint] = field(default_factory=list)        # [tid] (tid 0 = None)
    scalar_names: List[str] = field(default_factory=list)
    # count classes of PodTopologySpread / InterPodAffinity (ksim/topology.py)
    topo: Optional[TopologyIndex] = None
    class_count: Optional[np.ndarray] = None          # [C][N] int32
    topo_log: Optional[np.ndarray] = None             # [N+1] float64
    # NetworkBandwidth (ksim/netbw.py), milli-units
    nb_limit: Optional[np.ndarray] = None             # [N] int64
    nb_alloc: Optional[np.ndarray] = None             # [N] int64
    nb_args: netbw.NetworkBandwidthArgs = field(default_factory=netbw.NetworkBandwidthArgs)
    # node labels (nodeTree order): a label key gets a column only once a pod
    # references it (selector, affinity term, topology key), see label_col
    node_labels: Optional[List[Dict[str, str]]] = None

    def __post_init__(self):
        if self.topo is None:
            self.topo = TopologyIndex(self.n_nodes)
        if self.class_count is None:
            self.class_count = self.topo.class_count_array()
        if self.topo_log is None:
            self.topo_log = topo_log_table(self.n_nodes)
        if self.nb_limit is None:
            self.nb_limit = np.zeros(self.n_nodes, np.int64)
        if self.nb_alloc is None:
            self.nb_alloc = np.zeros(self.n_nodes, np.int64)

    def refresh_classes(self) -> None:
        """Re-materialise class_count after classes were registered."""
        self.class_count = self.topo.class_count_array()

    @property
    def n_label_cols(self) -> int:
        return int(self.labels.shape[0])

    def node_table(self) -> abi.NodeTable:
        t = abi.NodeTable()
        t.n_nodes = self.n_nodes
        t.n_scalar = self.n_scalar
        t.n_label_cols = self.n_label_cols
        for f in ("alloc_cpu", "alloc_mem", "alloc_eph", "alloc_pods", "alloc_scalar",
                  "req_cpu", "req_mem", "req_eph", "req_scalar", "nz_cpu", "nz_mem",
                  "num_pods", "flags", "taints", "labels"):
            setattr(t, f, abi._p(getattr(self, f)))
        t.n_classes = int(self.class_count.shape[0])
        t.class_count = abi._p(self.class_count)
        t.nb_limit = abi._p(self.nb_limit)
        t.nb_alloc = abi._p(self.nb_alloc)
        return t

    def vocab(self) -> abi.Vocab:
        v = abi.Vocab()
        v.n_taints = int(self.taint_effect.size)
        v.n_label_values = int(self.label_num.size)
        v.taint_effect = abi._p(self.taint_effect)
        v.label_col_offset = abi._p(self.label_col_offset)
        v.label_num = abi._p(self.label_num)
        v.label_num_ok = abi._p(self.label_num_ok)
        v.n_topo_log = int(self.topo_log.size)
        v.topo_log = abi._p(self.topo_log)
        return v

    def shard(self, base: int, count: int) -> "EncodedCluster":
        """Nodes [base, base + count) as a shard snapshot: the
        same vocabularies, the node columns sliced.  Positions stay global
        (the engine is told the base by ksim_set_shard)."""
        import copy
        sl = slice(base, base + count)
        c = copy.copy(self)
        c.n_nodes = count
        for f in ("alloc_cpu", "alloc_mem", "alloc_eph", "alloc_pods", "req_cpu", "req_mem", "req_eph",
                  "nz_cpu", "nz_mem", "num_pods", "flags", "nb_limit", "nb_alloc"):
            setattr(c, f, np.ascontiguousarray(getattr(self, f)[sl]))
        for f in ("alloc_scalar", "req_scalar", "taints", "labels", "class_count"):
            setattr(c, f, np.ascontiguousarray(getattr(self, f)[:, sl]))
        c.node_names = self.node_names[sl]
        if self.node_labels is not None:
            c.node_labels = self.node_labels[sl]
        return c

    def label_col(self, key: str) -> int:
        """The key's label column; a key some node carries gets one on first
        use (nodes carry many keys, the engine needs only the referenced ones).
        -1: no node carries the key."""
        if key in self.label_keys:
            return self.label_keys.index(key)
        if self.node_labels is None or not any(key in lb for lb in self.node_labels):
            return -1
        if len(self.label_keys) >= abi.MAX_LABEL_COLS:
            raise EncodeError(f"more than {abi.MAX_LABEL_COLS} referenced label keys")
        values = [""]
        index: Dict[str, int] = {}
        row = np.zeros((1, self.n_nodes), np.uint32)
        for pos, lb in enumerate(self.node_labels):
            v = lb.get(key)
            if v is None:
                continue
            vid = index.get(v)
            if vid is None:
                vid = index[v] = len(values)
                values.append(v)
            row[0, pos] = vid
        # new lists / arrays (never in place: copies of this cluster share them)
        self.label_col_offset = np.append(self.label_col_offset, np.int32(self.label_num.size)).astype(np.int32)
        nums = [_parse_int64(v) if v != "" else None for v in values]
        self.label_num = np.concatenate([self.label_num, np.array([x if x is not None else 0 for x in nums], np.int64)])
        self.label_num_ok = np.concatenate([self.label_num_ok, np.array([x is not None for x in nums], np.uint8)])
        self.labels = np.concatenate([self.labels.reshape(-1, self.n_nodes), row]).astype(np.uint32)
        self.label_keys = self.label_keys + [key]
        self.label_values = self.label_values + [values]
        return len(self.label_keys) - 1

    def value_id(self, col: int, value: str) -> int:
        if col < 0:
            return 0
        try:
            return self.label_values[col].index(value)
        except ValueError:
            return 0

    def copy_state(self) -> "EncodedCluster":
        import copy
        c = copy.copy(self)
        for f in ("req_cpu", "req_mem", "req_eph", "req_scalar", "nz_cpu", "nz_mem", "num_pods",
                  "class_count", "nb_alloc"):
            setattr(c, f, getattr(self, f).copy())
        return c


@dataclass
class EncodedPods:
    pods: np.ndarray                  # POD_DTYPE
    exprs: np.ndarray                 # LABEL_EXPR_DTYPE
    terms: np.ndarray                 # TERM_DTYPE
    names: List[Tuple[str, str]] = field(default_factory=list)   # (namespace, name)
    uses: np.ndarray = field(default_factory=lambda: np.zeros(0, abi.TOPO_USE_DTYPE))
    adds: np.ndarray = field(default_factory=lambda: np.zeros(0, abi.CLASS_ADD_DTYPE))
    nn: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int32))   # PreFilterResult node positions
    # per pod: NodeAffinity's PreFilterResult.NodeNames (sorted names, as the
    # wrapper records them) or None (all nodes); [] = conflicting terms
    prefilter_names: List[Optional[List[str]]] = field(default_factory=list)
    # per pod: a PreFilter rejection (plugin, message) the hosts record instead
    # of Filter (VolumeBinding's UnschedulableAndUnresolvable); [] = none at all
    prefilter_reject: List[Optional[Tuple[str, str]]] = field(default_factory=list)

    def rejection(self, index: int) -> Optional[Tuple[str, str]]:
        return self.prefilter_reject[index] if self.prefilter_reject else None

    @property
    def n_pods(self) -> int:
        return int(self.pods.size)

    def pod_set(self) -> abi.PodSet:
        s = abi.PodSet()
        s.n_pods = int(self.pods.size)
        s.n_exprs = int(self.exprs.size)
        s.n_terms = int(self.terms.size)
        s.pods = abi._p(self.pods)
        s.exprs = abi._p(self.exprs)
        s.terms = abi._p(self.terms)
        s.n_uses = int(self.uses.size)
        s.n_adds = int(self.adds.size)
        s.uses = abi._p(self.uses)
        s.adds = abi._p(self.adds)
        s.n_nn = int(self.nn.size)
        s.nn = abi._p(self.nn)
        return s

    def subset(self, first: int, count: int) -> "EncodedPods":
        return EncodedPods(self.pods[first:first + count].copy(), self.exprs, self.terms,
                           self.names[first:first + count], self.uses, self.adds, self.nn,
                           self.prefilter_names[first:first + count], self.prefilter_reject[first:first + count])

    def subset_indices(self, idx) -> "EncodedPods":
        """The pods at ``idx`` (any order, repeats allowed) sharing this set's tables."""
        idx = [int(i) for i in idx]
        return EncodedPods(self.pods[idx].copy(), self.exprs, self.terms, [self.names[i] for i in idx],
                           self.uses, self.adds, self.nn,
                           [self.prefilter_names[i] for i in idx] if self.prefilter_names else self.prefilter_names,
                           [self.prefilter_reject[i] for i in idx] if self.prefilter_reject else [])


# ---- cluster encoder --------------------------------------------------------
def _parse_int64(s: str) -> Optional[int]:
    """strconv.ParseInt(s, 10, 64)."""
    t = s[1:] if s[:1] in "+-" else s
    if not t or not t.isdigit():
        return None
    v = int(s)
    if v < -(2 ** 63) or v > 2 ** 63 - 1:
        return None
    return v


def encode_cluster(nodes: Sequence[Node], bound_pods: Sequence[Pod] = (),
                   extra_scalar: Sequence[str] = (),
                   namespaces: Optional[Dict[str, Dict[str, str]]] = None,
                   nb_args: Optional[netbw.NetworkBandwidthArgs] = None,
                   scalar_order: Sequence[str] = (), classes_from: Optional[TopologyIndex] = None,
                   matcher=None) -> Tuple[EncodedCluster, List[int]]:
    """Encode nodes in nodeTree order.  Returns (cluster, order) where
    order[position] = index into ``nodes``.  ``bound_pods`` (spec.nodeName set)
    are added to their node's aggregates like NodeInfo.AddPod (and to the
    PodTopologySpread / InterPodAffinity count classes).  ``namespaces`` maps
    namespace name -> labels (for namespaceSelector terms).  ``scalar_order``:
    scalar columns to place first, in this order, and ``classes_from``: a
    snapshot's TopologyIndex whose count classes are registered first (a re-encoded snapshot keeps the columns and
    class ids of the one it replaces, ksim.ingest.NodeCache).  ``matcher``: match the count classes' selectors
    on the device (ksim.termmatch.DeviceMatcher, ksim_match_terms); encode_pods uses it as well."""
    order = node_tree_order([zone_key(n.labels) for n in nodes])
    ns = [nodes[i] for i in order]
    N = len(ns)
    if N > abi.MAX_NODES:
        raise EncodeError("too many nodes")
    # scalar resources: every non-native allocatable / requested name
    scalar: List[str] = list(scalar_order)
    for n in ns:
        for k in n.allocatable:
            if k not in _NATIVE and k not in scalar:
                scalar.append(k)
    for k in extra_scalar:
        if k not in scalar:
            scalar.append(k)
    if len(scalar) > abi.MAX_SCALAR:
        raise EncodeError("too many scalar resources")
    S = len(scalar)
    # label columns are created on first reference (EncodedCluster.label_col)
    keys: List[str] = []
    values: List[List[str]] = []
    labels = np.zeros((0, N), np.uint32)
    offs = np.zeros(0, np.int32)
    nums: List[int] = []
    oks: List[int] = []
    # taints
    tvocab: List[Taint] = [None]  # type: ignore[list-item]
    tindex: Dict[Tuple[str, str, str], int] = {}
    taints = np.zeros((abi.MAX_NODE_TAINTS, N), np.uint16)
    for pos, n in enumerate(ns):
        if len(n.taints) > abi.MAX_NODE_TAINTS:
            raise EncodeError(f"node {n.name}: more than {abi.MAX_NODE_TAINTS} taints")
        for k, t in enumerate(n.taints):
            key = (t.key, t.value, t.effect)
            tid = tindex.get(key)
            if tid is None:
                tid = len(tvocab)
                tvocab.append(Taint(t.key, t.value, t.effect))
                tindex[key] = tid
            taints[k, pos] = tid
    if len(tvocab) > 64 * abi.TAINT_WORDS:
        raise EncodeError("taint vocabulary too large")
    effect = np.array([0] + [abi.EFFECT_ID.get(t.effect, 0) for t in tvocab[1:]], np.uint8)

    def col(name):
        return np.array([_res(n.allocatable, name) for n in ns], np.int64)

    nb_args = nb_args or netbw.NetworkBandwidthArgs()
    flags = np.array([abi.NODE_UNSCHEDULABLE if n.unschedulable else 0 for n in ns], np.uint32)
    nb_limit = np.zeros(N, np.int64)
    try:
        for pos, n in enumerate(ns):
            fl, q = netbw.node_limit(n.annotations, nb_args)
            flags[pos] |= fl
            nb_limit[pos] = q
    except netbw.QuantityError as e:
        raise EncodeError(str(e)) from e

    c = EncodedCluster(
        n_nodes=N, n_scalar=S,
        alloc_cpu=col("cpu"), alloc_mem=col("memory"), alloc_eph=col("ephemeral-storage"),
        alloc_pods=np.array([_res(n.allocatable, "pods") for n in ns], np.int32),
        alloc_scalar=np.array([[_res(n.allocatable, s) for n in ns] for s in scalar], np.int64).reshape(S, N),
        req_cpu=np.zeros(N, np.int64), req_mem=np.zeros(N, np.int64), req_eph=np.zeros(N, np.int64),
        req_scalar=np.zeros((S, N), np.int64),
        nz_cpu=np.zeros(N, np.int64), nz_mem=np.zeros(N, np.int64),
        num_pods=np.zeros(N, np.int32),
        flags=flags,
        taints=taints, labels=labels, taint_effect=effect, label_col_offset=offs,
        label_num=np.array(nums, np.int64), label_num_ok=np.array(oks, np.uint8),
        node_names=[n.name for n in ns], label_keys=keys, label_values=values,
        taint_vocab=tvocab, scalar_names=scalar,
        nb_limit=nb_limit, nb_alloc=np.zeros(N, np.int64), nb_args=nb_args,
        node_labels=[dict(n.labels) for n in ns],
    )
    c.topo = TopologyIndex(N, namespaces)
    pos_of = {name: i for i, name in enumerate(c.node_names)}
    c.topo.set_images(nodes, pos_of)                 # input order = the order nodes were added
    c.topo.matcher = matcher
    c.topo.deferred = matcher is not None
    if classes_from is not None:
        c.topo.preregister(classes_from)
    carried = [c.topo.carried_terms(p) if p.node_name in pos_of else None   # every carried class exists first
               for p in bound_pods]
    for p, ct in zip(bound_pods, carried):
        if p.node_name not in pos_of:
            continue
        c.topo.add_bound(p, pos_of[p.node_name], ct)
        i = pos_of[p.node_name]
        r = pod_requests(p)
        nz = pod_nonzero_requests(p)
        c.req_cpu[i] += r.get("cpu", 0)
        c.req_mem[i] += r.get("memory", 0)
        c.req_eph[i] += r.get("ephemeral-storage", 0)
        for k, s in enumerate(scalar):
            c.req_scalar[k, i] += r.get(s, 0)
        c.nz_cpu[i] += nz[0]
        c.nz_mem[i] += nz[1]
        c.num_pods[i] += 1
        try:
            c.nb_alloc[i] += netbw.pod_allocated(p.annotations, nb_args)
        except netbw.QuantityError as e:
            raise EncodeError(str(e)) from e
    if c.topo.deferred:
        c.topo.resolve()
    c.refresh_classes()
    return c, order


# ---- pod encoder --------------------------------------------------------------
class _PodBuilder:
    def __init__(self, cluster: EncodedCluster):
        self.c = cluster
        self.exprs: List[np.void] = []
        self.terms: List[Tuple[int, int, int]] = []
        self.pos_of = {n: i for i, n in enumerate(cluster.node_names)}

    def _expr(self, col=0, op=abi.OP_FALSE, vals=(), num=0):
        if len(vals) > abi.EXPR_VALS:
            raise EncodeError("requirement has too many values after vocabulary filtering")
        e = np.zeros((), abi.LABEL_EXPR_DTYPE)
        e["col"] = max(col, 0)
        e["op"] = op
        e["nvals"] = len(vals)
        for i, v in enumerate(vals):
            e["vals"][i] = v
        e["num"] = num
        self.exprs.append(e)

    def requirement(self, r) -> None:
        """nodeSelectorRequirementsAsSelector / fields selector, compiled to ids.
        Invalid requirements compile to OP_FALSE (LazyErrorNodeSelector drops
        the term, so it can never match)."""
        c = self.c
        col = c.label_col(r.key)
        op = r.operator
        if op in ("In", "NotIn"):
            if not r.values:
                return self._expr()
            vids = sorted({c.value_id(col, v) for v in r.values} - {0})
            if op == "In":
                return self._expr(col, abi.OP_IN, vids) if vids else self._expr()
            if not vids:
                return self._expr(0, abi.OP_TRUE)
            return self._expr(col, abi.OP_NOT_IN, vids)
        if op in ("Exists", "DoesNotExist"):
            if r.values:
                return self._expr()
            if col < 0:
                # key unknown on every node: Exists never, DoesNotExist always
                return self._expr() if op == "Exists" else self._expr(0, abi.OP_TRUE)
            return self._expr(col, abi.OP_EXISTS if op == "Exists" else abi.OP_DOES_NOT_EXIST)
        if op in ("Gt", "Lt"):
            if len(r.values) != 1:
                return self._expr()
            v = _parse_int64(r.values[0])
            if v is None or col < 0:
                return self._expr()
            return self._expr(col, abi.OP_GT if op == "Gt" else abi.OP_LT, [], v)
        return self._expr()

    def field_requirement(self, r) -> None:
        # nodeSelectorRequirementsAsFieldSelector: metadata.name In/NotIn with
        # exactly one value; anything else is a parse error (term dropped).
        # ksim.volumes hands PV terms over already decided ("__true__" /
        # "__false__": CheckNodeAffinity's node has no name).
        if r.operator in ("__true__", "__false__"):
            return self._expr(0, abi.OP_TRUE) if r.operator == "__true__" else self._expr()
        if r.key != "metadata.name" or r.operator not in ("In", "NotIn") or len(r.values) != 1:
            return self._expr()
        pos = [self.pos_of[r.values[0]]] if r.values[0] in self.pos_of else []
        if r.operator == "In":
            return self._expr(0, abi.OP_FIELD_IN, pos) if pos else self._expr()
        return self._expr(0, abi.OP_FIELD_NOT_IN, pos) if pos else self._expr(0, abi.OP_TRUE)

    def term(self, t, weight=0) -> None:
        first = len(self.exprs)
        for r in t.match_expressions:
            self.requirement(r)
        for r in t.match_fields:
            self.field_requirement(r)
        self.terms.append((first, len(self.exprs) - first, weight))


def prefilter_node_names(pod: Pod) -> Optional[List[str]]:
    """[upstream] nodeaffinity.PreFilter (v1.26) PreFilterResult.NodeNames: over
    the required node-affinity terms, the union of each term's intersection of
    its metadata.name In matchFields.  None: every node (no required terms, or
    a term without such a field); [] : the terms conflict (the plugin returns
    UnschedulableAndUnresolvable "pod affinity terms conflict").  Sorted, as
    sets.String.List() hands them to the result store (store.go:517-530)."""
    if not pod.required_terms:
        return None
    names = None
    for t in pod.required_terms:
        term_names = None
        for r in t.match_fields:
            if r.key == "metadata.name" and r.operator == "In":
                vals = set(r.values)
                term_names = vals if term_names is None else term_names & vals
        if term_names is None:
            return None
        names = set(term_names) if names is None else names | term_names
    return sorted(names)


def _tol_bits(tolerations: Sequence[Toleration], vocab: Sequence[Taint]) -> np.ndarray:
    w = np.zeros(abi.TAINT_WORDS, np.uint64)
    for tid in range(1, len(vocab)):
        if any(t.tolerates(vocab[tid]) for t in tolerations):
            w[tid >> 6] |= np.uint64(1) << np.uint64(tid & 63)
    return w


def encode_pods(cluster: EncodedCluster, pods: Sequence[Pod], volumes=None, added_affinity=None,
                spread=None) -> EncodedPods:
    """Compile pods against the cluster vocabulary (the per-pod PreFilter /
    PreScore precomputation of Fit, TaintToleration and NodeAffinity).
    ``volumes``: a ksim.volumes.VolumeIndex for pods with PersistentVolumeClaims
    (VolumeBinding / VolumeZone groups); without one such pods are flagged
    KSIM_POD_HAS_VOLUMES (the engine refuses them).
    ``added_affinity``: the profile's NodeAffinityArgs (ksim.profile): its
    required terms become every pod's KSIM_POD_ADDED_AFFINITY terms (one shared
    term range), its preferred terms are appended to every pod's own
    (nodeaffinity.Score adds both sums).
    ``spread``: a ksim.topology.SpreadDefaults (the profile's PodTopologySpread
    default constraints and the Services / controllers that select pods)."""
    b = _PodBuilder(cluster)
    added_first = added_count = 0
    added_pref = []
    if added_affinity is not None:
        if added_affinity.required is not None:
            added_first = len(b.terms)
            for t in added_affinity.required:
                b.term(t)
            added_count = len(b.terms) - added_first
        added_pref = [pt for pt in added_affinity.preferred if pt.weight]
    arr = np.zeros(len(pods), abi.POD_DTYPE)
    names = []
    topo = cluster.topo
    topo.deferred = topo.matcher is not None
    try:
        for p in pods:                        # pass 1: every class exists before any adds
            register_pod_classes(topo, p, spread)
    except TopologyError as e:
        raise EncodeError(str(e)) from e
    if topo.deferred:                         # the new classes' counts, the pods' matches (device)
        topo.resolve(pods)
    uses: List[tuple] = []
    adds: List[Tuple[int, int]] = []
    nn: List[int] = []
    pf_names: List[Optional[List[str]]] = []
    pf_reject: Dict[int, Tuple[str, str]] = {}
    for i, p in enumerate(pods):
        r = pod_requests(p)
        nz = pod_nonzero_requests(p)
        rec = arr[i]
        rec["req_cpu"] = r.get("cpu", 0)
        rec["req_mem"] = r.get("memory", 0)
        rec["req_eph"] = r.get("ephemeral-storage", 0)
        rec["nz_cpu"], rec["nz_mem"] = nz
        flags = 0
        scal = [k for k in r if k not in _NATIVE]
        if scal:
            flags |= abi.POD_HAS_SCALAR
        for k in scal:
            if k not in cluster.scalar_names:
                # no node offers it: allocatable 0 everywhere -> needs a column
                raise EncodeError(f"scalar resource {k} unknown to the cluster encoder (pass extra_scalar)")
            rec["scalar_req"][cluster.scalar_names.index(k)] = r[k]
        rec["tol_filter"] = _tol_bits(p.tolerations, cluster.taint_vocab)
        prefer = [t for t in p.tolerations if t.effect in ("", "PreferNoSchedule")]
        rec["tol_prefer"] = _tol_bits(prefer, cluster.taint_vocab)
        if any(t.tolerates(Taint(TAINT_NODE_UNSCHEDULABLE, "", "NoSchedule")) for t in p.tolerations):
            flags |= abi.POD_TOLERATES_UNSCHEDULABLE
        if p.node_name:
            rec["node_name"] = b.pos_of.get(p.node_name, -2)
        else:
            rec["node_name"] = -1
        # spec.nodeSelector -> labels.SelectorFromSet (Equals requirements)
        rec["sel_first"] = len(b.exprs)
        for k, v in p.node_selector.items():
            col = cluster.label_col(k)
            vid = cluster.value_id(col, v)
            if vid:
                b._expr(col, abi.OP_IN, [vid])
            else:
                b._expr()
        rec["sel_count"] = len(b.exprs) - rec["sel_first"]
        if p.required_terms is not None:
            flags |= abi.POD_HAS_REQUIRED_AFFINITY
            rec["req_term_first"] = len(b.terms)
            for t in p.required_terms:
                b.term(t)
            rec["req_term_count"] = len(b.terms) - rec["req_term_first"]
        rec["pref_term_first"] = len(b.terms)
        for pt in p.preferred_terms:
            if pt.weight == 0:
                continue
            b.term(pt.term, pt.weight)
        for pt in added_pref:                 # pl.addedPrefSchedTerms.Score(node)
            b.term(pt.term, pt.weight)
        rec["pref_term_count"] = len(b.terms) - rec["pref_term_first"]
        if added_count:
            flags |= abi.POD_ADDED_AFFINITY
            rec["added_term_first"], rec["added_term_count"] = added_first, added_count
        if p.has_volumes:
            flags |= abi.POD_HAS_VOLUMES
        elif p.pvc_claims:
            groups = None
            if volumes is not None:
                try:
                    groups = volumes.groups(p)
                except VolumeUnsupported:
                    groups = None
            if groups is None:
                flags |= abi.POD_HAS_VOLUMES
            else:
                vb, vz, n_bound = groups
                for key, terms_of, nb in (("vb", vb, n_bound), ("vz", vz, len(vz))):
                    rec[f"{key}_first"] = len(b.terms)
                    for g, ts in enumerate(terms_of):
                        gid = g if g < nb else g | abi.VB_UNBOUND_GROUP   # unbound-claim group
                        for t in ts:
                            b.term(t, gid)
                    rec[f"{key}_count"] = len(b.terms) - rec[f"{key}_first"]
                msg = volumes.prefilter_rejection(p)
                if msg is not None:                   # VolumeBinding PreFilter: no Filter runs
                    pf_reject[i] = ("VolumeBinding", msg)
        pf = prefilter_node_names(p)
        pf_names.append(pf)
        if pf is not None:                    # findNodesThatFitPod scans only these nodes
            flags |= abi.POD_NODE_NAMES
            known = sorted(b.pos_of[n] for n in pf if n in b.pos_of)
            if len(known) < len(pf):
                flags |= abi.POD_NODE_NAMES_UNKNOWN
            rec["nn_first"], rec["nn_count"] = len(nn), len(known)
            nn.extend(known)
        rec["flags"] = flags
        try:
            u, tflags = pod_uses(topo, cluster, p, spread)
        except TopologyError as e:
            raise EncodeError(str(e)) from e
        rec["use_first"], rec["use_count"] = len(uses), len(u)
        uses.extend(u)
        a = topo.adds(p)
        rec["add_first"], rec["add_count"] = len(adds), len(a)
        adds.extend(a)
        rec["topo_flags"] = tflags
        try:
            rec["nb_flags"], rec["nb_req"] = netbw.pod_request(p.annotations, cluster.nb_args)
            rec["nb_add"] = netbw.pod_allocated(p.annotations, cluster.nb_args)
        except netbw.QuantityError as e:
            raise EncodeError(f"pod {p.namespace}/{p.name}: {e}") from e
        names.append((p.namespace, p.name))
    exprs = np.array(b.exprs, abi.LABEL_EXPR_DTYPE) if b.exprs else np.zeros(0, abi.LABEL_EXPR_DTYPE)
    terms = np.zeros(len(b.terms), abi.TERM_DTYPE)
    for i, (f, n, w) in enumerate(b.terms):
        terms[i]["first_expr"], terms[i]["n_expr"], terms[i]["weight"] = f, n, w
    uarr = np.zeros(len(uses), abi.TOPO_USE_DTYPE)
    for i, (cls, arg, col, kind, fl) in enumerate(uses):
        uarr[i]["cls"], uarr[i]["arg"], uarr[i]["col"], uarr[i]["kind"], uarr[i]["flags"] = cls, arg, col, kind, fl
    aarr = np.zeros(len(adds), abi.CLASS_ADD_DTYPE)
    if adds:
        aarr["cls"] = [x[0] for x in adds]
        aarr["count"] = [x[1] for x in adds]
    cluster.refresh_classes()
    return EncodedPods(arr, exprs, terms, names, uarr, aarr, np.array(nn, np.int32), pf_names,
                       [pf_reject.get(i) for i in range(len(pods))] if pf_reject else [])
