"""The native snapshot encoder (ksim_encode_nodes / ksim_encode_pods, ABI 10).

SURVEY.md §2.3 specifies the host snapshot encoder (NodeInfo -> SoA rows,
label / taint vocabularies, nodeTree order, the count-class compile) as a
native component.  ``csrc/ksim_encode.cpp`` is that encoder; this module is
its Python binding: ``Pool`` lays Kubernetes objects (ksim.model) out as the
flat ``ksim_k8s_pool`` a Go host would build from v1 objects
(integration/go/engine/encoder.go), and ``NativeEncoder`` returns the same
``EncodedCluster`` / ``EncodedPods`` as ksim.encode.encode_cluster /
encode_pods, byte for byte (tests/test_native_encode.py).

The encoder is host code: it runs without a GPU (it lives in
libksim_engine.so next to the device entry points).
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import abi, netbw
from .encode import EncodedCluster, EncodedPods, EncodeError, prefilter_node_names
from .model import LabelSelector, Node, Pod, Taint
from .topology import TopologyIndex
from .volumes import VolumeUnsupported


class Pool:
    """A ksim_k8s_pool under construction: strings interned once, every list a
    (first, count) range of a typed array (include/ksim_engine.h).  Tables of
    int32 records are kept as flat int lists (one extend per record)."""

    def __init__(self):
        self._sid: Dict[str, int] = {}
        self._strs: List[str] = []
        self.lists = {name: [] for name, _ in abi.POOL_ARRAYS}
        # records of objects several pods share (the pods of one workload share
        # their spec's selectors, terms and containers): id -> (object, record),
        # the object kept alive so its id is not reused
        self._memo: Dict[tuple, tuple] = {}
        self._width = {name: (len(dt.names) if dt.names else 1) for name, dt in abi.POOL_ARRAYS}

    def count(self, name: str) -> int:
        return len(self.lists[name]) // self._width[name] if name != "images" else len(self.lists[name])

    # ---- strings ----------------------------------------------------------
    def s(self, x) -> int:
        i = self._sid.get(x)
        if i is None:
            x = str(x)
            i = self._sid.get(x)
            if i is None:
                i = self._sid[x] = len(self._strs)
                self._strs.append(x)
        return i

    def strs(self, xs) -> Tuple[int, int]:
        if not xs:
            return 0, 0
        L = self.lists["str_list"]
        first = len(L)
        s = self.s
        L.extend([s(x) for x in xs])
        return first, len(L) - first

    def kv(self, d: Optional[dict]) -> Tuple[int, int]:
        if not d:
            return 0, 0
        L = self.lists["kv"]
        first = len(L) >> 1
        s = self.s
        for k, v in d.items():
            L.append(s(k))
            L.append(s(v))
        return first, len(d)

    # ---- selectors and terms --------------------------------------------------
    def reqs(self, rs) -> Tuple[int, int]:
        if not rs:
            return 0, 0
        rows = []
        s, strs = self.s, self.strs
        for r in rs:
            rows.append(s(r.key))
            rows.append(s(r.operator))
            rows.extend(strs(r.values))
        L = self.lists["reqs"]
        first = len(L) >> 2
        L.extend(rows)
        return first, len(rs)

    def term(self, t) -> int:
        e, f = self.reqs(t.match_expressions), self.reqs(t.match_fields)
        L = self.lists["terms"]
        L.extend(e + f)
        return (len(L) >> 2) - 1

    def terms(self, ts) -> Tuple[int, int]:
        idx = [self.term(t) for t in ts]
        return (idx[0], len(idx)) if idx else (0, 0)

    def preferred(self, pts) -> Tuple[int, int]:
        if not pts:
            return 0, 0
        rows = []
        for pt in pts:
            rows.append(int(pt.weight))
            rows.append(self.term(pt.term))
        L = self.lists["preferred"]
        first = len(L) >> 1
        L.extend(rows)
        return first, len(pts)

    def selector(self, sel: Optional[LabelSelector]) -> int:
        if sel is None:
            return -1
        hit = self._memo.get(("sel", id(sel)))
        if hit is not None:
            return hit[1]
        L = self.lists["selectors"]
        L.extend(self.kv(sel.match_labels) + self.reqs(sel.match_expressions))
        self._memo[("sel", id(sel))] = (sel, (len(L) >> 2) - 1)
        return (len(L) >> 2) - 1

    def pod_terms(self, ts, weighted: bool) -> Tuple[int, int]:
        if not ts:
            return 0, 0
        mk = ("pt", weighted) + tuple(map(id, ts))
        hit = self._memo.get(mk)
        if hit is not None:
            return hit[1]
        rng = self._pod_terms(ts, weighted)
        self._memo[mk] = (list(ts), rng)
        return rng

    def _pod_terms(self, ts, weighted: bool) -> Tuple[int, int]:
        rows = []
        for w in ts:
            t, wt = (w.term, int(w.weight)) if weighted else (w, 0)
            rows.append(self.s(t.topology_key))
            rows.append(self.selector(t.label_selector))
            rows.extend(self.strs(t.namespaces))
            rows.append(self.selector(t.namespace_selector))
            rows.append(wt)
        L = self.lists["pod_terms"]
        first = len(L) // 6
        L.extend(rows)
        return first, len(ts)

    def spread(self, cs) -> Tuple[int, int]:
        if not cs:
            return 0, 0
        rows = []
        for c in cs:
            rows.extend((int(c.max_skew), self.s(c.topology_key), self.s(c.when_unsatisfiable),
                         self.selector(c.label_selector),
                         -1 if c.node_affinity_policy is None else self.s(c.node_affinity_policy),
                         -1 if c.node_taints_policy is None else self.s(c.node_taints_policy)))
        L = self.lists["spread"]
        first = len(L) // 6
        L.extend(rows)
        return first, len(cs)

    def containers(self, cs) -> Tuple[int, int]:
        if not cs:
            return 0, 0
        mk = ("c",) + tuple(map(id, cs))
        hit = self._memo.get(mk)
        if hit is not None:
            return hit[1]
        rng = self._containers(cs)
        self._memo[mk] = (list(cs), rng)
        return rng

    def _containers(self, cs) -> Tuple[int, int]:
        rows = []
        s = self.s
        pl = self.lists["ports"]
        for c in cs:
            pf = len(pl) // 3
            for p in c.ports:
                pl.append(int(p.host_port))
                pl.append(s(p.protocol or ""))
                pl.append(s(p.host_ip or ""))
            rows.extend(self.kv(c.requests))
            rows.append(pf)
            rows.append(len(c.ports))
            rows.append(s(c.image or ""))
        L = self.lists["containers"]
        first = len(L) // 5
        L.extend(rows)
        return first, len(cs)

    def groups(self, gs) -> Tuple[int, int]:
        rows = []
        for ts in gs:
            rows.extend(self.terms(ts))
        L = self.lists["volume_groups"]
        first = len(L) >> 1
        L.extend(rows)
        return first, len(gs)

    # ---- objects ----------------------------------------------------------------
    def node(self, n: Node) -> None:
        s = self.s
        tl = self.lists["taints"]
        tf = len(tl) // 3
        for t in n.taints:
            tl.append(s(t.key))
            tl.append(s(t.value))
            tl.append(s(t.effect))
        il = self.lists["images"]
        imf = len(il)
        for names, size in n.images:
            il.append(self.strs(names) + (int(size),))
        self.lists["nodes"].extend((s(n.name), 1 if n.unschedulable else 0) + self.kv(n.labels) +
                                   (tf, len(n.taints)) + self.kv(n.allocatable) + self.kv(n.annotations) +
                                   (imf, len(n.images)))

    def pod(self, p: Pod, volumes=None) -> None:
        """One pod; ``volumes`` (a ksim.volumes.VolumeIndex) compiles its claims
        into VolumeBinding / VolumeZone groups as ksim.encode.encode_pods does."""
        s = self.s
        mode, vb, vz, nb = abi.K8S_VOLUMES_NONE, (0, 0), (0, 0), 0
        if p.has_volumes:
            mode = abi.K8S_VOLUMES_REFUSE
        elif p.pvc_claims:
            groups = None
            if volumes is not None:
                try:
                    groups = volumes.groups(p)
                except VolumeUnsupported:
                    groups = None
            if groups is None:
                mode = abi.K8S_VOLUMES_REFUSE
            else:
                mode = abi.K8S_VOLUMES_GROUPS
                gb, gz, nb = groups
                vb, vz = self.groups(gb), self.groups(gz)
        tf = 0
        if p.tolerations:
            tl = self.lists["tolerations"]
            tf = len(tl) >> 2
            for t in p.tolerations:
                tl.extend((s(t.key), s(t.operator), s(t.value), s(t.effect)))
        if p.required_terms is None:
            req = (-1, 0)
        elif not p.required_terms:
            req = (0, 0)
        else:
            req = self.terms(p.required_terms)
        owner = (-1, -1, -1) if p.owner is None else (s(p.owner[0]), s(p.owner[1]), s(p.owner[2]))
        kv, pt, Z = self.kv, self.pod_terms, (0, 0)
        self.lists["pods"].extend(
            (s(p.name), s(p.namespace)) + (kv(p.labels) if p.labels else Z) +
            (kv(p.annotations) if p.annotations else Z) + self.containers(p.containers) +
            (self.containers(p.init_containers) if p.init_containers else Z) +
            (kv(p.overhead) if p.overhead else Z) + (kv(p.node_selector) if p.node_selector else Z) + req +
            (self.preferred(p.preferred_terms) if p.preferred_terms else Z) + (tf, len(p.tolerations)) +
            (self.spread(p.topology_spread) if p.topology_spread else Z) +
            (pt(p.pod_affinity_required, False) if p.pod_affinity_required else Z) +
            (pt(p.pod_affinity_preferred, True) if p.pod_affinity_preferred else Z) +
            (pt(p.pod_anti_affinity_required, False) if p.pod_anti_affinity_required else Z) +
            (pt(p.pod_anti_affinity_preferred, True) if p.pod_anti_affinity_preferred else Z) +
            (s(p.node_name or ""),) + owner + (mode,) + vb + (nb,) + vz + (0,))

    # ---- the C struct -------------------------------------------------------------
    def build(self) -> abi.K8sPool:
        """The ksim_k8s_pool (this object keeps its arrays alive)."""
        enc = [x.encode() for x in self._strs]
        self._blob = np.frombuffer(b"".join(enc), np.uint8) if enc else np.zeros(0, np.uint8)
        off = np.zeros(len(enc) + 1, np.int64)
        if enc:
            np.cumsum(np.fromiter((len(x) for x in enc), np.int64, len(enc)), out=off[1:])
        self._off = off
        c = abi.K8sPool()
        c.strings = abi._p(self._blob)
        c.str_off = ctypes.c_void_p(off.ctypes.data)
        c.n_strings = len(enc)
        self._arrays = {}
        for name, dt in abi.POOL_ARRAYS:
            rows = self.lists[name]
            if name == "images":
                arr = np.array(rows, dtype=dt) if rows else np.zeros(0, dt)
            else:
                flat = np.array(rows, np.int32) if rows else np.zeros(0, np.int32)
                arr = flat.view(dt) if dt.names else flat
            self._arrays[name] = arr
            setattr(c, name, abi._p(arr))
            setattr(c, "n_" + name, int(arr.size))
        self.c = c
        return c


def _as_array(ptr, n, dtype, shape=None) -> np.ndarray:
    dt = np.dtype(dtype)
    if n == 0 or not ptr:
        return np.zeros(shape if shape is not None else 0, dt)
    buf = (ctypes.c_char * (n * dt.itemsize)).from_address(ptr)
    a = np.frombuffer(buf, dt, count=n).copy()
    return a.reshape(shape) if shape is not None else a


class NativeEncoder:
    """ksim_encoder: a snapshot and the queue compiled against it."""

    def __init__(self):
        from .engine import lib
        self.L = lib()
        h = ctypes.c_void_p()
        if self.L.ksim_encoder_create(ctypes.byref(h)) != 0:
            raise MemoryError("ksim_encoder_create")
        self.h = h
        self.cluster: Optional[EncodedCluster] = None
        self.seconds = {}

    def __del__(self):
        if getattr(self, "h", None):
            self.L.ksim_encoder_destroy(self.h)
            self.h = None

    def _chk(self, rc: int) -> None:
        if rc != 0:
            raise EncodeError(self.L.ksim_encoder_last_error(self.h).decode(errors="replace"))

    def _str(self, what: int, i: int, j: int = 0) -> str:
        s = self.L.ksim_encoder_string(self.h, what, i, j)
        if s is None:
            raise IndexError((what, i, j))
        return s.decode()

    # ---- snapshot ------------------------------------------------------------------
    def encode_cluster(self, nodes: Sequence[Node], bound_pods: Sequence[Pod] = (),
                       namespaces: Optional[Dict[str, Dict[str, str]]] = None,
                       nb_args: Optional[netbw.NetworkBandwidthArgs] = None, extra_scalar: Sequence[str] = (),
                       keep_previous: bool = False) -> Tuple[EncodedCluster, List[int]]:
        """ksim.encode.encode_cluster on the native encoder (no device matcher:
        the encoder matches the deduplicated signatures on the host)."""
        import gc
        import time
        t0 = time.perf_counter()
        pool = Pool()
        gc_was = gc.isenabled()
        gc.disable()                  # the pool's many small records are acyclic
        try:
            for n in nodes:
                pool.node(n)
            for p in bound_pods:
                pool.pod(p)
        finally:
            if gc_was:
                gc.enable()
        for name, labels in (namespaces or {}).items():
            pool.lists["namespaces"].extend((pool.s(name),) + pool.kv(labels) + (0,))
        nb_args = nb_args or netbw.NetworkBandwidthArgs()
        self.nb_args = nb_args
        self.namespaces = dict(namespaces or {})
        o = abi.EncodeNodesOpts()
        o.nb_node_limit = pool.s(nb_args.node_limit_annotation)
        o.nb_ingress_request = pool.s(nb_args.ingress_request_annotation)
        o.nb_egress_request = pool.s(nb_args.egress_request_annotation)
        o.keep_previous = 1 if keep_previous else 0
        o.extra_scalar_first, o.extra_scalar_count = pool.strs(extra_scalar)
        c = pool.build()
        t1 = time.perf_counter()
        self._chk(self.L.ksim_encode_nodes(self.h, ctypes.byref(c), ctypes.byref(o)))
        t2 = time.perf_counter()
        self.nodes = {n.name: n for n in nodes}
        cl, order = self._new_cluster()
        self.seconds = {"pool_s": t1 - t0, "native_s": t2 - t1}
        return cl, order

    def _new_cluster(self) -> Tuple[EncodedCluster, List[int]]:
        """A fresh EncodedCluster over the encoder's snapshot (``self.nodes``
        holds the node objects by name)."""
        info = self.info()
        N = info.n_nodes
        order = np.zeros(N, np.int32)
        self._chk(self.L.ksim_encoder_node_order(self.h, order.ctypes.data_as(ctypes.c_void_p)))
        order = [int(i) for i in order]
        names = [self._str(abi.ENC_STR_NODE_NAME, i) for i in range(N)]
        taint_vocab = [None] + [Taint(self._str(abi.ENC_STR_TAINT_KEY, t), self._str(abi.ENC_STR_TAINT_VALUE, t),
                                      self._str(abi.ENC_STR_TAINT_EFFECT, t)) for t in range(1, info.n_taints)]
        cl = EncodedCluster(n_nodes=N, n_scalar=info.n_scalar, alloc_cpu=None, alloc_mem=None, alloc_eph=None,
                            alloc_pods=None, alloc_scalar=None, req_cpu=None, req_mem=None, req_eph=None,
                            req_scalar=None, nz_cpu=None, nz_mem=None, num_pods=None, flags=None, taints=None,
                            labels=None, taint_effect=None, label_col_offset=None, label_num=None,
                            label_num_ok=None, topo=TopologyIndex(N, self.namespaces),
                            class_count=np.zeros((0, N), np.int32), topo_log=np.zeros(0),
                            nb_limit=np.zeros(0, np.int64), nb_alloc=np.zeros(0, np.int64),
                            node_names=names,
                            taint_vocab=taint_vocab,
                            scalar_names=[self._str(abi.ENC_STR_SCALAR, k) for k in range(info.n_scalar)],
                            nb_args=self.nb_args, node_labels=[dict(self.nodes[n].labels) for n in names])
        cl.native = self
        self.cluster = cl
        self._refresh(cl, full=True)
        return cl, order

    # ---- snapshot deltas (ABI 11) ----------------------------------------------------
    def update_nodes(self, nodes: Sequence[Node] = (), removed: Sequence[str] = ()
                     ) -> Tuple[EncodedCluster, np.ndarray, Optional[np.ndarray]]:
        """ksim_encoder_update_nodes: ``nodes`` added or updated, ``removed``
        names leave.  Returns the new snapshot (a new EncodedCluster), old_pos
        for ksim_upsert_nodes, and the updated rows when the delta was in place
        (ksim_encoder_changed_rows: ksim_update_node_rows takes it), else None."""
        pool = Pool()
        for n in nodes:
            pool.node(n)
        rem = np.array([pool.s(x) for x in removed], np.int32)
        c = pool.build()
        self._chk(self.L.ksim_encoder_update_nodes(self.h, ctypes.byref(c), rem.ctypes.data_as(ctypes.c_void_p),
                                                   int(rem.size)))
        for x in removed:
            self.nodes.pop(x, None)
        for n in nodes:
            self.nodes[n.name] = n
        cl, _ = self._new_cluster()
        old_pos = np.zeros(cl.n_nodes, np.int32)
        self._chk(self.L.ksim_encoder_old_pos(self.h, old_pos.ctypes.data_as(ctypes.c_void_p)))
        rows = np.zeros(max(len(nodes), 1), np.int32)
        k = self.L.ksim_encoder_changed_rows(self.h, rows.ctypes.data_as(ctypes.c_void_p), rows.size)
        return cl, old_pos, (rows[:k].copy() if k >= 0 else None)

    def bind(self, index: int, node: int) -> None:
        """ksim_encoder_bind: pod ``index`` of the last encode_pods is bound at ``node``."""
        self._chk(self.L.ksim_encoder_bind(self.h, index, node))

    def unbind(self, namespace: str, name: str) -> int:
        """ksim_encoder_unbind: returns the position the pod was bound at."""
        pos = ctypes.c_int32(-1)
        self._chk(self.L.ksim_encoder_unbind(self.h, namespace.encode(), name.encode(), ctypes.byref(pos)))
        return int(pos.value)

    def bound_node(self, namespace: str, name: str) -> int:
        pos = ctypes.c_int32(-1)
        self._chk(self.L.ksim_encoder_bound_node(self.h, namespace.encode(), name.encode(), ctypes.byref(pos)))
        return int(pos.value)

    def info(self) -> abi.EncoderInfo:
        info = abi.EncoderInfo()
        self._chk(self.L.ksim_encoder_get_info(self.h, ctypes.byref(info)))
        return info

    def _refresh(self, cl: EncodedCluster, full: bool) -> None:
        """Copy the encoder's node table / vocabulary into ``cl`` (new arrays,
        as EncodedCluster.label_col does: copies of a cluster share none)."""
        t, v = abi.NodeTable(), abi.Vocab()
        self._chk(self.L.ksim_encoder_cluster(self.h, ctypes.byref(t), ctypes.byref(v)))
        N, S, L = t.n_nodes, t.n_scalar, t.n_label_cols
        if full:
            for f, dt in (("alloc_cpu", np.int64), ("alloc_mem", np.int64), ("alloc_eph", np.int64),
                          ("alloc_pods", np.int32), ("req_cpu", np.int64), ("req_mem", np.int64),
                          ("req_eph", np.int64), ("nz_cpu", np.int64), ("nz_mem", np.int64),
                          ("num_pods", np.int32), ("flags", np.uint32), ("nb_limit", np.int64),
                          ("nb_alloc", np.int64)):
                setattr(cl, f, _as_array(getattr(t, f), N, dt))
            cl.alloc_scalar = _as_array(t.alloc_scalar, S * N, np.int64, (S, N))
            cl.req_scalar = _as_array(t.req_scalar, S * N, np.int64, (S, N))
            cl.taints = _as_array(t.taints, abi.MAX_NODE_TAINTS * N, np.uint16, (abi.MAX_NODE_TAINTS, N))
            cl.taint_effect = _as_array(v.taint_effect, v.n_taints, np.uint8)
            cl.topo_log = _as_array(v.topo_log, v.n_topo_log, np.float64)
        cl.labels = _as_array(t.labels, L * N, np.uint32, (L, N))
        cl.label_col_offset = _as_array(v.label_col_offset, L, np.int32)
        cl.label_num = _as_array(v.label_num, v.n_label_values, np.int64)
        cl.label_num_ok = _as_array(v.label_num_ok, v.n_label_values, np.uint8)
        cl.class_count = _as_array(t.class_count, t.n_classes * N, np.int32, (t.n_classes, N))
        cl.label_keys = [self._str(abi.ENC_STR_LABEL_KEY, k) for k in range(L)]
        off = list(cl.label_col_offset) + [int(v.n_label_values)]
        cl.label_values = [[self._str(abi.ENC_STR_LABEL_VALUE, k, j) for j in range(off[k + 1] - off[k])]
                           for k in range(L)]

    # ---- queue ---------------------------------------------------------------------
    def encode_pods(self, cluster: EncodedCluster, pods: Sequence[Pod], volumes=None, added_affinity=None,
                    spread=None) -> EncodedPods:
        """ksim.encode.encode_pods on the native encoder (``cluster`` must be
        this encoder's last snapshot; its label columns and classes grow)."""
        import time
        if cluster is not self.cluster:
            raise EncodeError("encode_pods needs the cluster this encoder encoded last")
        import gc
        t0 = time.perf_counter()
        pool = Pool()
        gc_was = gc.isenabled()
        gc.disable()
        try:
            for p in pods:
                pool.pod(p, volumes)
        finally:
            if gc_was:
                gc.enable()
        o = abi.EncodePodsOpts()
        o.added_required_first, o.added_required_count = -1, 0
        if added_affinity is not None:
            if added_affinity.required is not None:
                o.added_required_first, o.added_required_count = pool.terms(added_affinity.required)
                if not added_affinity.required:
                    o.added_required_first = 0
            o.added_preferred_first, o.added_preferred_count = pool.preferred(added_affinity.preferred)
        if spread is not None and spread.defaults:
            o.spread_defaults = abi.SPREAD_DEFAULTS_SYSTEM if spread.system else abi.SPREAD_DEFAULTS_LIST
            if not spread.system:
                o.spread_first, o.spread_count = pool.spread(spread.defaults)
            for ns, svcs in spread.services.items():
                for svc in svcs:
                    sel = (-1, 0) if svc.selector is None else pool.kv(svc.selector)
                    if svc.selector is not None and not svc.selector:
                        sel = (0, 0)
                    pool.lists["services"].extend((pool.s(svc.namespace),) + sel + (0,))
            for (kind, ns, name), ctl in spread.controllers.items():
                if kind == "ReplicationController":
                    rc = (-1, 0) if ctl.selector is None else pool.kv(ctl.selector)
                    if ctl.selector is not None and not ctl.selector:
                        rc = (0, 0)
                    sel = -1
                else:
                    rc, sel = (-1, 0), pool.selector(ctl.selector)
                pool.lists["controllers"].extend((pool.s(kind), pool.s(ns), pool.s(name)) + rc + (sel,))
        c = pool.build()
        t1 = time.perf_counter()
        self._chk(self.L.ksim_encode_pods(self.h, ctypes.byref(c), ctypes.byref(o)))
        t2 = time.perf_counter()
        self._refresh(cluster, full=False)
        ps = abi.PodSet()
        self._chk(self.L.ksim_encoder_pods(self.h, ctypes.byref(ps)))
        out = EncodedPods(_as_array(ps.pods, ps.n_pods, abi.POD_DTYPE),
                          _as_array(ps.exprs, ps.n_exprs, abi.LABEL_EXPR_DTYPE),
                          _as_array(ps.terms, ps.n_terms, abi.TERM_DTYPE),
                          [(p.namespace, p.name) for p in pods],
                          _as_array(ps.uses, ps.n_uses, abi.TOPO_USE_DTYPE),
                          _as_array(ps.adds, ps.n_adds, abi.CLASS_ADD_DTYPE),
                          _as_array(ps.nn, ps.n_nn, np.int32),
                          [prefilter_node_names(p) for p in pods])
        if volumes is not None:
            rej = []
            for p in pods:
                r = None
                if not p.has_volumes and p.pvc_claims:
                    try:
                        volumes.groups(p)
                        msg = volumes.prefilter_rejection(p)
                        r = None if msg is None else ("VolumeBinding", msg)
                    except VolumeUnsupported:
                        r = None
                rej.append(r)
            out.prefilter_reject = rej if any(x is not None for x in rej) else []
        self.seconds.update({"pods_pool_s": t1 - t0, "pods_native_s": t2 - t1})
        return out


def encode(nodes, bound, pods, **kw):
    """(EncodedCluster, EncodedPods) of a snapshot and its queue on a fresh encoder."""
    e = NativeEncoder()
    pod_kw = {k: kw.pop(k) for k in ("volumes", "added_affinity", "spread") if k in kw}
    cluster, _ = e.encode_cluster(nodes, bound, **kw)
    return cluster, e.encode_pods(cluster, pods, **pod_kw)
