"""Binding of libksim_engine.so (the product path).

Fails loudly when the HIP library is missing or no GPU is present: there is no
CPU fallback anywhere in the product path.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np

from . import abi

_HERE = os.path.dirname(os.path.abspath(__file__))
# KSIM_LIB_VARIANT=<tag> loads an A/B build of the batch geometry
# (csrc/Makefile "variant": libksim_engine_<tag>.so); the default is the product build.
_VARIANT = os.environ.get("KSIM_LIB_VARIANT", "")
LIB_PATH = os.path.join(_HERE, f"libksim_engine_{_VARIANT}.so" if _VARIANT else "libksim_engine.so")
_LIB = None

# Exported symbols declared in include/ksim_engine.h (checked by tests).
EXPORTS = [
    "ksim_abi_version", "ksim_abi_sizeof", "ksim_create", "ksim_destroy", "ksim_last_error",
    "ksim_set_profile", "ksim_set_cluster", "ksim_get_node_state", "ksim_get_class_count", "ksim_get_nb_alloc", "ksim_get_next_start",
    "ksim_set_next_start", "ksim_set_pod_seq", "ksim_eval_pod", "ksim_assume", "ksim_forget",
    "ksim_load_pods", "ksim_schedule_loaded", "ksim_schedule_batch", "ksim_reset_cluster",
    "ksim_time_kernels", "ksim_kernel_name", "ksim_time_eval", "ksim_get_diag", "ksim_batch_geometry",
    "ksim_set_shard", "ksim_comm_unique_id", "ksim_comm_init", "ksim_group_schedule_loaded",
    "ksim_emit_cycle_json", "ksim_eval_pod_filter", "ksim_eval_pod_finish",
    "ksim_set_bound_pods", "ksim_preempt", "ksim_upsert_nodes", "ksim_remove_node",
    "ksim_match_terms", "ksim_set_eval_range", "ksim_fw_prefilter", "ksim_fw_score", "ksim_fw_normalize",
    "ksim_fw_filter_nominated", "ksim_preempt_nominated",
    "ksim_encoder_create", "ksim_encoder_destroy", "ksim_encoder_last_error", "ksim_encode_nodes",
    "ksim_encode_pods", "ksim_encoder_cluster", "ksim_encoder_pods", "ksim_encoder_get_info",
    "ksim_encoder_node_order", "ksim_encoder_string", "ksim_encoder_update_nodes", "ksim_encoder_old_pos",
    "ksim_encoder_bind", "ksim_encoder_unbind", "ksim_encoder_bound_node", "ksim_encoder_changed_rows",
    "ksim_update_node_rows",
]


def _nominated_groups(groups):
    """(node, [pod indices]) groups -> the C arrays: the pods of group k are
    entries [first[k], first[k] + count[k]) of the pod set re-ordered by ``order``."""
    nodes, first, count, order = [], [], [], []
    for node, idx in groups:
        nodes.append(int(node))
        first.append(len(order))
        count.append(len(idx))
        order.extend(int(i) for i in idx)
    return (np.array(nodes, np.int32), np.array(first, np.int32), np.array(count, np.int32), order)


class KsimError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"ksim error {code}: {msg}")
        self.code = code


_VARIANTS = {}


def lib_variant(tag: str):
    """An A/B or instrumented flavor of the library (same ABI), loaded next to
    the product build."""
    if tag not in _VARIANTS:
        _VARIANTS[tag] = _load(os.path.join(_HERE, f"libksim_engine_{tag}.so"))
    return _VARIANTS[tag]


def lib():
    global _LIB
    if _LIB is None:
        _LIB = _load(LIB_PATH)
    return _LIB


def _load(path):
    if not os.path.exists(path):
        raise RuntimeError(f"{path} missing: build it with `make -C kube-scheduler-simulator_amd/csrc` "
                           "(or __graft_entry__.build()); there is no CPU fallback")
    L = ctypes.CDLL(path)
    vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
    L.ksim_abi_version.restype = ctypes.c_int
    L.ksim_abi_sizeof.restype = ctypes.c_size_t
    L.ksim_abi_sizeof.argtypes = [ctypes.c_int]
    L.ksim_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
    L.ksim_destroy.argtypes = [vp]
    L.ksim_destroy.restype = None
    L.ksim_last_error.argtypes = [vp]
    L.ksim_last_error.restype = ctypes.c_char_p
    L.ksim_set_profile.argtypes = [vp, vp]
    L.ksim_set_cluster.argtypes = [vp, vp, vp]
    L.ksim_upsert_nodes.argtypes = [vp, vp, vp, vp]
    L.ksim_remove_node.argtypes = [vp, i32]
    L.ksim_get_node_state.argtypes = [vp] * 7
    L.ksim_get_class_count.argtypes = [vp, vp]
    L.ksim_get_nb_alloc.argtypes = [vp, vp]
    L.ksim_get_next_start.argtypes = [vp, vp]
    L.ksim_set_next_start.argtypes = [vp, i32]
    L.ksim_set_pod_seq.argtypes = [vp, i64]
    L.ksim_eval_pod.argtypes = [vp, vp, i32, vp]
    L.ksim_eval_pod_filter.argtypes = [vp, vp, i32, vp]
    L.ksim_set_bound_pods.argtypes = [vp, vp]
    L.ksim_preempt.argtypes = [vp, vp, i32, i32, vp]
    L.ksim_preempt_nominated.argtypes = [vp, vp, i32, i32, vp, i32, vp, vp, vp, vp]
    L.ksim_eval_pod_finish.argtypes = [vp, vp, vp, vp]
    L.ksim_match_terms.argtypes = [vp, vp, vp, vp]
    L.ksim_set_eval_range.argtypes = [vp, i32, i32]
    L.ksim_fw_prefilter.argtypes = [vp, vp, i32, vp]
    L.ksim_fw_score.argtypes = [vp, vp, i32, vp]
    L.ksim_fw_filter_nominated.argtypes = [vp, vp, i32, vp, vp, vp, vp, vp]
    L.ksim_fw_normalize.argtypes = [vp, i32, vp, vp, i32, vp]
    L.ksim_assume.argtypes = [vp, vp, i32, i32]
    L.ksim_forget.argtypes = [vp, vp, i32, i32]
    L.ksim_load_pods.argtypes = [vp, vp]
    L.ksim_schedule_loaded.argtypes = [vp, i32, i32, vp, vp]
    L.ksim_schedule_batch.argtypes = [vp, vp, vp, vp]
    L.ksim_reset_cluster.argtypes = [vp]
    L.ksim_time_kernels.argtypes = [vp, i32, i32, vp, vp, i32]
    L.ksim_kernel_name.argtypes = [i32]
    L.ksim_emit_cycle_json.argtypes = [vp, vp, i64, vp, i64, vp, i64, vp]
    L.ksim_time_eval.argtypes = [vp, i32, i32, vp, vp]
    L.ksim_kernel_name.restype = ctypes.c_char_p
    L.ksim_get_diag.argtypes = [vp, vp, i32]
    L.ksim_batch_geometry.argtypes = [vp, i32]
    L.ksim_set_shard.argtypes = [vp, i32, i32]
    L.ksim_comm_unique_id.argtypes = [vp]
    L.ksim_comm_init.argtypes = [vp, i32, i32, vp]
    L.ksim_group_schedule_loaded.argtypes = [vp, i32, i32, i32, vp, vp]
    # the native snapshot encoder (host code: callable without a GPU)
    L.ksim_encoder_create.argtypes = [ctypes.POINTER(vp)]
    L.ksim_encoder_destroy.argtypes = [vp]
    L.ksim_encoder_destroy.restype = None
    L.ksim_encoder_last_error.argtypes = [vp]
    L.ksim_encoder_last_error.restype = ctypes.c_char_p
    L.ksim_encode_nodes.argtypes = [vp, vp, vp]
    L.ksim_encode_pods.argtypes = [vp, vp, vp]
    L.ksim_encoder_cluster.argtypes = [vp, vp, vp]
    L.ksim_encoder_pods.argtypes = [vp, vp]
    L.ksim_encoder_get_info.argtypes = [vp, vp]
    L.ksim_encoder_node_order.argtypes = [vp, vp]
    L.ksim_encoder_string.argtypes = [vp, i32, i32, i32]
    L.ksim_encoder_string.restype = ctypes.c_char_p
    L.ksim_encoder_update_nodes.argtypes = [vp, vp, vp, i32]
    L.ksim_encoder_old_pos.argtypes = [vp, vp]
    L.ksim_encoder_bind.argtypes = [vp, i32, i32]
    L.ksim_encoder_changed_rows.argtypes = [vp, vp, i32]
    L.ksim_update_node_rows.argtypes = [vp, vp, vp, vp, i32]
    L.ksim_encoder_unbind.argtypes = [vp, ctypes.c_char_p, ctypes.c_char_p, vp]
    L.ksim_encoder_bound_node.argtypes = [vp, ctypes.c_char_p, ctypes.c_char_p, vp]
    return L


def batch_geometry() -> dict:
    """Batch-path geometry compiled into libksim_engine.so (no GPU needed)."""
    out = np.zeros(4, np.int32)
    lib().ksim_batch_geometry(out.ctypes.data_as(ctypes.c_void_p), 4)
    return {"pods_per_batch": int(out[0]), "top_t": int(out[1]), "top_threads": int(out[2]),
            "lane_cand": int(out[3])}


COMM_ID_BYTES = 128


def comm_unique_id() -> bytes:
    """ncclGetUniqueId through the engine (rank 0 of a node-sharded run)."""
    buf = (ctypes.c_uint8 * COMM_ID_BYTES)()
    rc = lib().ksim_comm_unique_id(buf)
    if rc != 0:
        raise KsimError(rc, "ksim_comm_unique_id failed (librccl?)")
    return bytes(buf)


def group_schedule_loaded(engines, first: int, count: int):
    """In-process shard group on one device (ksim_group_schedule_loaded)."""
    arr = (ctypes.c_void_p * len(engines))(*[e.h.value for e in engines])
    chosen = np.zeros(count, np.int32)
    st = abi.BatchStats()
    L = engines[0].L
    rc = L.ksim_group_schedule_loaded(arr, len(engines), first, count,
                                      chosen.ctypes.data_as(ctypes.c_void_p), ctypes.byref(st))
    if rc != 0:
        raise KsimError(rc, L.ksim_last_error(engines[0].h).decode())
    return chosen, st


class Engine:
    """One engine handle on one GPU (one scheduler profile, one snapshot)."""

    def __init__(self, device: int = 0, variant: Optional[str] = None):
        # variant: an instrumented / experimental build of the same ABI
        # (csrc/Makefile "flavor": libksim_engine_<variant>.so), e.g. the
        # chain-delay build of the race regression test
        self.L = lib() if variant is None else lib_variant(variant)
        h = ctypes.c_void_p()
        rc = self.L.ksim_create(device, ctypes.byref(h))
        if rc != 0:
            raise KsimError(rc, f"ksim_create(device={device}) failed (no GPU / HIP runtime?)")
        self.h = h
        self.n_nodes = 0
        self.n_score = 0
        self._keep = []
        self.cluster = None
        self._ran = False

    def _chk(self, rc: int):
        if rc != 0:
            raise KsimError(rc, self.L.ksim_last_error(self.h).decode())

    def close(self):
        if getattr(self, "h", None) and getattr(self, "L", None) is not None:
            self.L.ksim_destroy(self.h)
        self.h = None

    __del__ = close

    def set_shard(self, node_base: int, n_total: int):
        """This handle holds global node positions [node_base, node_base + n) of n_total."""
        self._chk(self.L.ksim_set_shard(self.h, node_base, n_total))
        self._split = True

    def set_eval_range(self, lo: int, hi: int):
        """Replicated sharding: this handle (whole cluster) evaluates nodes [lo, hi)."""
        self._chk(self.L.ksim_set_eval_range(self.h, lo, hi))
        self._split = True

    def comm_init(self, rank: int, world: int, uid: bytes):
        buf = (ctypes.c_uint8 * COMM_ID_BYTES).from_buffer_copy(uid)
        self._chk(self.L.ksim_comm_init(self.h, rank, world, buf))

    def set_profile(self, prof: abi.Profile):
        self._chk(self.L.ksim_set_profile(self.h, ctypes.byref(prof)))
        self.n_score = prof.n_score

    def set_cluster(self, cluster):
        nt, vo = cluster.node_table(), cluster.vocab()
        self._chk(self.L.ksim_set_cluster(self.h, ctypes.byref(nt), ctypes.byref(vo)))
        self._track(cluster, nt)
        self._ran = False

    def _track(self, cluster, nt):
        self.cluster = cluster
        self.n_nodes = cluster.n_nodes
        self.n_classes = nt.n_classes
        self._layout = (cluster.n_label_cols, int(nt.n_classes))

    def upsert_nodes(self, cluster, old_pos):
        """Node informer deltas (ksim_upsert_nodes): ``cluster`` is the new
        snapshot, old_pos[i] the current position of its node i or -1."""
        nt, vo = cluster.node_table(), cluster.vocab()
        op = np.ascontiguousarray(old_pos, np.int32)
        if op.size != cluster.n_nodes:
            raise ValueError("old_pos must have one entry per node of the new snapshot")
        self._chk(self.L.ksim_upsert_nodes(self.h, ctypes.byref(nt), ctypes.byref(vo),
                                          op.ctypes.data_as(ctypes.c_void_p)))
        self._track(cluster, nt)
        self._keep = []

    def update_node_rows(self, cluster, rows):
        """UpdateNode in place (ksim_update_node_rows): the static columns of
        ``rows`` from ``cluster`` (same layout and vocabulary as the handle's)."""
        nt, vo = cluster.node_table(), cluster.vocab()
        r = np.ascontiguousarray(rows, np.int32)
        self._chk(self.L.ksim_update_node_rows(self.h, ctypes.byref(nt), ctypes.byref(vo),
                                               r.ctypes.data_as(ctypes.c_void_p), int(r.size)))
        self.cluster = cluster
        self._layout = (cluster.n_label_cols, int(nt.n_classes))
        self._keep = []

    def remove_node(self, pos: int):
        """RemoveNode of the node at ``pos`` (ksim_remove_node); the host
        snapshot object is no longer the engine's (positions moved)."""
        self._chk(self.L.ksim_remove_node(self.h, pos))
        self.n_nodes -= 1
        self.cluster = None
        self._keep = []

    def _sync(self):
        """Pods encoded after set_cluster may have added label columns (keys a
        pod references get one on first use) or count classes to the host
        snapshot: re-send it in place (every node kept)."""
        c = getattr(self, "cluster", None)
        if c is None or (c.n_label_cols, int(c.class_count.shape[0])) == self._layout:
            return
        if getattr(self, "_split", False):
            # a shard or a replica must not turn into a whole-snapshot handle
            # behind its group's back: encode every pod before sharding
            raise RuntimeError("pods encoded after the cluster was sharded / replicated added label columns or "
                               "count classes: encode every pod before shard() / set_cluster")
        if int(c.class_count.shape[0]) != self._layout[1] and self._ran:
            raise RuntimeError("count classes were registered after cycles ran on this engine: "
                               "encode every pod before scheduling, or re-send the snapshot (upsert_nodes)")
        self.upsert_nodes(c, np.arange(c.n_nodes, dtype=np.int32))

    def class_count(self) -> np.ndarray:
        """Count classes [n_classes][n_nodes] as the device holds them now."""
        out = np.zeros((self.n_classes, self.n_nodes), np.int32)
        self._chk(self.L.ksim_get_class_count(self.h, out.ctypes.data_as(ctypes.c_void_p)))
        return out

    def nb_alloc(self) -> np.ndarray:
        """NetworkBandwidth allocated amount per node (milli-units), as the device holds it."""
        out = np.zeros(self.n_nodes, np.int64)
        self._chk(self.L.ksim_get_nb_alloc(self.h, out.ctypes.data_as(ctypes.c_void_p)))
        return out

    def eval_pod(self, pods, index: int) -> dict:
        self._sync()
        self._ran = True
        buf = abi.EvalBuffers(self.n_nodes, self.n_score)
        ps = pods.pod_set()
        self._chk(self.L.ksim_eval_pod(self.h, ctypes.byref(ps), index, ctypes.byref(buf.out)))
        return buf.result()

    def eval_pod_extenders(self, pods, index: int, extender) -> dict:
        """A compat cycle around an extender round trip: ``extender(filter
        result) -> (ext_fail[n] or None, ext_score[n] or None)`` sees the filter
        pass (kept nodes: fail_plugin == PASSED)."""
        self._sync()
        self._ran = True
        buf = abi.EvalBuffers(self.n_nodes, self.n_score)
        ps = pods.pod_set()
        self._chk(self.L.ksim_eval_pod_filter(self.h, ctypes.byref(ps), index, ctypes.byref(buf.out)))
        ef, es = extender(buf.result())
        ef = None if ef is None else np.ascontiguousarray(ef, np.uint8)
        es = None if es is None else np.ascontiguousarray(es, np.int64)
        buf2 = abi.EvalBuffers(self.n_nodes, self.n_score)
        self._chk(self.L.ksim_eval_pod_finish(self.h, None if ef is None else ef.ctypes.data_as(ctypes.c_void_p),
                                             None if es is None else es.ctypes.data_as(ctypes.c_void_p),
                                             ctypes.byref(buf2.out)))
        return buf2.result()

    # ---- framework-driven compat mode (ksim_fw_*) ----------------------------
    def fw_prefilter(self, pods, index: int) -> dict:
        """PreFilter + Filter of every node of the pod's scan set (the framework
        chooses which of them its workers visit)."""
        self._sync()
        self._ran = True
        buf = abi.EvalBuffers(self.n_nodes, self.n_score)
        ps = pods.pod_set()
        self._chk(self.L.ksim_fw_prefilter(self.h, ctypes.byref(ps), index, ctypes.byref(buf.out)))
        return buf.result()

    def fw_filter_nominated(self, nominated, groups):
        """RunFilterPluginsWithNominatedPods' first pass for the cycle in flight:
        ``groups`` = [(node, [pod indices of ``nominated``]), ...].  Returns
        (fail_plugin, fail_detail) arrays, one entry per group."""
        nodes, first, count, order = _nominated_groups(groups)
        fp = np.zeros(len(nodes), np.uint8)
        fd = np.zeros(len(nodes), np.uint32)
        sub = nominated.subset_indices(order)      # kept alive: the pod set points into it
        ps = sub.pod_set()
        self._chk(self.L.ksim_fw_filter_nominated(self.h, ctypes.byref(ps), len(nodes),
                                                  *(a.ctypes.data_as(ctypes.c_void_p) for a in (nodes, first, count)),
                                                  fp.ctypes.data_as(ctypes.c_void_p),
                                                  fd.ctypes.data_as(ctypes.c_void_p)))
        return fp, fd

    def fw_score(self, nodes) -> dict:
        """PreScore / Score / NormalizeScore over exactly the framework's feasible list."""
        arr = np.ascontiguousarray(nodes, np.int32)
        buf = abi.EvalBuffers(self.n_nodes, self.n_score)
        self._chk(self.L.ksim_fw_score(self.h, arr.ctypes.data_as(ctypes.c_void_p), arr.size,
                                      ctypes.byref(buf.out)))
        return buf.result()

    def fw_normalize(self, slot: int, nodes, scores) -> np.ndarray:
        """NormalizeScore of score slot ``slot`` over an explicit (node, score) list."""
        nd = np.ascontiguousarray(nodes, np.int32)
        sc = np.ascontiguousarray(scores, np.int64)
        if nd.size != sc.size:
            raise ValueError("one score per node")
        out = np.zeros(nd.size, np.int64)
        self._chk(self.L.ksim_fw_normalize(self.h, slot, nd.ctypes.data_as(ctypes.c_void_p),
                                          sc.ctypes.data_as(ctypes.c_void_p), nd.size,
                                          out.ctypes.data_as(ctypes.c_void_p)))
        return out

    def set_bound_pods(self, bound):
        """The bound-pod table DefaultPreemption may evict (ksim.abi.BoundPods)."""
        self._bound_n = bound.n
        self._chk(self.L.ksim_set_bound_pods(self.h, ctypes.byref(bound.c)))

    def preempt(self, pods, index: int, priority: int, groups=None) -> tuple:
        """DefaultPreemption PostFilter dry run: (nominated node or -1, victim
        indices into the bound-pod table, potential nodes, candidates).
        ``groups`` = [(node, [indices of ``pods``]), ...]: the PodNominator's
        pods of priority >= ``priority`` per node (ksim_preempt_nominated)."""
        self._sync()
        self._ran = True
        out = abi.PreemptOut(max(getattr(self, "_bound_n", 1), 1))
        ps = pods.pod_set()
        if not groups:
            self._chk(self.L.ksim_preempt(self.h, ctypes.byref(ps), index, priority, ctypes.byref(out.c)))
            return out.result()
        nodes, first, count, order = _nominated_groups(groups)
        sub = pods.subset_indices(order)      # kept alive: the pod set points into it
        nps = sub.pod_set()
        self._chk(self.L.ksim_preempt_nominated(self.h, ctypes.byref(ps), index, priority, ctypes.byref(nps),
                                                len(nodes), *(a.ctypes.data_as(ctypes.c_void_p)
                                                              for a in (nodes, first, count)),
                                                ctypes.byref(out.c)))
        return out.result()

    def match_terms(self, mp: abi.MatchProblem, n_words: int, counts: Optional[np.ndarray]) -> np.ndarray:
        """ksim_match_terms: [n_sigs][n_words] matcher bits; ``counts``
        ([n_classes][n_nodes] int32, or None) receives the class counts."""
        bits = np.zeros((max(mp.n_sigs, 1), max(n_words, 1)), np.uint32)
        cp = None if counts is None else counts.ctypes.data_as(ctypes.c_void_p)
        self._chk(self.L.ksim_match_terms(self.h, ctypes.byref(mp), bits.ctypes.data_as(ctypes.c_void_p), cp))
        return bits[:mp.n_sigs, :n_words]

    def last_match_ms(self) -> float:
        """Device time of the last match_terms call (its kernels, HIP events)."""
        return self.diag()["match_ns"] / 1e6

    def assume(self, pods, index: int, node: int):
        self._sync()
        self._ran = True
        ps = pods.pod_set()
        self._chk(self.L.ksim_assume(self.h, ctypes.byref(ps), index, node))

    def forget(self, pods, index: int, node: int):
        self._sync()
        self._ran = True
        ps = pods.pod_set()
        self._chk(self.L.ksim_forget(self.h, ctypes.byref(ps), index, node))

    def load_pods(self, pods):
        self._sync()
        ps = pods.pod_set()
        self._chk(self.L.ksim_load_pods(self.h, ctypes.byref(ps)))
        self._keep = [pods]

    def schedule_loaded(self, first: int, count: int, want_chosen: bool = True):
        chosen = np.zeros(count, np.int32) if want_chosen else None
        st = abi.BatchStats()
        self._ran = True
        self._chk(self.L.ksim_schedule_loaded(
            self.h, first, count, chosen.ctypes.data_as(ctypes.c_void_p) if chosen is not None else None,
            ctypes.byref(st)))
        return chosen, st

    def schedule_batch(self, pods):
        self.load_pods(pods)
        return self.schedule_loaded(0, pods.n_pods)

    def node_state(self) -> dict:
        n = self.n_nodes
        out = {k: np.zeros(n, np.int64) for k in ("req_cpu", "req_mem", "req_eph", "nz_cpu", "nz_mem")}
        out["num_pods"] = np.zeros(n, np.int32)
        a = [out[k].ctypes.data_as(ctypes.c_void_p) for k in
             ("req_cpu", "req_mem", "req_eph", "nz_cpu", "nz_mem", "num_pods")]
        self._chk(self.L.ksim_get_node_state(self.h, *a))
        return out

    @property
    def next_start(self) -> int:
        v = ctypes.c_int32()
        self._chk(self.L.ksim_get_next_start(self.h, ctypes.byref(v)))
        return v.value

    def set_next_start(self, s: int):
        self._chk(self.L.ksim_set_next_start(self.h, s))

    def set_pod_seq(self, s: int):
        self._chk(self.L.ksim_set_pod_seq(self.h, s))

    def reset_cluster(self):
        """Restore the uploaded snapshot's dynamic node state (device-side copy)."""
        self._chk(self.L.ksim_reset_cluster(self.h))

    def diag(self) -> dict:
        """Batch-path diagnostics of the last schedule_loaded call."""
        out = np.zeros(27, np.int64)
        n = self.L.ksim_get_diag(self.h, out.ctypes.data_as(ctypes.c_void_p), 27)
        if n < 0:
            self._chk(n)
        d = {"batches": int(out[0]), "truncations": int(out[1]), "cuts": int(out[2]),
             "graph_captures": int(out[19]), "dbg": [int(x) for x in out[3:19]], "match_ns": int(out[20]),
             "fw_score_host": int(out[21]), "fw_score_device": int(out[22]), "fw_normalize_cached": int(out[23]),
             "fw_normalize_device": int(out[24]), "variants": int(out[25]), "tb_variant_pods": int(out[26])}
        if out[6]:
            d["chain_us"] = {"setup": out[3] / out[6] / 100.0, "rounds": out[4] / out[6] / 100.0,
                             "epilogue": out[5] / out[6] / 100.0, "rounds_per_batch": out[7] / out[6]}
        return d

    def time_eval(self, first: int, reps: int = 200):
        """(kernel name, mean ms) of the evaluation kernel launched back to back (ksim_time_eval)."""
        ms = ctypes.c_double()
        k = ctypes.c_int32()
        self._chk(self.L.ksim_time_eval(self.h, first, reps, ctypes.byref(ms), ctypes.byref(k)))
        return self.L.ksim_kernel_name(k.value).decode(), ms.value

    def time_kernels(self, first: int, count: int) -> dict:
        """Schedule loaded pods [first, first+count) with HIP events between the
        kernels on the engine's own stream.  Returns {kernel: (mean ms, launches)}
        for every kernel that ran."""
        out = np.zeros(32, np.float64)
        cnt = np.zeros(32, np.int64)
        n = self.L.ksim_time_kernels(self.h, first, count, out.ctypes.data_as(ctypes.c_void_p),
                                    cnt.ctypes.data_as(ctypes.c_void_p), 32)
        if n < 0:
            self._chk(n)
        return {self.L.ksim_kernel_name(k).decode(): (float(out[k]), int(cnt[k]))
                for k in range(n) if cnt[k] > 0}


# ---- result emission (ksim_emit_cycle_json) -------------------------------------------
class _EmitInput(ctypes.Structure):
    _fields_ = [("n_nodes", ctypes.c_int32), ("n_filter", ctypes.c_int32), ("n_score", ctypes.c_int32),
                ("n_messages", ctypes.c_int32),
                ("node_names", ctypes.c_void_p), ("filter_names", ctypes.c_void_p),
                ("score_names", ctypes.c_void_p), ("score_weight", ctypes.c_void_p),
                ("has_normalize", ctypes.c_void_p), ("fail_plugin", ctypes.c_void_p),
                ("msg_id", ctypes.c_void_p), ("messages", ctypes.c_void_p), ("scored", ctypes.c_void_p),
                ("raw", ctypes.c_void_p), ("norm", ctypes.c_void_p)]


def _cstrs(names):
    arr = (ctypes.c_char_p * max(len(names), 1))()
    for i, n in enumerate(names):
        arr[i] = n.encode()
    return arr


def emit_cycle_json(node_names, filter_names, score_names, score_weight, has_normalize, fail_plugin, msg_id,
                    messages, scored, raw, norm):
    """(filter-result, score-result, finalscore-result) annotation values of one
    cycle, encoded natively (host C++, no GPU)."""
    keep = []

    def arr(a, dt):
        a = np.ascontiguousarray(a, dt)
        keep.append(a)
        return a.ctypes.data_as(ctypes.c_void_p)

    names = [_cstrs(node_names), _cstrs(filter_names), _cstrs(score_names), _cstrs(messages)]
    e = _EmitInput(len(node_names), len(filter_names), len(score_names), len(messages),
                   ctypes.cast(names[0], ctypes.c_void_p), ctypes.cast(names[1], ctypes.c_void_p),
                   ctypes.cast(names[2], ctypes.c_void_p), arr(score_weight, np.int32),
                   arr(has_normalize, np.uint8), arr(fail_plugin, np.uint8), arr(msg_id, np.int32),
                   ctypes.cast(names[3], ctypes.c_void_p), arr(scored, np.uint8), arr(raw, np.int64),
                   arr(norm, np.int64))
    lens = np.zeros(3, np.int64)
    n = max(len(node_names), 1)
    caps = [n * (32 + 48 * len(filter_names)) + 64, n * (32 + 48 * len(score_names)) + 64,
            n * (32 + 48 * len(score_names)) + 64]
    for _ in range(2):
        bufs = [ctypes.create_string_buffer(c) for c in caps]
        rc = lib().ksim_emit_cycle_json(ctypes.byref(e), bufs[0], caps[0], bufs[1], caps[1], bufs[2], caps[2],
                                        lens.ctypes.data_as(ctypes.c_void_p))
        if rc == 0:
            return tuple(b.value.decode() for b in bufs)
        if all(lens[k] + 1 <= caps[k] for k in range(3)):
            raise KsimError(rc, "ksim_emit_cycle_json: invalid input")
        caps = [int(n) + 1 for n in lens]
    raise KsimError(rc, "ksim_emit_cycle_json failed")
