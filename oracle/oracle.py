"""ctypes binding of libksim_oracle.so — the CPU restatement.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py.  The product path never imports this module.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "libksim_oracle.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run `make -C oracle`")
        L = ctypes.CDLL(path)
        vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
        L.ksim_oracle_create.restype = vp
        L.ksim_oracle_create.argtypes = [vp, vp, vp]
        L.ksim_oracle_destroy.argtypes = [vp]
        L.ksim_oracle_upsert_nodes.argtypes = [vp, vp, vp, vp]
        L.ksim_oracle_cycle.argtypes = [vp, vp, i32, vp]
        L.ksim_oracle_cycle_ext.argtypes = [vp, vp, i32, vp, vp, vp]
        L.ksim_oracle_preempt.argtypes = [vp, vp, i32, i32, vp, vp]
        L.ksim_oracle_preempt_nominated.argtypes = [vp, vp, i32, i32, vp, vp, i32, vp, vp, vp, vp]
        L.ksim_oracle_fw_filter.argtypes = [vp, vp, i32, vp]
        L.ksim_oracle_fw_score.argtypes = [vp, vp, i32, vp, i32, vp]
        L.ksim_oracle_fw_normalize.argtypes = [vp, i32, vp, vp, i32, vp]
        L.ksim_oracle_fw_filter_nominated.argtypes = [vp, vp, i32, vp, i32, vp, vp, vp, vp, vp]
        L.ksim_oracle_assume.argtypes = [vp, vp, i32, i32, ctypes.c_int]
        L.ksim_oracle_schedule.argtypes = [vp, vp, i32, i32, vp, ctypes.c_int, vp]
        L.ksim_oracle_get_node_state.argtypes = [vp] * 7
        L.ksim_oracle_get_class_count.argtypes = [vp, vp]
        L.ksim_oracle_get_nb_alloc.argtypes = [vp, vp]
        L.ksim_oracle_next_start.argtypes = [vp]
        L.ksim_oracle_next_start.restype = i32
        L.ksim_oracle_set_next_start.argtypes = [vp, i32]
        L.ksim_oracle_set_pod_seq.argtypes = [vp, i64]
        L.ksim_oracle_num_feasible_nodes_to_find.argtypes = [i32, i32]
        L.ksim_oracle_num_feasible_nodes_to_find.restype = i32
        L.ksim_oracle_least_requested_score.argtypes = [i64, i64]
        L.ksim_oracle_least_requested_score.restype = i64
        L.ksim_oracle_balanced_score.argtypes = [i32, vp, vp]
        L.ksim_oracle_balanced_score.restype = i64
        L.ksim_oracle_most_requested_score.argtypes = [i64, i64]
        L.ksim_oracle_most_requested_score.restype = i64
        L.ksim_oracle_broken_linear.argtypes = [vp, i64]
        L.ksim_oracle_broken_linear.restype = i64
        L.ksim_oracle_default_normalize.argtypes = [i64, ctypes.c_int, i32, vp]
        L.ksim_oracle_tb_key.argtypes = [i64, ctypes.c_uint64, i64, i32]
        L.ksim_oracle_tb_key.restype = ctypes.c_uint64
        _LIB = L
    return _LIB


class Oracle:
    """One simulated scheduler over an encoded cluster (CPU restatement)."""

    def __init__(self, cluster, profile):
        from ksim import abi  # noqa: F401
        self._keep = (cluster, profile)
        self.cluster = cluster
        self.profile = profile
        self._nt = cluster.node_table()
        self._vo = cluster.vocab()
        self.h = lib().ksim_oracle_create(ctypes.byref(self._nt), ctypes.byref(self._vo),
                                          ctypes.byref(profile))
        if not self.h:
            raise RuntimeError("ksim_oracle_create failed")
        self._layout = (cluster.n_label_cols, int(cluster.class_count.shape[0]))
        self._ran = False

    def upsert_nodes(self, cluster, old_pos):
        """ksim_engine.h ksim_upsert_nodes on the oracle (node informer deltas)."""
        nt, vo = cluster.node_table(), cluster.vocab()
        op = np.ascontiguousarray(old_pos, np.int32)
        assert op.size == cluster.n_nodes
        if lib().ksim_oracle_upsert_nodes(self.h, ctypes.byref(nt), ctypes.byref(vo),
                                          op.ctypes.data_as(ctypes.c_void_p)) != 0:
            raise RuntimeError("ksim_oracle_upsert_nodes failed")
        self.cluster = cluster
        self._keep = (cluster, self.profile)
        self._layout = (cluster.n_label_cols, int(cluster.class_count.shape[0]))

    def _sync(self):
        """As ksim.engine.Engine._sync: label columns / classes added by pods
        encoded after the oracle was made are re-sent in place."""
        c = self.cluster
        if (c.n_label_cols, int(c.class_count.shape[0])) == self._layout:
            return
        if int(c.class_count.shape[0]) != self._layout[1] and self._ran:
            raise RuntimeError("count classes registered after cycles ran on this oracle")
        self.upsert_nodes(c, np.arange(c.n_nodes, dtype=np.int32))

    def close(self):
        if self.h:
            lib().ksim_oracle_destroy(self.h)
            self.h = None

    __del__ = close

    def cycle(self, pods, index: int, ext_fail=None, ext_score=None) -> dict:
        """One compat cycle; ext_fail / ext_score (per node) model the extenders."""
        self._sync()
        self._ran = True
        from ksim import abi
        buf = abi.EvalBuffers(self.cluster.n_nodes, self.profile.n_score)
        ps = pods.pod_set()
        ef = None if ext_fail is None else np.ascontiguousarray(ext_fail, np.uint8)
        es = None if ext_score is None else np.ascontiguousarray(ext_score, np.int64)
        rc = lib().ksim_oracle_cycle_ext(self.h, ctypes.byref(ps), index,
                                         None if ef is None else ef.ctypes.data_as(ctypes.c_void_p),
                                         None if es is None else es.ctypes.data_as(ctypes.c_void_p),
                                         ctypes.byref(buf.out))
        if rc != 0:
            raise RuntimeError(f"oracle cycle failed: {rc}")
        return buf.result()

    # ---- framework-driven compat mode (ksim_oracle_fw_*) ----------------------
    def fw_prefilter(self, pods, index: int) -> dict:
        self._sync()
        self._ran = True
        from ksim import abi
        buf = abi.EvalBuffers(self.cluster.n_nodes, self.profile.n_score)
        self._fw = (pods, index)
        ps = pods.pod_set()
        if lib().ksim_oracle_fw_filter(self.h, ctypes.byref(ps), index, ctypes.byref(buf.out)) != 0:
            raise RuntimeError("oracle fw_filter failed")
        return buf.result()

    def fw_score(self, nodes) -> dict:
        from ksim import abi
        pods, index = self._fw
        arr = np.ascontiguousarray(nodes, np.int32)
        buf = abi.EvalBuffers(self.cluster.n_nodes, self.profile.n_score)
        ps = pods.pod_set()
        if lib().ksim_oracle_fw_score(self.h, ctypes.byref(ps), index, arr.ctypes.data_as(ctypes.c_void_p),
                                      arr.size, ctypes.byref(buf.out)) != 0:
            raise RuntimeError("oracle fw_score failed")
        return buf.result()

    def fw_filter_nominated(self, nominated, groups):
        """ksim_oracle_fw_filter_nominated (see ksim.engine.Engine.fw_filter_nominated)."""
        from ksim.engine import _nominated_groups
        pods, index = self._fw
        nodes, first, count, order = _nominated_groups(groups)
        fp = np.zeros(len(nodes), np.uint8)
        fd = np.zeros(len(nodes), np.uint32)
        ps = pods.pod_set()
        sub = nominated.subset_indices(order)      # kept alive: the pod set points into it
        nps = sub.pod_set()
        if lib().ksim_oracle_fw_filter_nominated(self.h, ctypes.byref(ps), index, ctypes.byref(nps), len(nodes),
                                                 *(a.ctypes.data_as(ctypes.c_void_p) for a in (nodes, first, count)),
                                                 fp.ctypes.data_as(ctypes.c_void_p),
                                                 fd.ctypes.data_as(ctypes.c_void_p)) != 0:
            raise RuntimeError("oracle fw_filter_nominated failed")
        return fp, fd

    def fw_normalize(self, slot: int, nodes, scores) -> np.ndarray:
        nd = np.ascontiguousarray(nodes, np.int32)
        sc = np.ascontiguousarray(scores, np.int64)
        out = np.zeros(nd.size, np.int64)
        if lib().ksim_oracle_fw_normalize(self.h, slot, nd.ctypes.data_as(ctypes.c_void_p),
                                          sc.ctypes.data_as(ctypes.c_void_p), nd.size,
                                          out.ctypes.data_as(ctypes.c_void_p)) != 0:
            raise RuntimeError("oracle fw_normalize failed")
        return out

    def assume(self, pods, index: int, node: int, sign: int = 1):
        """NodeInfo.AddPod (sign 1) / RemovePod (-1): Reserve / Unreserve."""
        self._sync()
        self._ran = True
        ps = pods.pod_set()
        if lib().ksim_oracle_assume(self.h, ctypes.byref(ps), index, node, sign) != 0:
            raise RuntimeError("oracle assume failed")

    def forget(self, pods, index: int, node: int):
        self.assume(pods, index, node, -1)

    def preempt(self, pods, index: int, priority: int, bound, groups=None) -> tuple:
        """DefaultPreemption PostFilter (ksim_oracle_preempt / _nominated).  ``bound``
        is a ksim.abi.BoundPods; ``groups`` as ksim.engine.Engine.preempt.  Returns
        (nominated node position or -1, victim indices, potential, candidates)."""
        self._sync()
        self._ran = True
        from ksim import abi
        from ksim.engine import _nominated_groups
        out = abi.PreemptOut(max(bound.n, 1))
        ps = pods.pod_set()
        if groups:
            nodes, first, count, order = _nominated_groups(groups)
            sub = pods.subset_indices(order)      # kept alive: the pod set points into it
            nps = sub.pod_set()
            rc = lib().ksim_oracle_preempt_nominated(self.h, ctypes.byref(ps), index, priority, ctypes.byref(bound.c),
                                                     ctypes.byref(nps), len(nodes),
                                                     *(a.ctypes.data_as(ctypes.c_void_p) for a in (nodes, first, count)),
                                                     ctypes.byref(out.c))
        else:
            rc = lib().ksim_oracle_preempt(self.h, ctypes.byref(ps), index, priority, ctypes.byref(bound.c),
                                           ctypes.byref(out.c))
        if rc != 0:
            raise RuntimeError(f"oracle preempt failed: {rc}")
        return out.result()

    def schedule(self, pods, first=0, count=None, nthreads=1):
        self._sync()
        self._ran = True
        from ksim import abi
        count = pods.n_pods - first if count is None else count
        chosen = np.zeros(count, np.int32)
        st = abi.BatchStats()
        ps = pods.pod_set()
        rc = lib().ksim_oracle_schedule(self.h, ctypes.byref(ps), first, count,
                                        chosen.ctypes.data_as(ctypes.c_void_p), nthreads,
                                        ctypes.byref(st))
        if rc != 0:
            raise RuntimeError(f"oracle schedule failed: {rc}")
        return chosen, st

    def node_state(self) -> dict:
        n = self.cluster.n_nodes
        out = {k: np.zeros(n, np.int64) for k in ("req_cpu", "req_mem", "req_eph", "nz_cpu", "nz_mem")}
        out["num_pods"] = np.zeros(n, np.int32)
        a = [out[k].ctypes.data_as(ctypes.c_void_p) for k in
             ("req_cpu", "req_mem", "req_eph", "nz_cpu", "nz_mem", "num_pods")]
        lib().ksim_oracle_get_node_state(self.h, *a)
        return out

    def class_count(self) -> np.ndarray:
        out = np.zeros((self.cluster.class_count.shape[0], self.cluster.n_nodes), np.int32)
        lib().ksim_oracle_get_class_count(self.h, out.ctypes.data_as(ctypes.c_void_p))
        return out

    def nb_alloc(self) -> np.ndarray:
        out = np.zeros(self.cluster.n_nodes, np.int64)
        lib().ksim_oracle_get_nb_alloc(self.h, out.ctypes.data_as(ctypes.c_void_p))
        return out

    @property
    def next_start(self) -> int:
        return lib().ksim_oracle_next_start(self.h)

    def set_next_start(self, s: int):
        lib().ksim_oracle_set_next_start(self.h, s)

    def set_pod_seq(self, s: int):
        lib().ksim_oracle_set_pod_seq(self.h, s)
