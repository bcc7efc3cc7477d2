"""Helpers of tests/test_native_encode.py: the Python compile (ksim/encode.py)
and the native encoder (csrc/ksim_encode.cpp) on the same objects, compared
array by array and byte for byte."""
import numpy as np

from ksim import nativeenc
from ksim.encode import encode_cluster, encode_pods

CLUSTER_ARRAYS = ("alloc_cpu", "alloc_mem", "alloc_eph", "alloc_pods", "alloc_scalar", "req_cpu", "req_mem",
                  "req_eph", "req_scalar", "nz_cpu", "nz_mem", "num_pods", "flags", "taints", "labels",
                  "taint_effect", "label_col_offset", "label_num", "label_num_ok", "class_count", "topo_log",
                  "nb_limit", "nb_alloc")
CLUSTER_META = ("n_nodes", "n_scalar", "node_names", "label_keys", "label_values", "scalar_names")
POD_ARRAYS = ("pods", "exprs", "terms", "uses", "adds", "nn")


def _same_array(a, b, what):
    a, b = np.asarray(a), np.asarray(b)
    assert a.dtype == b.dtype, (what, a.dtype, b.dtype)
    assert a.shape == b.shape, (what, a.shape, b.shape)
    assert a.tobytes() == b.tobytes(), (what, _first_diff(a, b))


def _first_diff(a, b):
    if a.dtype.names:
        for f in a.dtype.names:
            if not np.array_equal(a[f], b[f]):
                i = int(np.flatnonzero((a[f] != b[f]).reshape(len(a), -1).any(axis=1))[0])
                return f, i, a[f][i], b[f][i]
    d = np.flatnonzero(a.reshape(-1) != b.reshape(-1))
    return int(d[0]), a.reshape(-1)[d[0]], b.reshape(-1)[d[0]]


def same_cluster(py, nat):
    for f in CLUSTER_ARRAYS:
        _same_array(getattr(py, f), getattr(nat, f), f)
    for f in CLUSTER_META:
        assert getattr(py, f) == getattr(nat, f), f
    assert [None if t is None else (t.key, t.value, t.effect) for t in py.taint_vocab] == \
        [None if t is None else (t.key, t.value, t.effect) for t in nat.taint_vocab]


def same_pods(py, nat):
    for f in POD_ARRAYS:
        _same_array(getattr(py, f), getattr(nat, f), f)
    assert py.names == nat.names
    assert py.prefilter_names == nat.prefilter_names
    assert py.prefilter_reject == nat.prefilter_reject


def both(nodes, bound, queues, cluster_kw=None, pods_kw=None):
    """Encode the snapshot and each queue of ``queues`` (in turn, on the same
    snapshot) both ways; assert equality after every step."""
    cluster_kw, pods_kw = cluster_kw or {}, pods_kw or {}
    pc, porder = encode_cluster(nodes, bound, **cluster_kw)
    enc = nativeenc.NativeEncoder()
    nc, norder = enc.encode_cluster(nodes, bound, **cluster_kw)
    assert porder == norder
    same_cluster(pc, nc)
    out = []
    for q in queues:
        pp = encode_pods(pc, q, **pods_kw)
        npods = enc.encode_pods(nc, q, **pods_kw)
        same_pods(pp, npods)
        same_cluster(pc, nc)
        out.append((pp, npods))
    return pc, nc, out
