"""Framework-driven cycles at 100 and 5,000 nodes (bench.py --mode fw's
sequence, 200 cycles): where ksim_fw_score / ksim_fw_normalize were answered
(host or device) and the per-call times, to find a slow path."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kube-scheduler-simulator_amd")]
import numpy as np  # noqa: E402
from ksim import abi, engine, gen, profile  # noqa: E402
from ksim.wrapped import HAS_NORMALIZE  # noqa: E402

for n_nodes in (100, 5000):
    cluster, pods = gen.config1(n_nodes=n_nodes, n_pods=400)
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=0)
    prof = profile.compile_profile(sp)
    nslots = [k for k, p in enumerate(sp.score_plugins()) if p.name in HAS_NORMALIZE]
    e = engine.Engine(0)
    e.set_profile(prof)
    e.set_cluster(cluster.copy_state())
    N = cluster.n_nodes
    K = profile.num_feasible_nodes_to_find(N, 0)
    ps = pods.pod_set()
    fb, sb = abi.EvalBuffers(N, prof.n_score), abi.EvalBuffers(N, prof.n_score)
    nout = np.zeros(N, np.int64)
    ns = 0
    t = {"pre": 0.0, "score": 0.0, "norm": 0.0, "misses": []}
    for i in range(200):
        c0 = time.perf_counter()
        assert e.L.ksim_fw_prefilter(e.h, ctypes.byref(ps), i, ctypes.byref(fb.out)) == 0
        t["pre"] += time.perf_counter() - c0
        order = np.roll(np.arange(N, dtype=np.int32), -ns)
        feas = order[fb.fail_plugin[order] == abi.PASSED]
        lst = np.ascontiguousarray(feas[:K])
        proc = int(np.nonzero(order == feas[K])[0][0]) if feas.size > K else N
        ns = (ns + proc) % N
        if lst.size <= 1:
            continue
        c0 = time.perf_counter()
        assert e.L.ksim_fw_score(e.h, lst.ctypes.data_as(ctypes.c_void_p), lst.size, ctypes.byref(sb.out)) == 0
        t["score"] += time.perf_counter() - c0
        for k in nslots:
            before = e.diag()["fw_normalize_device"]
            sc = np.ascontiguousarray(sb.raw[k][lst])
            c0 = time.perf_counter()
            assert e.L.ksim_fw_normalize(e.h, k, lst.ctypes.data_as(ctypes.c_void_p), sc.ctypes.data_as(ctypes.c_void_p),
                                         lst.size, nout.ctypes.data_as(ctypes.c_void_p)) == 0
            t["norm"] += time.perf_counter() - c0
            if e.diag()["fw_normalize_device"] != before and len(t["misses"]) < 5:
                t["misses"].append((i, k, int(lst.size), sc[:6].tolist()))
        node = int(lst[int(np.argmax(sb.total[lst]))])
        assert e.L.ksim_assume(e.h, ctypes.byref(ps), i, node) == 0
    d = e.diag()
    print(n_nodes, {k: round(v / 200 * 1e6, 1) if isinstance(v, float) else v for k, v in t.items()},
          {k: d[k] for k in ("fw_score_host", "fw_score_device", "fw_normalize_cached", "fw_normalize_device")},
          flush=True)
    e.close()
