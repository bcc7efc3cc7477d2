#!/usr/bin/env python3
"""bench.py — pod x node filter+score evaluations/s of the scheduling cycle on MI355X.

Metric (BASELINE.json): pod x node filter+score evals/sec (pods scheduled/sec
reported beside it).  One step = one full pass of the workload on the engine:
reset the node snapshot (device-side copy) and run every scheduling cycle
(Filter over every node, Score, NormalizeScore, weights, selectHost, bind).
Inputs (cluster SoA + pod queue) are resident in HBM before the timed region.

  python bench.py [--gpus N --steps K --warmup W] [--config 2|3|4|5] [--mode p100|adapt]

Workloads:
  config 2 (default)  N = 1: 5,000 nodes x 50,000 pods, default profile, P100;
                      the same workload under ADAPT (the simulator's forced
                      default, percentageOfNodesToScore 0) is timed beside it
                      ("adapt" in the JSON line).
                      N > 1: node-sharded weak scaling, --nodes-per-gpu (5,000)
                      x N nodes, the same 50,000 pods; one process per GPU, per
                      batch an RCCL all-gather of candidates + all-reduce (max).
  config 3            PodTopologySpread + InterPodAffinity heavy (10k nodes, 3
                      zones, 100k existing pods with anti-affinity terms), per-pod
                      path; N > 1 node-shards the one cluster (strong scaling).
  config 4            100,000 nodes x 1M pods, node-sharded over N GPUs (strong).
  config 5            policy sweep: 1,024 score-weight vectors over config 2
                      (first 10,000 pods), vectors split over the N GPUs.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "kube-scheduler-simulator_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

B_EVAL = 112            # algorithmic HBM bytes per pod x node evaluation
B_FILTER = 60           # the filter columns of a row: allocatable 28 + requested 24 + pods 4 + flags 4
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E peak (MI355X_MICROARCH.md chip table)
# VALU issue peak: 256 CUs x 4 SIMDs, a wave64 vector instruction holds a SIMD
# for 2 cycles (MI355X_MICROARCH.md "Wave scheduling"), 2.4 GHz
VALU_PEAK_G = 256 * 4 * 0.5 * 2.4          # G wave-instructions / s


def _k_adapt(n: int) -> int:
    from ksim.profile import num_feasible_nodes_to_find
    return num_feasible_nodes_to_find(n, 0)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def kernel_alg_bytes(name: str, n_nodes: int, n_norm: int, geom: dict) -> int:
    """Algorithmic HBM bytes per launch of each kernel:
    the node rows an evaluation kernel must read once per pod it evaluates;
    the small bookkeeping kernels are priced by the keys they move."""
    B, T = geom["pods_per_batch"], geom["top_t"]
    if name == "k_filter_score":
        return B_EVAL * n_nodes                       # one node row per pod x node eval
    if name == "k_extrema":
        return n_nodes * (1 + 8 * n_norm)             # fail code + normalized raws
    if name == "k_select":
        return n_nodes * (1 + 8 + 8 * n_norm)         # fail code + partial total + normalized raws
    if name == "k_batch_top":
        return B_EVAL * n_nodes * B                   # B pods x N nodes evals per launch
    if name == "k_batch_top_commit":                  # the evaluation + the previous batch's commit
        return B_EVAL * n_nodes * B + 8 * B * 3
    if name == "k_batch_chain_pairs":                 # the chain runs inside every pairs block
        return B * (B - 1) // 2 * B_EVAL + 8 * B * T * 2   # one bound-row re-eval per pod pair + the lists
    if name.startswith("k_tb_"):                      # topology batches: Bt pods per launch on average
        bt = geom.get("tb_pods_per_batch", 1.0)
        nblk = (n_nodes + 255) // 256
        if name == "k_tb_filter":
            return int(B_EVAL * n_nodes * bt)         # one node row per pod x node eval
        if name == "k_tb_select":
            return int(n_nodes * bt * (1 + 1 + 8 + 8 * n_norm + 4))   # fail, ign, part, raws, stat
        if name == "k_tb_merge":
            return int(8 * bt * (nblk * T + T))
        if name == "k_tb_chain_pairs":
            return int(bt * (bt - 1) / 2 * B_EVAL + 8 * bt * T * 2)
        return int(8 * B * 3)
    if name == "k_adapt_mask":
        return B_FILTER * n_nodes * B                 # filter columns of every node row, per pod
    if name == "k_adapt_top":
        return B_EVAL * geom.get("adapt_k", n_nodes) * B  # the K kept rows scored per pod
    if name == "k_batch_commit":
        return 8 * B * 3                                  # guesses, pair maxima, placements
    return 0


# the kernel that carries the pod x node evaluations on each path
EVAL_KERNELS = ("k_batch_top_commit", "k_batch_top", "k_adapt_top", "k_tb_filter", "k_filter_score")


def _profile_entry(fname: str, kernel: str, nodes: int, config: int, mode: str = None):
    """The committed PMC measurement (profiles/<fname>) of a kernel at a size,
    on this bench config (config 1 and 2 run the same kernels on 5,000 nodes
    with different pods); mode: the entry's mode too, when it names one."""
    path = os.path.join(ROOT, "profiles", fname)
    try:
        tj = json.load(open(path))
    except (OSError, ValueError):
        return None
    for entry in (tj if isinstance(tj, list) else [tj]):
        if (isinstance(entry, dict) and entry.get("kernel") == kernel and entry.get("nodes") == nodes
                and entry.get("config") == config and (mode is None or entry.get("mode", mode) == mode)):
            return entry
    return None


def host_cpu() -> dict:
    """What the CPU baseline ran on: logical CPUs, the CPUs this process may
    run on (affinity), the cgroup CPU quota when one is set, the model name."""
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    return {"nproc": os.cpu_count(), "affinity_cpus": affinity, "cgroup_cpu_quota": quota, "model": model}


def cpu_threads_sweep(arg: str) -> list:
    """--cpu-threads: a comma list, "sweep" (1, 4, 8, 16, 64 and every logical
    CPU: the 1 -> 16 scaling is reported), or one count.  The sweep stops at
    4x the cgroup CPU quota when one is set: the GPU box grants 16 CPUs of its
    256, and 256 OpenMP threads time-sliced on them ran 100 cycles in 43.6 s
    against 4.7 s for 49,900 cycles at 16 (profiles/r03/reentry/
    bench_default.json threads_sweep)."""
    n = os.cpu_count() or 1
    if arg == "sweep":
        quota = host_cpu()["cgroup_cpu_quota"]
        cap = n if not quota else max(16, int(4 * quota))
        return sorted({t for t in (1, 4, 8, 16, 64, n) if t <= min(n, cap)} | {min(16, n)})
    return [int(x) for x in arg.split(",")]


def cpu_baseline(cluster, pods, sp, seconds: float, threads, label: str) -> dict:
    """The CPU restatement (oracle, OpenMP over nodes) on a bounded sample,
    at each thread count of ``threads``; the best rate is the baseline (the
    whole host's, when the sweep reaches every logical CPU)."""
    from ksim import profile
    from oracle.oracle import Oracle
    prof = profile.compile_profile(sp)
    sweep = []
    for t in threads:
        o = Oracle(cluster.copy_state(), prof)
        t0 = time.perf_counter()
        _, st = o.schedule(pods, 0, 100, nthreads=t)
        dt = time.perf_counter() - t0
        n = int(min(pods.n_pods - 100, max(100, (seconds / max(dt, 1e-6)) * 100)))
        t0 = time.perf_counter()
        _, st2 = o.schedule(pods, 100, n, nthreads=t)
        dt2 = time.perf_counter() - t0
        sweep.append({"threads": t, "value": st2.evals / dt2, "pods_per_s": n / dt2, "cycles": n,
                      "evals": int(st2.evals), "seconds": dt2})
        log(f"[rank 0] cpu baseline {t} threads: {st2.evals / dt2:.3e} evals/s ({n} cycles, {dt2:.1f} s)")
    best = max(sweep, key=lambda x: x["value"])
    one = next((x for x in sweep if x["threads"] == 1), None)
    scaling = {f"{x['threads']}_threads_vs_1": x["value"] / one["value"] for x in sweep} if one else None
    return {"value": best["value"], "unit": "pod x node evals/s", "cores": best["threads"], "kind": "port",
            "pods_per_s": best["pods_per_s"], "host": host_cpu(), "threads_sweep": sweep, "scaling": scaling,
            "sample": f"{label} pods 100..{100 + best['cycles']} ({best['cycles']} cycles, {best['evals']} evals) "
                      f"after 100 warm cycles from the empty cluster, same profile/mode, oracle/ksim_oracle.c "
                      f"OpenMP (filter, scan, scores, NormalizeScore extrema, totals and selectHost split per "
                      f"thread); best of {[x['threads'] for x in sweep]} threads ({best['threads']}), "
                      f"{best['seconds']:.1f} s"}


HOST_COMPILE = {}
SWEEP = {}


class TimedMatcher:
    """DeviceMatcher with its wall time per call (host CSR build + device call)
    and the device time of the ksim_match_terms kernels (HIP events)."""

    def __init__(self, inner):
        self.inner = inner
        self.seconds = []
        self.device_ms = []

    def match(self, mp):
        t = time.perf_counter()
        r = self.inner.match(mp)
        self.seconds.append(time.perf_counter() - t)
        self.device_ms.append(self.inner.engine.last_match_ms())
        return r


def host_compile(args, nodes, bound, incoming):
    """The snapshot and queue compile (once per snapshot / queue, outside the
    timed region; it replaces upstream's per-pod PreFilter / PreScore scans of
    the existing pods).  Default: the native encoder (csrc/ksim_encode.cpp,
    ksim_encode_nodes / ksim_encode_pods); the ksim.model objects are first
    laid out as its flat ksim_k8s_pool, the step a Go host does with its v1
    objects (pool_build_s, Python here).  --python-encode: the Python compile
    (ksim/encode.py) with the count classes matched on the device."""
    if not args.python_encode:
        from ksim.nativeenc import NativeEncoder
        enc = NativeEncoder()
        cluster, _ = enc.encode_cluster(nodes, bound)
        pods = enc.encode_pods(cluster, incoming)
        sec = enc.seconds
        HOST_COMPILE.update({
            "encoder": "native (ksim_encode_nodes / ksim_encode_pods)",
            "native_s": sec["native_s"] + sec["pods_native_s"],
            "native_encode_nodes_s": sec["native_s"], "native_encode_pods_s": sec["pods_native_s"],
            "pool_build_s": sec["pool_s"] + sec["pods_pool_s"],
            "existing_pods": len(bound), "incoming_pods": len(incoming),
            "note": "count-class compile, once per snapshot / queue, not in the timed region; pool_build_s lays "
                    "the Python objects out as the encoder's flat input (a Go host builds it from v1 objects)"})
        return cluster, pods
    from ksim.encode import encode_cluster, encode_pods
    matcher = None
    if not args.host_match and bound:
        # selector / term matching of the count classes on the device
        # (ksim_match_terms, int8 MFMA contraction)
        from ksim.engine import Engine
        from ksim.termmatch import DeviceMatcher
        matcher = TimedMatcher(DeviceMatcher(Engine(int(os.environ.get("LOCAL_RANK", "0")))))
    t0 = time.perf_counter()
    cluster, _ = encode_cluster(nodes, bound, matcher=matcher)
    t1 = time.perf_counter()
    pods = encode_pods(cluster, incoming)
    t2 = time.perf_counter()
    HOST_COMPILE.update({"encoder": "python (ksim/encode.py)", "encode_cluster_s": t1 - t0, "encode_pods_s": t2 - t1,
                         "existing_pods": len(bound), "incoming_pods": len(incoming),
                         "term_matching": "host (Python)" if matcher is None else "device (ksim_match_terms)",
                         "note": "count-class compile (ksim/encode.py + ksim/topology.py), once per "
                                 "snapshot/queue, not in the timed region"})
    if matcher is not None:
        HOST_COMPILE["match_calls_s"] = matcher.seconds
        HOST_COMPILE["match_device_ms"] = matcher.device_ms
        matcher.inner.engine.close()
    return cluster, pods


def build(cfg: int, args, rank: int, world: int):
    """(cluster, pods, profile, description, sharded, scaling) for one rank."""
    from ksim import gen, profile
    pct = 100 if args.mode == "p100" else 0
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=pct)
    if cfg == 2:
        n = args.nodes if world == 1 else args.nodes_per_gpu * world
        cluster, pods = gen.config2(n, args.pods)
        desc = f"config2: default profile, {n} nodes x {pods.n_pods} pods, {args.mode.upper()}"
        if world > 1:
            desc += f", node-sharded {world} x {args.nodes_per_gpu} nodes (weak scaling)"
        return cluster, pods, sp, desc, world > 1, "weak"
    if cfg == 1:
        # config 1's object distribution (taints incl. PreferNoSchedule,
        # tolerations, required / preferred node affinity) scaled to config 2's
        # size: the batch path with per-node normalized scores
        nodes, pobjs = gen.config1_objects(n_nodes=args.nodes, n_pods=args.pods)
        cluster, pods = host_compile(args, nodes, [], pobjs)
        desc = (f"config1-scaled: default profile, config-1 distribution on {cluster.n_nodes} nodes x "
                f"{pods.n_pods} pods, {args.mode.upper()}")
        return cluster, pods, sp, desc, False, "strong"
    if cfg == 4:
        cluster, pods = gen.config4(args.nodes4, args.pods4)
        desc = f"config4: default profile, {cluster.n_nodes} nodes x {pods.n_pods} pods, {args.mode.upper()}, " \
               f"node-sharded over {world} GPU(s)"
        return cluster, pods, sp, desc, world > 1, "strong"
    if cfg == 3:
        nodes, bound, incoming = gen.config3_objects(n_nodes=args.nodes3, n_incoming=args.pods3)
        cluster, pods = host_compile(args, nodes, bound, incoming)
        desc = (f"config3: default profile, {cluster.n_nodes} nodes / 3 zones, "
                f"{int(cluster.num_pods.sum())} existing pods with anti-affinity terms, {pods.n_pods} incoming "
                f"pods with spread constraints + preferred anti-affinity, {args.mode.upper()}")
        if world > 1:
            desc += f", node-sharded over {world} GPUs"
        return cluster, pods, sp, desc, world > 1, "strong"
    if cfg == 5:
        cluster, pods = gen.config2(5000, 10000)
        desc = f"config5: {args.sweep} score-weight vectors over 5000 nodes x 10000 pods, {args.mode.upper()}, " \
               f"vectors split over {world} GPU(s), {args.sweep_streams} concurrent engines per GPU"
        return cluster, pods, sp, desc, False, "strong"
    raise SystemExit(f"unknown config {cfg}")


def kernel_table(kt, kt_pods, n_pods, ms_per_step, knodes, n_norm, geom, sharded, concurrent=False) -> dict:
    """Per-kernel times that add up to the step.  ksim_time_kernels brackets
    every launch with HIP events on the engine's stream, run eagerly, which
    adds a few microseconds per launch that the graph-replayed step does not
    pay; each kernel's event time is kept as ``avg_ms_events`` and ``avg_ms``
    is it scaled by (step device time for the timed pods) / (sum of event
    times), so sum(avg_ms x launches) reconciles with ms_per_step (exactly for
    unsharded runs, whose step is device time; the rocprof summaries under
    profiles/ give the unscaled kernel durations).  ``share`` is the fraction
    of the step.  ``concurrent`` (config 5: many weight vectors per step on
    concurrent streams): the table is one vector's run, event times as
    measured (a step holds no single vector's device time to reconcile to)."""
    total = sum(v[0] * v[1] for v in kt.values())
    target = ms_per_step * kt_pods / max(n_pods, 1)
    scale = target / total if total > 0 and not sharded and not concurrent else 1.0
    out = {}
    for k, (ms, n) in kt.items():
        a = ms * scale
        out[k] = {"avg_ms": a, "avg_ms_events": ms, "launches": n, "share": (ms * n / total) if total else None,
                  "alg_GBps": kernel_alg_bytes(k, knodes, n_norm, geom) / (a * 1e-3) / 1e9}
    if concurrent:
        out["_reconciled"] = {"per": "one weight vector, its own run (event times)", "timed_pods": kt_pods,
                              "sum_ms": sum(v["avg_ms"] * v["launches"] for k, v in out.items())}
        return out
    out["_reconciled"] = {"sum_ms_for_timed_pods": sum(v["avg_ms"] * v["launches"] for k, v in out.items()),
                          "timed_pods": kt_pods, "step_ms_scaled_to_timed_pods": target, "event_scale": scale}
    return out


def roofline_entry(dominant, achieved, traffic, alg, avg_ms, timing, knodes, by_time, valu) -> dict:
    """The dominant kernel's roofline.  With a committed PMC instruction count
    (profiles/valu.json) the bound is the VALU issue rate: the batch kernels
    sweep an L2-resident node table (PMC HBM traffic far below the 112 B per
    evaluation), so their algorithmic-HBM fraction can exceed 1 and bounds
    nothing; that figure is kept under "hbm", the PMC bytes under "traffic"."""
    # the HBM side of a VALU-bound kernel: the PMC bytes it moves per launch
    # over its launch time; the algorithmic rate (112 B per evaluation, from
    # L2 / MALL mostly) is no HBM utilisation and carries no fraction
    hbm = {"achieved": (traffic / (avg_ms * 1e-3) / 1e9) if traffic else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": (traffic / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS) if traffic else None,
           "source": "PMC traffic (profiles/traffic.json) over this run's launch time",
           "alg_bytes_per_launch": alg, "alg_rate_GBps": achieved,
           "note": "algorithmic bytes = 112 B per pod x node evaluation (SURVEY 8(d)), served from L2 / MALL"}
    common = {"kernel": dominant, "traffic": traffic, "traffic_unit": "HBM bytes per launch (PMC)",
              "avg_launch_ms": avg_ms, "timing": timing, "kernel_nodes": knodes, "dominant_by_time": by_time}
    if valu is None:
        return {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "alg_bytes_per_launch": alg, **common}
    return {"bound": "valu", "achieved": valu["achieved"], "peak": valu["peak"], "unit": valu["unit"],
            "frac": valu["frac"], **common, "valu": valu, "hbm": hbm,
            "note": ("VALU issue peak = 256 CUs x 4 SIMDs x one wave64 instruction per 2 cycles x 2.4 GHz; "
                     "instructions per launch from rocprofv3 --pmc SQ_INSTS_VALU (profiles/valu.json) over this "
                     "run's launch time")}


def bench_fw(args, out):
    """--mode fw: the drop-in's per-pod cost.  The calls the Go adapter makes
    for one scheduling cycle (integration/go/engine/plugins.go, encoder.go):
    ksim_encode_pods (the pod compiled against the snapshot by the native
    encoder), ksim_fw_prefilter (Filter of every node, F x N answers and the
    raw scores copied back), the framework's feasible list (here the
    sequential worker's first K in scan order from nextStartNodeIndex),
    ksim_fw_score over it (answered on the host when no PreScore depends on
    the list), ksim_fw_normalize per NormalizeScore plugin, the max total,
    ksim_assume; output buffers reused as the adapter would.  Config 1's
    distribution at 100 nodes (the reference's own config 1) and 5,000 nodes;
    the oracle's ksim_oracle_fw_* calls beside it on the same sequence (CPU,
    one thread; pods pre-compiled).  The Python objects are laid out as the
    encoder's flat pool before the loop (a Go host builds it from its v1 pod:
    ``pool_build_us``, Python here, is reported, not counted).  One JSON line;
    Python ctypes glue included in ``us_per_cycle``, the C calls alone in
    ``us_in_calls``."""
    import ctypes
    import time
    import numpy as np
    from ksim import abi, engine, gen, profile
    from ksim.nativeenc import NativeEncoder, Pool
    from ksim.wrapped import HAS_NORMALIZE
    from oracle.oracle import Oracle, lib as olib

    class FwDriveFns(ctypes.Structure):
        _fields_ = [(nm, ctypes.c_void_p) for nm in ("encode_pods", "encoder_pods", "prefilter", "score",
                                                      "normalize", "assume")]

    class FwDriveResult(ctypes.Structure):
        _fields_ = [("sec", ctypes.c_double * 5), ("total", ctypes.c_double), ("bound", ctypes.c_int64),
                    ("cycles", ctypes.c_int64)]

    drv_path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools", "libksim_fwdrive.so")
    DRV = ctypes.CDLL(drv_path) if os.path.exists(drv_path) else None
    if DRV is not None:
        DRV.fwdrive_run.restype = ctypes.c_int
        DRV.fwdrive_run.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                                    ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p]
    rows = []
    for n_nodes, n_pods in ((100, 1000), (5000, 3000)):
        nodes, pobjs = gen.config1_objects(n_nodes=n_nodes, n_pods=n_pods)
        enc = NativeEncoder()
        cluster, _ = enc.encode_cluster(nodes)
        pods = enc.encode_pods(cluster, pobjs)      # every label column / class of the queue exists
        sp = profile.SchedulerProfile(percentage_of_nodes_to_score=0)
        prof = profile.compile_profile(sp)
        snames = [p.name for p in sp.score_plugins()]
        nslots = [k for k, nm in enumerate(snames) if nm in HAS_NORMALIZE]
        N = cluster.n_nodes
        K = profile.num_feasible_nodes_to_find(N, 0)
        ps_all = pods.pod_set()
        # one flat pool per pod (the Go host's marshalling of its v1 pod)
        t0 = time.perf_counter()
        pools = []
        for p in pobjs:
            pl = Pool()
            pl.pod(p)
            pl.build()
            pools.append(pl)
        pool_us = (time.perf_counter() - t0) / n_pods * 1e6
        opts = abi.EncodePodsOpts()
        opts.added_required_first = -1
        EL = engine.lib()

        def run(kind, count):
            if kind == "engine":
                e = engine.Engine(0)
                e.set_profile(prof)
                e.set_cluster(cluster.copy_state())
                L, h = e.L, e.h
                pset = abi.PodSet()

                def encode(i):
                    rc = EL.ksim_encode_pods(enc.h, ctypes.byref(pools[i].c), ctypes.byref(opts))
                    return rc or EL.ksim_encoder_pods(enc.h, ctypes.byref(pset))
                pre = lambda i, out: L.ksim_fw_prefilter(h, ctypes.byref(pset), 0, ctypes.byref(out))
                score = lambda arr, out: L.ksim_fw_score(h, arr.ctypes.data_as(ctypes.c_void_p), arr.size,
                                                         ctypes.byref(out))
                norm = lambda k, arr, sc, o: L.ksim_fw_normalize(h, k, arr.ctypes.data_as(ctypes.c_void_p),
                                                                 sc.ctypes.data_as(ctypes.c_void_p), arr.size,
                                                                 o.ctypes.data_as(ctypes.c_void_p))
                assume = lambda i, node: L.ksim_assume(h, ctypes.byref(pset), 0, node)
            else:
                e = Oracle(cluster.copy_state(), prof)
                O, h = olib(), e.h
                encode = lambda i: 0
                pre = lambda i, out: O.ksim_oracle_fw_filter(h, ctypes.byref(ps_all), i, ctypes.byref(out))
                score = lambda arr, out: O.ksim_oracle_fw_score(h, ctypes.byref(ps_all), cur[0],
                                                               arr.ctypes.data_as(ctypes.c_void_p), arr.size,
                                                               ctypes.byref(out))
                norm = lambda k, arr, sc, o: O.ksim_oracle_fw_normalize(h, k, arr.ctypes.data_as(ctypes.c_void_p),
                                                                        sc.ctypes.data_as(ctypes.c_void_p),
                                                                        arr.size, o.ctypes.data_as(ctypes.c_void_p))
                assume = lambda i, node: O.ksim_oracle_assume(h, ctypes.byref(ps_all), i, node, 1)
            cur = [0]
            fb, sb = abi.EvalBuffers(N, prof.n_score), abi.EvalBuffers(N, prof.n_score)
            nout = np.zeros(N, np.int64)
            ns, in_calls, bound = 0, 0.0, 0
            split = {"encode": 0.0, "prefilter": 0.0, "score": 0.0, "normalize": 0.0, "assume": 0.0}
            t0 = time.perf_counter()
            for i in range(count):
                cur[0] = i
                c0 = time.perf_counter()
                rc = encode(i)
                c1 = time.perf_counter()
                rc = rc or pre(i, fb.out)
                c2 = time.perf_counter()
                split["encode"] += c1 - c0
                split["prefilter"] += c2 - c1
                in_calls += c2 - c0
                if rc != 0:
                    raise RuntimeError(f"{kind} encode / fw_prefilter rc {rc}")
                order = np.roll(np.arange(N, dtype=np.int32), -ns)
                feas = order[fb.fail_plugin[order] == abi.PASSED]
                lst = np.ascontiguousarray(feas[:K])
                proc = int(np.nonzero(order == feas[K])[0][0]) if feas.size > K else N
                ns = (ns + proc) % N
                if lst.size == 0:
                    continue
                node = int(lst[0])
                if lst.size > 1:
                    c0 = time.perf_counter()
                    rc = score(lst, sb.out)
                    c1 = time.perf_counter()
                    for k in nslots:
                        rc |= norm(k, lst, np.ascontiguousarray(sb.raw[k][lst]), nout)
                    c2 = time.perf_counter()
                    split["score"] += c1 - c0
                    split["normalize"] += c2 - c1
                    in_calls += c2 - c0
                    if rc != 0:
                        raise RuntimeError(f"{kind} fw_score / normalize rc {rc}")
                    node = int(lst[int(np.argmax(sb.total[lst]))])
                c0 = time.perf_counter()
                assume(i, node)
                split["assume"] += time.perf_counter() - c0
                in_calls += time.perf_counter() - c0
                bound += 1
            dt = time.perf_counter() - t0
            r = {"us_per_cycle": dt / count * 1e6, "us_in_calls": in_calls / count * 1e6, "cycles": count,
                 "bound": bound, "us_per_call": {k: v / count * 1e6 for k, v in split.items()}}
            if kind == "engine":   # where fw_score / fw_normalize were answered (host or device)
                d = e.diag()
                r["answered"] = {k: d[k] for k in ("fw_score_host", "fw_score_device", "fw_normalize_cached",
                                                   "fw_normalize_device")}
                e.close()
            return r

        def run_c():
            """The same engine cycles driven from C (tools/fwdrive.c): what a cgo
            host pays, without the ctypes glue of run("engine")."""
            e = engine.Engine(0)
            e.set_profile(prof)
            e.set_cluster(cluster.copy_state())
            fns = FwDriveFns(*[ctypes.cast(getattr(EL, nm), ctypes.c_void_p).value for nm in
                               ("ksim_encode_pods", "ksim_encoder_pods", "ksim_fw_prefilter", "ksim_fw_score",
                                "ksim_fw_normalize", "ksim_assume")])
            arr = (ctypes.c_void_p * n_pods)(*[ctypes.addressof(pl.c) for pl in pools])
            ns = (ctypes.c_int32 * max(1, len(nslots)))(*nslots)
            res = FwDriveResult()
            rc = DRV.fwdrive_run(ctypes.byref(fns), e.h, enc.h, arr, n_pods, ctypes.byref(opts), N, K, ns,
                                 len(nslots), prof.n_score, ctypes.byref(res))
            if rc != 0:
                raise RuntimeError(f"fwdrive rc {rc}: {EL.ksim_last_error(e.h).decode()}")
            d = e.diag()
            e.close()
            names = ("encode", "prefilter", "score", "normalize", "assume")
            return {"us_per_cycle": res.total / n_pods * 1e6, "cycles": int(res.cycles), "bound": int(res.bound),
                    "us_per_call": {nm: res.sec[q] / n_pods * 1e6 for q, nm in enumerate(names)},
                    "answered": {k: d[k] for k in ("fw_score_host", "fw_score_device", "fw_normalize_cached",
                                                   "fw_normalize_device")}}

        run("engine", min(200, n_pods))                      # warm-up (graphs, first launches)
        e_r = run("engine", n_pods)
        c_r = run_c() if DRV is not None else None
        o_r = run("oracle", min(n_pods, 1000 if n_nodes <= 100 else 300))
        row = {"nodes": n_nodes, "engine": e_r, "engine_c_driver": c_r, "oracle_cpu_1thread": o_r,
               "pool_build_us": pool_us, "engine_vs_oracle_in_calls": o_r["us_in_calls"] / e_r["us_in_calls"]}
        if DRV is not None and n_nodes >= 5000:
            ext, upd = _fw_delta_objects(nodes, pobjs, seed=5)
            row["engine_c_driver_deltas"] = _fw_run_deltas(DRV, EL, enc, cluster, prof, pools, opts, N, K, nslots,
                                                           ext, upd)
        rows.append(row)
    if DRV is not None:
        # config 3's cluster: 10,000 nodes in 3 zones, 100,000 bound pods with
        # anti-affinity terms, spreading incoming pods; the snapshot encoded
        # once, then deltas
        n3 = min(args.nodes3, 10000)
        nodes3, bound3, inc3 = gen.config3_objects(n_nodes=n3, pods_per_node=10, n_incoming=1500)
        enc3 = NativeEncoder()
        t0 = time.perf_counter()
        cl3, _ = enc3.encode_cluster(nodes3, bound3)
        full_s = time.perf_counter() - t0
        enc3.encode_pods(cl3, inc3)
        sp3 = profile.SchedulerProfile(percentage_of_nodes_to_score=0)
        prof3 = profile.compile_profile(sp3)
        pools3 = []
        for p3 in inc3:
            pl = Pool()
            pl.pod(p3)
            pl.build()
            pools3.append(pl)
        ext3, upd3 = _fw_delta_objects(nodes3, bound3, seed=6)
        N3 = cl3.n_nodes
        r3 = _fw_run_deltas(DRV, EL, enc3, cl3, prof3, pools3, opts, N3, profile.num_feasible_nodes_to_find(N3, 0),
                            [k for k, p3 in enumerate(sp3.score_plugins()) if p3.name in HAS_NORMALIZE], ext3, upd3)
        r3["full_encode_s"] = full_s
        rows.append({"nodes": N3, "bound_pods": len(bound3), "workload": "config 3 (PTS + IPA)",
                     "engine_c_driver_deltas": r3})
    best = rows[1].get("engine_c_driver_deltas") or rows[1]["engine_c_driver"] or rows[1]["engine"]
    line = {"metric": "framework_driven_cycle_us", "value": best["us_per_cycle"],
            "unit": "us per pod cycle (5000 nodes, deltas and pool build included)", "higher_is_better": False,
            "n_gpus": 1,
            "config": {"workload": "config-1 distribution, framework-driven compat cycle (drop-in)",
                       "parallelism": "single GPU"},
            "rows": rows,
            "note": "per cycle: ksim_encode_pods (native) + fw_prefilter + fw_score + fw_normalize per "
                    "NormalizeScore plugin + assume, with the copies back to host memory; value: the C driver "
                    "(tools/fwdrive.c, the calls a cgo host makes) with the incremental snapshot's work "
                    "(engine_c_driver_deltas: the pod's pool copied into a fresh allocation, the encoder bind "
                    "after Reserve, an external bound-pod add every 4 cycles and its delete 8 adds later, a node "
                    "update every 50 cycles) when built, else the Python loop, whose us_per_cycle includes the "
                    "ctypes glue; the oracle's calls take pre-compiled pods"}
    out.write(json.dumps(line) + "\n")
    out.flush()


def _fw_delta_objects(nodes, pods, seed):
    """Informer events for bench_fw's incremental run: bound pods added on
    random nodes (copies of ``pods``, renamed), node updates (allocatable cpu
    changed, same zone)."""
    import copy
    import random
    rng = random.Random(seed)
    ext = []
    for k in range(2000):
        p = copy.copy(pods[rng.randrange(len(pods))])
        p.name = f"ext-{k:06d}"
        p.node_name = nodes[rng.randrange(len(nodes))].name
        ext.append(p)
    upd = []
    for k in range(64):
        n = copy.copy(nodes[rng.randrange(len(nodes))])
        n.allocatable = dict(n.allocatable, cpu=str(rng.choice([8, 16, 24, 48])))
        upd.append(n)
    return ext, upd


def _fw_run_deltas(DRV, EL, enc, cluster, prof, pools, opts, N, K, nslots, ext, upd):
    """tools/fwdrive.c fwdrive_run_deltas on a fresh engine over ``cluster``
    (the encoder ``enc`` keeps the snapshot's membership)."""
    import ctypes
    from ksim import engine
    from ksim.nativeenc import Pool

    class Fns(ctypes.Structure):
        _fields_ = [(nm, ctypes.c_void_p) for nm in ("encode_pods", "encoder_pods", "prefilter", "score",
                                                      "normalize", "assume")]

    class DFns(ctypes.Structure):
        _fields_ = [(nm, ctypes.c_void_p) for nm in ("encoder_bind", "encoder_unbind", "encoder_update_nodes",
                                                      "encoder_old_pos", "encoder_cluster", "encoder_info",
                                                      "upsert_nodes", "forget", "encoder_changed_rows",
                                                      "update_node_rows")]

    class Deltas(ctypes.Structure):
        _fields_ = [("ext", ctypes.c_void_p), ("ext_ns", ctypes.c_void_p), ("ext_name", ctypes.c_void_p),
                    ("ext_node", ctypes.c_void_p), ("n_ext", ctypes.c_int32), ("ext_every", ctypes.c_int32),
                    ("lag", ctypes.c_int32), ("node_upd", ctypes.c_void_p), ("n_node_upd", ctypes.c_int32),
                    ("node_every", ctypes.c_int32)]

    class Res(ctypes.Structure):
        _fields_ = [("sec", ctypes.c_double * 7), ("total", ctypes.c_double)] + \
                   [(nm, ctypes.c_int64) for nm in ("bound", "cycles", "pod_adds", "pod_deletes", "node_updates",
                                                     "resends", "node_rows_in_place")]

    DRV.fwdrive_run_deltas.restype = ctypes.c_int
    DRV.fwdrive_run_deltas.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                                               ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                                               ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                                               ctypes.c_void_p]
    import numpy as np
    pos = {n: i for i, n in enumerate(cluster.node_names)}
    ext_pools, ext_ns, ext_name = [], [], []
    for p in ext:
        pl = Pool()
        pl.pod(p)
        pl.build()
        ext_pools.append(pl)
        ext_ns.append(p.namespace.encode())
        ext_name.append(p.name.encode())
    ext_node = np.array([pos[p.node_name] for p in ext], np.int32)
    upd_pools = []
    for n in upd:
        pl = Pool()
        pl.node(n)
        pl.build()
        upd_pools.append(pl)
    e = engine.Engine(0)
    e.set_profile(prof)
    e.set_cluster(cluster.copy_state())
    f = Fns(*[ctypes.cast(getattr(EL, nm), ctypes.c_void_p).value for nm in
              ("ksim_encode_pods", "ksim_encoder_pods", "ksim_fw_prefilter", "ksim_fw_score", "ksim_fw_normalize",
               "ksim_assume")])
    g = DFns(*[ctypes.cast(getattr(EL, nm), ctypes.c_void_p).value for nm in
               ("ksim_encoder_bind", "ksim_encoder_unbind", "ksim_encoder_update_nodes", "ksim_encoder_old_pos",
                "ksim_encoder_cluster", "ksim_encoder_get_info", "ksim_upsert_nodes", "ksim_forget",
                "ksim_encoder_changed_rows", "ksim_update_node_rows")])
    a_ext = (ctypes.c_void_p * len(ext_pools))(*[ctypes.addressof(pl.c) for pl in ext_pools])
    a_ns = (ctypes.c_char_p * len(ext_ns))(*ext_ns)
    a_name = (ctypes.c_char_p * len(ext_name))(*ext_name)
    a_upd = (ctypes.c_void_p * len(upd_pools))(*[ctypes.addressof(pl.c) for pl in upd_pools])
    dl = Deltas(ctypes.cast(a_ext, ctypes.c_void_p), ctypes.cast(a_ns, ctypes.c_void_p),
                ctypes.cast(a_name, ctypes.c_void_p), ext_node.ctypes.data, len(ext_pools), 4, 8,
                ctypes.cast(a_upd, ctypes.c_void_p), len(upd_pools), 50)
    n_pods = len(pools)
    arr = (ctypes.c_void_p * n_pods)(*[ctypes.addressof(pl.c) for pl in pools])
    ns = (ctypes.c_int32 * max(1, len(nslots)))(*nslots)
    res = Res()
    rc = DRV.fwdrive_run_deltas(ctypes.byref(f), ctypes.byref(g), e.h, enc.h, arr, n_pods, ctypes.byref(opts), N, K,
                                ns, len(nslots), prof.n_score, ctypes.byref(dl), ctypes.byref(res))
    if rc != 0:
        err = EL.ksim_last_error(e.h).decode() + " / " + (EL.ksim_encoder_last_error(enc.h) or b"").decode()
        raise RuntimeError(f"fwdrive_run_deltas rc {rc}: {err}")
    d = e.diag()
    e.close()
    names = ("encode", "prefilter", "score", "normalize", "assume_bind", "deltas", "pool_build")
    return {"us_per_cycle": res.total / n_pods * 1e6, "cycles": int(res.cycles), "bound": int(res.bound),
            "us_per_call": {nm: res.sec[q] / n_pods * 1e6 for q, nm in enumerate(names)},
            "events": {"pod_adds": int(res.pod_adds), "pod_deletes": int(res.pod_deletes),
                       "node_updates": int(res.node_updates), "node_rows_in_place": int(res.node_rows_in_place),
                       "resends": int(res.resends)},
            "full_encodes_after_first": 0,
            "answered": {k: d[k] for k in ("fw_score_host", "fw_score_device", "fw_normalize_cached",
                                           "fw_normalize_device")}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", type=int, default=2, choices=[1, 2, 3, 4, 5])
    ap.add_argument("--mode", choices=["p100", "adapt", "fw"], default="p100",
                    help="fw: the drop-in's framework-driven per-pod cycle (bench_fw)")
    ap.add_argument("--nodes", type=int, default=5000)
    ap.add_argument("--pods", type=int, default=50000)
    ap.add_argument("--nodes-per-gpu", type=int, default=5000)
    ap.add_argument("--nodes3", type=int, default=10000)
    ap.add_argument("--pods3", type=int, default=10000)
    ap.add_argument("--nodes4", type=int, default=100000)
    ap.add_argument("--pods4", type=int, default=1000000)
    ap.add_argument("--sweep", type=int, default=1024)
    ap.add_argument("--sweep-streams", type=int, default=8,
                    help="config 5: engines (streams) sweeping weight vectors concurrently per GPU")
    ap.add_argument("--force-shard", action="store_true",
                    help="run the node-sharded RCCL path even at N = 1 (a one-rank communicator)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--shard-mode", choices=["replicated", "nodes"], default="replicated",
                    help="configs 2 / 4 (P100) over N > 1 GPUs: replicated snapshot with the evaluation split by node range "
                         "(one collective per batch), or node shards (two)")
    ap.add_argument("--python-encode", action="store_true",
                    help="compile configs 1 / 3 with the Python encoder (ksim/encode.py) instead of the native one")
    ap.add_argument("--host-match", action="store_true",
                    help="config 3: match the count classes' selectors on the host instead of ksim_match_terms")
    ap.add_argument("--no-adapt", action="store_true", help="skip the secondary ADAPT measurement (config 2)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample per thread count")
    ap.add_argument("--cpu-threads", default="sweep",
                    help='CPU baseline threads: "sweep" (16, 64, every logical CPU; best reported) or a comma list')
    args = ap.parse_args()

    # The JSON line goes to the original stdout; native libraries (RCCL's
    # version banner) that write to fd 1 land on stderr instead.
    out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))

    # torch first: libksim_engine.so then binds to the HIP runtime torch already
    # loaded (same SONAME), so both share one runtime; the reverse order leaves
    # torch without a device (probed in tools/rt_probe.py).
    import torch
    torch.cuda.init()
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    from ksim import engine, gen, profile, shard

    engine.lib()
    if args.mode == "fw":
        bench_fw(args, out)
        return
    cfg = args.config
    cluster, pods, sp, desc, sharded, scaling = build(cfg, args, rank, world)
    prof = profile.compile_profile(sp)
    if args.force_shard and cfg in (2, 3, 4):
        sharded = True
        desc += " [sharded path forced]"

    if sharded:
        uid = shard.broadcast_unique_id(dist, rank) if world > 1 else engine.comm_unique_id()
        if cfg in (2, 4) and args.mode == "p100" and args.shard_mode == "replicated":
            # every rank holds the whole snapshot, the batch top-T is split:
            # one all-gather per batch instead of an all-gather + all-reduce
            eng = shard.replicated_engine(cluster, prof, rank, world, local, uid)
            desc += ", replicated snapshot (evaluation split by node range)"
        else:
            eng = shard.sharded_engine(cluster, prof, rank, world, local, uid)
    else:
        eng = engine.Engine(local)
        eng.set_profile(prof)
        eng.set_cluster(cluster)
    eng.load_pods(pods)

    if cfg == 5:
        from ksim import sweep
        weights = gen.config5_weights(args.sweep)[sweep.rank_vectors(args.sweep, rank, world)]
        names = [p.name for p in sp.score_plugins()]
        profs = [profile.compile_profile(sp.with_weights({n: int(x) for n, x in zip(names, w)})) for w in weights]
        # Independent weight vectors run concurrently: one engine (own stream,
        # own copy of the 5,000-node snapshot) per host thread, so one sweep's
        # latency-bound batch kernels overlap another's (ctypes releases the GIL).
        engs = [eng]
        for _ in range(max(1, args.sweep_streams) - 1):
            e = engine.Engine(local)
            e.set_profile(prof)
            e.set_cluster(cluster)
            e.load_pods(pods)
            engs.append(e)
        from concurrent.futures import ThreadPoolExecutor
        pool = ThreadPoolExecutor(len(engs))

        def run_part(j):
            e, agg, rows = engs[j], None, []
            for pr in profs[j::len(engs)]:
                e.set_profile(pr)
                e.load_pods(pods)
                e.reset_cluster()
                chosen, st = e.schedule_loaded(0, pods.n_pods)       # the placements of this vector
                rows.append(chosen)
                if agg is None:
                    agg = st
                else:
                    for f in ("pods", "scheduled", "unschedulable", "evals", "batches", "truncations",
                              "perpod_cycles"):
                        setattr(agg, f, getattr(agg, f) + getattr(st, f))
                    agg.device_ms += st.device_ms
            return agg, rows

        def step():
            res = list(pool.map(run_part, range(len(engs))))
            # C4: every vector's placements, gathered to rank 0 in global order
            local_rows = sweep.order_engine_results([r for _, r in res], len(profs))
            SWEEP["placements"] = sweep.gather_placements(local_rows, rank, world, args.sweep, dist,
                                                          "cuda" if dist is not None else None, n_pods=pods.n_pods)
            parts = [p for p, _ in res if p is not None]
            agg = parts[0]
            for st in parts[1:]:
                for f in ("pods", "scheduled", "unschedulable", "evals", "batches", "truncations", "perpod_cycles"):
                    setattr(agg, f, getattr(agg, f) + getattr(st, f))
                agg.device_ms += st.device_ms
            return agg
    else:
        def step():
            eng.reset_cluster()
            _, st = eng.schedule_loaded(0, pods.n_pods, want_chosen=False)
            return st

    for i in range(args.warmup):
        st = step()
        log(f"[rank {rank}] warmup {i}: {st.device_ms:.1f} ms device, {st.evals} evals")

    def barrier():
        if dist is not None:
            dist.barrier()

    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    evals = sched = cycles = 0
    for k in range(args.steps):
        st = step()
        evals += st.evals
        sched += st.scheduled
        cycles += st.pods
        log(f"[rank {rank}] step {k}: {st.device_ms:.1f} ms device")
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0

    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        c = torch.tensor([evals, cycles], dtype=torch.float64, device="cuda")
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
        evals = int(c[0].item())
        # sharded: every rank ran the same cycles (count them once)
        cycles = int(c[1].item()) // (world if sharded else 1)

    # Roofline of the evaluation kernel: per-kernel HIP events on an engine
    # stream, over this rank's nodes (a sharded rank times its own shard).
    geom = engine.batch_geometry()
    from ksim.profile import num_feasible_nodes_to_find
    geom["adapt_k"] = num_feasible_nodes_to_find(cluster.n_nodes, sp.percentage_of_nodes_to_score)
    if st.batches > 0 and st.perpod_cycles == 0:
        geom["tb_pods_per_batch"] = st.pods / st.batches   # the topology batches' mean size (config 3)
    if sharded:
        base, cnt = shard.partition(cluster.n_nodes, world)[rank]
        keng = engine.Engine(local)
        keng.set_profile(profile.compile_profile(sp if cfg != 5 else sp))
        keng.set_cluster(cluster.shard(base, cnt))
        keng.load_pods(pods)
        knodes = cnt
    else:
        keng, knodes = eng, cluster.n_nodes
        keng.reset_cluster()
    kt_pods = min(pods.n_pods, 50000 if cfg != 3 else 2000)
    kt = keng.time_kernels(0, kt_pods)
    by_time = max(kt, key=lambda k: kt[k][0] * kt[k][1])      # largest share of device time
    dominant = by_time                                        # the roofline prices the by-time dominant kernel
    n_norm = sum(1 for p in sp.score_plugins()
                 if p.name in ("TaintToleration", "NodeAffinity", "PodTopologySpread", "InterPodAffinity"))
    alg = kernel_alg_bytes(dominant, knodes, n_norm, geom)
    # the evaluation kernel's mean duration: HIP events around back-to-back
    # launches on the engine's stream (no event records between launches,
    # which add 2-4 us each in the per-kernel table above)
    ktab = kernel_table(kt, kt_pods, pods.n_pods, elapsed / args.steps * 1e3, knodes, n_norm, geom, sharded,
                        concurrent=cfg == 5)
    avg_ms, timing = ktab[dominant]["avg_ms"], ("per-kernel HIP events inside the run, reconciled with the "
                                                "graph-replayed step (kernels table)")
    try:
        name, ms = keng.time_eval(0, 200)
        if name == dominant:
            avg_ms, timing = ms, "HIP events around 200 back-to-back launches (engine stream)"
    except engine.KsimError:
        pass
    # the kernel's in-graph duration from the committed rocprofv3 summary of
    # this line (profiles/kernel_ms.json): the graph-replayed step interleaves
    # the batch's kernels, whose other working sets the back-to-back launches
    # above do not evict; when the two differ by more than 5 % the roofline is
    # priced at the in-graph figure, the live one kept beside it
    live_ms, live_timing = avg_ms, timing
    ke = _profile_entry("kernel_ms.json", dominant, knodes, cfg, mode=args.mode)
    if ke and ke.get("avg_ms") and abs(ke["avg_ms"] / avg_ms - 1) > 0.05:
        avg_ms, timing = ke["avg_ms"], f"rocprofv3 kernel trace, in-graph mean ({ke.get('source')})"
    achieved = alg / (avg_ms * 1e-3) / 1e9
    # PMC measurements committed under profiles/ (by kernel and size): HBM
    # bytes per launch (traffic.json) and vector instructions per launch
    # (valu.json), priced with this run's launch time
    te = _profile_entry("traffic.json", dominant, knodes, cfg)
    traffic = te.get("hbm_bytes_per_launch") if te else None
    ve = _profile_entry("valu.json", dominant, knodes, cfg)
    valu = None
    if ve and ve.get("valu_insts_per_launch"):
        g = ve["valu_insts_per_launch"] / (avg_ms * 1e-3) / 1e9
        per_eval = ve.get("valu_insts_per_eval_lane")
        if per_eval is None and dominant in ("k_batch_top_commit", "k_batch_top", "k_adapt_top"):
            # one block per pod of the batch, each over the evaluated node range
            per_eval = ve["valu_insts_per_launch"] * 64 / (geom["pods_per_batch"] *
                                                           (geom["adapt_k"] if dominant == "k_adapt_top" else knodes))
        valu = {"achieved": g, "peak": VALU_PEAK_G, "unit": "G wave-instructions/s", "frac": g / VALU_PEAK_G,
                "valu_insts_per_launch": ve["valu_insts_per_launch"],
                "salu_insts_per_launch": ve.get("salu_insts_per_launch"),
                "valu_insts_per_eval_lane": per_eval, "source": ve.get("source")}
        act, wcyc, waves = (ve.get("valu_active_quad_cycles_per_launch"), ve.get("wave_quad_cycles_per_launch"),
                            ve.get("waves_per_launch"))
        fills = ve.get("waves_per_launch", 0) >= 256 * 4     # at least one wave per SIMD of the chip
        if act and wcyc and waves and fills:
            # SQ_ACTIVE_INST_VALU per SIMD over the mean wave lifetime (SQ_WAVE_CYCLES / SQ_WAVES): the
            # share of the launch its SIMDs spend issuing VALU work (1,024 SIMDs, every one holding waves
            # of the launch for its whole duration; a 64-bit or f64 op holds the SIMD longer than the
            # 2-cycle issue slot the "frac" above prices every instruction at)
            valu["busy_frac_pmc"] = (act / 1024.0) / (wcyc / waves)
            valu["wait_mem_frac_pmc"] = ve.get("wait_any_quad_cycles_per_launch", 0) / wcyc
            valu["wait_issue_frac_pmc"] = ve.get("wait_inst_any_quad_cycles_per_launch", 0) / wcyc
            if ve.get("valu_mix_per_launch"):
                valu["mix_per_launch"] = ve["valu_mix_per_launch"]

    seeds = {1: "0x4B53494D0001", 2: "0x4B53494D0002", 3: "0x4B53494D0003", 4: "0x4B53494D0004", 5: "0x4B53494D0002/0005"}
    result = {
        "metric": "pod x node filter+score evals/sec",
        "value": evals / elapsed,
        "unit": "evals/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "int64",
        "data": f"synthetic (SplitMix64 seed {seeds[cfg]})",
        "config": {"workload": desc, "nodes": cluster.n_nodes, "pods": pods.n_pods, "mode": args.mode,
                   "parallelism": (f"node-sharded over {world} GPUs (RCCL)" if sharded else
                                   f"{world} independent replicas" if world > 1 else "single GPU")},
        "pods_per_s": cycles / elapsed,
        "kernels": ktab,
        "batch_stats": {"batches": st.batches, "truncations": st.truncations,
                        "perpod_cycles": st.perpod_cycles},
        "roofline": dict(roofline_entry(dominant, achieved, traffic, alg, avg_ms, timing, knodes, by_time, valu),
                         live_avg_launch_ms=live_ms, live_timing=live_timing),
        "batch_geometry": geom,
    }
    if HOST_COMPILE:
        result["host_compile"] = HOST_COMPILE
    if SWEEP.get("placements") is not None:
        from ksim import sweep
        pl = SWEEP["placements"]
        result["sweep"] = {"vectors": int(pl.shape[0]), "pods": int(pl.shape[1]),
                           "placements_gathered": "rank 0, [vectors][pods] int32, one all-gather per step (C4)",
                           "scheduled_per_vector_mean": float((pl >= 0).sum(axis=1).mean()),
                           "digest": sweep.placement_digest(pl)}
    if cfg == 2 and world == 1 and args.mode == "p100" and not args.no_adapt:
        # the simulator's forced default (percentageOfNodesToScore = 0) on the
        # same cluster and pods, timed the same way: a secondary line item
        asp = profile.SchedulerProfile(percentage_of_nodes_to_score=0)
        aeng = engine.Engine(local)
        aeng.set_profile(profile.compile_profile(asp))
        aeng.set_cluster(cluster)
        aeng.load_pods(pods)
        aeng.schedule_loaded(0, pods.n_pods, want_chosen=False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        aev = 0
        for _ in range(args.steps):
            aeng.reset_cluster()
            _, ast = aeng.schedule_loaded(0, pods.n_pods, want_chosen=False)
            aev += ast.evals
        torch.cuda.synchronize()
        adt = time.perf_counter() - t0
        result["adapt"] = {"mode": "ADAPT (percentageOfNodesToScore 0, K = %d of %d nodes)" %
                           (_k_adapt(cluster.n_nodes), cluster.n_nodes),
                           "value": aev / adt, "unit": "evals/s", "pods_per_s": pods.n_pods * args.steps / adt,
                           "ms_per_step": adt / args.steps * 1e3, "batches": ast.batches,
                           "perpod_cycles": ast.perpod_cycles}
        log(f"[rank 0] adapt: {aev / adt:.3e} evals/s")
    if rank == 0 and world == 1 and not args.no_cpu:
        log("[rank 0] cpu baseline ...")
        result["cpu_baseline"] = cpu_baseline(cluster, pods, sp, args.cpu_seconds, cpu_threads_sweep(args.cpu_threads),
                                              f"config-{cfg}")
        result["vs_cpu"] = result["value"] / result["cpu_baseline"]["value"]
    if rank == 0:
        print(json.dumps(result), file=out, flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
