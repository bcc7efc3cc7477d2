#!/usr/bin/env python3
"""bench.py — pod x node filter+score evaluations/s of the scheduling cycle on MI355X.

Metric and config: BASELINE.json ("pod x node filter+score evals/sec and pods
scheduled/sec"; configs[1] = default profile, 5,000 nodes x 50,000 pods on one
MI355X).  One step = one full pass of that workload: reset the node snapshot
to empty (device-side copy) and run all 50,000 scheduling cycles (Filter over
every node, Score, NormalizeScore, weights, selectHost, bind) on the engine.
Inputs (cluster SoA + pod queue) are resident in HBM before the timed region.

  python bench.py [--gpus N --steps K --warmup W] [--mode p100|adapt]

N > 1 (torch.distributed.run, one rank per GPU): every rank runs the same
workload under its own score-weight vector (config 5 policy sweep: independent
profiles per GPU, no data-path collective) -> "scaling": "weak".
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
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E peak (MI355X_MICROARCH.md chip table)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def kernel_alg_bytes(name: str, n_nodes: int, n_norm: int, geom: dict) -> int:
    """Algorithmic HBM bytes per launch of each kernel:
    the node rows an evaluation kernel must read once per pod it evaluates;
    the small bookkeeping kernels are priced by the keys they move."""
    B, T = geom["pods_per_batch"], geom["top_t"]
    tiles = (n_nodes + geom["tile_nodes"] - 1) // geom["tile_nodes"]
    if name == "k_filter_score":
        return B_EVAL * n_nodes                       # one node row per pod x node eval
    if name == "k_finalize":
        return n_nodes * (1 + 8 + 8 * n_norm)         # fail code + partial total + normalized raws
    if name == "k_batch_eval":
        return B_EVAL * n_nodes * B                   # B pods x N nodes evals per launch
    if name == "k_batch_merge":
        return 8 * B * (tiles * geom["tile_cand"] + T)
    if name == "k_batch_chain":
        return 8 * B * T * 2
    if name == "k_batch_pairs":
        return B * (B - 1) // 2 * B_EVAL + 8 * B * 3      # one bound-row re-eval per pod pair
    return 0


# the kernel that carries the pod x node evaluations on each path
EVAL_KERNELS = ("k_batch_eval", "k_filter_score")


def cpu_baseline(cluster, pods, sp, seconds: float, threads: int) -> dict:
    """The CPU restatement (oracle, OpenMP over nodes) on a bounded sample."""
    from ksim import profile
    from oracle.oracle import Oracle
    prof = profile.compile_profile(sp)
    o = Oracle(cluster.copy_state(), prof)
    t = time.perf_counter()
    _, st = o.schedule(pods, 0, 100, nthreads=threads)
    dt = time.perf_counter() - t
    n = int(min(pods.n_pods - 100, max(100, (seconds / max(dt, 1e-6)) * 100)))
    t = time.perf_counter()
    _, st2 = o.schedule(pods, 100, n, nthreads=threads)
    dt2 = time.perf_counter() - t
    return {"value": st2.evals / dt2, "unit": "pod x node evals/s", "cores": threads, "kind": "port",
            "pods_per_s": n / dt2,
            "sample": f"config-2 pods 100..{100 + n} ({n} cycles, {st2.evals} evals) after 100 warm cycles "
                      f"from the empty cluster, same profile/mode, oracle/ksim_oracle.c OpenMP {threads} threads, "
                      f"{dt2:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--mode", choices=["p100", "adapt"], default="p100")
    ap.add_argument("--nodes", type=int, default=5000)
    ap.add_argument("--pods", type=int, default=50000)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--cpu-threads", type=int, default=min(16, os.cpu_count() or 1))
    args = ap.parse_args()

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
    from ksim import engine, gen, profile
    engine.lib()

    cluster, pods = gen.config2(args.nodes, args.pods)
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=100 if args.mode == "p100" else 0)
    if world > 1:
        w = gen.config5_weights()[rank % 1024]
        names = [p.name for p in sp.score_plugins()]
        sp = sp.with_weights({n: int(x) for n, x in zip(names, w)})
    prof = profile.compile_profile(sp)

    eng = engine.Engine(local)
    eng.set_profile(prof)
    eng.set_cluster(cluster)
    eng.load_pods(pods)

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
        evals, cycles = int(c[0].item()), int(c[1].item())

    # Roofline of the dominant kernel: per-kernel HIP events on the engine stream.
    eng.reset_cluster()
    kt = eng.time_kernels(0, min(pods.n_pods, 8192))
    geom = engine.batch_geometry()
    by_time = max(kt, key=lambda k: kt[k][0] * kt[k][1])      # largest share of device time
    dominant = next((k for k in EVAL_KERNELS if k in kt), by_time)
    n_norm = sum(1 for p in sp.score_plugins()
                 if p.name in ("TaintToleration", "NodeAffinity", "PodTopologySpread", "InterPodAffinity"))
    alg = kernel_alg_bytes(dominant, cluster.n_nodes, n_norm, geom)
    achieved = alg / (kt[dominant][0] * 1e-3) / 1e9
    traffic = None
    tpath = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tpath):
        try:
            tj = json.load(open(tpath))
            if tj.get("kernel") == dominant and tj.get("nodes") == cluster.n_nodes:
                traffic = tj.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None

    result = {
        "metric": "pod x node filter+score evals/sec",
        "value": evals / elapsed,
        "unit": "evals/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic (SplitMix64 seed 0x4B53494D0002)",
        "config": {"workload": f"config2: default profile, {cluster.n_nodes} nodes x {pods.n_pods} pods, "
                               f"{args.mode.upper()} (percentageOfNodesToScore={prof.percentage_of_nodes_to_score})",
                   "nodes": cluster.n_nodes, "pods": pods.n_pods, "mode": args.mode,
                   "parallelism": "replicas (per-GPU score-weight profiles)" if world > 1 else "single GPU"},
        "pods_per_s": cycles / elapsed,
        "kernels": {k: {"avg_ms": v[0], "launches": v[1],
                        "alg_GBps": kernel_alg_bytes(k, cluster.n_nodes, n_norm, geom) / (v[0] * 1e-3) / 1e9}
                    for k, v in kt.items()},
        "batch_stats": {"batches": st.batches, "truncations": st.truncations,
                        "perpod_cycles": st.perpod_cycles},
        "roofline": {"bound": "hbm", "kernel": dominant, "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "alg_bytes_per_launch": alg, "avg_launch_ms": kt[dominant][0],
                     "dominant_by_time": by_time},
        "batch_geometry": geom,
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        log("[rank 0] cpu baseline ...")
        result["cpu_baseline"] = cpu_baseline(cluster, pods, sp, args.cpu_seconds, args.cpu_threads)
        result["vs_cpu"] = result["value"] / result["cpu_baseline"]["value"]
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
