"""Numpy model of the node-sharded batch protocol.

TEST INFRASTRUCTURE ONLY: tests/test_shard_cpu.py runs it on world_size-2
``gloo`` process groups on the CPU and checks its placements against the C
oracle on the whole cluster.  It restates, rank by rank, what
csrc/ksim_batch.hip does between the two exchanges:

  per shard : keys of B pods x local nodes under the batch-start snapshot
              -> sorted top-T per pod + "complete" (every feasible node listed)
  all-gather: every shard's lists                        (ncclAllGather)
  global    : keys >= the last listed key of every incomplete shard are the
              provable global prefix (k_batch_gmerge)
  chain     : pod i guesses its best node not guessed earlier (k_batch_chain)
  pairs     : key of pod j on pod k's guess after pod k binds, owner shard only
  all-reduce: max over shards                             (ncclAllReduce MAX)
  commit    : up to the first pod whose exact choice is not its guess; the
              owner shard applies the binds (k_batch_commit)

Replicated sharding (ksim_set_eval_range, ``eval_range``): the Shard holds
every node, the top-T covers the rank's range only, the pair keys of every
guess are local (no all-reduce) and every rank binds every placement.

Batchable pods only (bare pods: Fit filter + LeastAllocated +
BalancedAllocation vary over nodes, every normalized plugin is constant).
Keys stay below 2^63 (totals < 2^19), so int64 tensors carry them.
"""
from __future__ import annotations

import numpy as np

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
NODE_MASK = (1 << 18) - 1


def _splitmix(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def tb_keys(total: np.ndarray, seed: int, seq: int, nodes: np.ndarray) -> np.ndarray:
    x = np.uint64(seed) ^ (np.uint64(seq) << np.uint64(20)) ^ nodes.astype(np.uint64)
    h = _splitmix(x) >> np.uint64(38)
    return ((total.astype(np.uint64) << np.uint64(44)) | (h << np.uint64(18)) |
            (np.uint64(NODE_MASK) - nodes.astype(np.uint64)))


class Shard:
    """One rank's nodes [base, base + n) of a bare config-2 style cluster."""

    def __init__(self, cluster, base: int, count: int):
        sl = slice(base, base + count)
        self.base, self.n = base, count
        self.alloc_cpu = cluster.alloc_cpu[sl].astype(np.int64)
        self.alloc_mem = cluster.alloc_mem[sl].astype(np.int64)
        self.alloc_pods = cluster.alloc_pods[sl].astype(np.int64)
        self.req_cpu = cluster.req_cpu[sl].astype(np.int64).copy()
        self.req_mem = cluster.req_mem[sl].astype(np.int64).copy()
        self.nz_cpu = cluster.nz_cpu[sl].astype(np.int64).copy()
        self.nz_mem = cluster.nz_mem[sl].astype(np.int64).copy()
        self.num_pods = cluster.num_pods[sl].astype(np.int64).copy()

    def keys(self, pod, rows, seed, seq, const, w_fit, w_ba, extra=None) -> np.ndarray:
        """TB keys of ``pod`` on local ``rows`` (0 = infeasible).  ``extra``:
        (row, pod) already bound there (the pair check)."""
        rc, rm = self.req_cpu[rows].copy(), self.req_mem[rows].copy()
        zc, zm = self.nz_cpu[rows].copy(), self.nz_mem[rows].copy()
        npods = self.num_pods[rows].copy()
        if extra is not None:
            rc += extra["req_cpu"]
            rm += extra["req_mem"]
            zc += extra["nz_cpu"]
            zm += extra["nz_mem"]
            npods += 1
        ac, am = self.alloc_cpu[rows], self.alloc_mem[rows]
        fits = (npods + 1 <= self.alloc_pods[rows]) & (pod["req_cpu"] <= ac - rc) & (pod["req_mem"] <= am - rm)
        la = np.zeros(len(rows), np.int64)
        cnt = np.zeros(len(rows), np.int64)
        for alloc, req in ((ac, zc + pod["nz_cpu"]), (am, zm + pod["nz_mem"])):
            ok = alloc != 0
            s = np.where(req > alloc, 0, ((alloc - req) * 100) // np.where(ok, alloc, 1))
            la += np.where(ok, s, 0)
            cnt += ok
        la = np.where(cnt > 0, la // np.maximum(cnt, 1), 0)
        f0 = np.minimum(1.0, (rc + pod["req_cpu"]).astype(np.float64) / ac.astype(np.float64))
        f1 = np.minimum(1.0, (rm + pod["req_mem"]).astype(np.float64) / am.astype(np.float64))
        ba = ((1 - np.abs((f0 - f1) / 2)) * 100).astype(np.int64)
        total = const + w_fit * la + w_ba * ba
        k = tb_keys(total, seed, seq, self.base + np.asarray(rows, np.int64))
        return np.where(fits, k, np.uint64(0))

    def bind(self, row: int, pod) -> None:
        self.req_cpu[row] += pod["req_cpu"]
        self.req_mem[row] += pod["req_mem"]
        self.nz_cpu[row] += pod["nz_cpu"]
        self.nz_mem[row] += pod["nz_mem"]
        self.num_pods[row] += 1


def global_merge(lists, completes, T: int):
    """k_batch_gmerge: lists[s] = shard s's keys (descending, <= T)."""
    thr = 0
    for keys, comp in zip(lists, completes):
        if not comp and len(keys):
            thr = max(thr, int(keys[-1]))
    allk = sorted((int(k) for keys in lists for k in keys if int(k) >= thr and int(k) != 0), reverse=True)
    complete = all(completes) and len(allk) <= T
    return allk[:T], complete


def schedule(pods, shard: Shard, rank: int, world: int, dist, n_total: int, seed: int, const: int,
             w_fit: int = 1, w_ba: int = 1, B: int = 16, T: int = 3, eval_range=None):
    """Run every pod through the sharded protocol; returns global placements.
    ``eval_range`` = (lo, hi): replicated sharding (the Shard is the whole
    cluster, this rank's top-T covers rows [lo, hi))."""
    import torch
    P = pods.n_pods
    chosen = np.full(P, -1, np.int64)
    cursor, seq0 = 0, 0
    rows = np.arange(shard.n) if eval_range is None else np.arange(*eval_range)
    while cursor < P:
        nb = min(B, P - cursor)
        # per shard: top-T per pod under the batch-start snapshot
        rec = np.zeros((nb, T + 1), np.int64)
        for j in range(nb):
            k = shard.keys(pods.pods[cursor + j], rows, seed, seq0 + j, const, w_fit, w_ba)
            order = np.sort(k[k != 0])[::-1]
            rec[j, :min(T, len(order))] = order[:T].astype(np.int64)
            rec[j, T] = min(T, len(order)) | ((1 if len(order) <= T else 0) << 32)
        gathered = [torch.zeros(nb * (T + 1), dtype=torch.int64) for _ in range(world)]
        dist.all_gather(gathered, torch.from_numpy(rec.reshape(-1)))
        g = [x.numpy().reshape(nb, T + 1) for x in gathered]
        # global lists + chain (identical on every rank)
        guessed, gkey, nchain = set(), [0] * nb, nb
        for j in range(nb):
            lists = [g[s][j, :g[s][j, T] & 0xFFFFFFFF] for s in range(world)]
            comps = [bool(g[s][j, T] >> 32) for s in range(world)]
            glist, gcomplete = global_merge(lists, comps, T)
            pick = next((k for k in glist if NODE_MASK - (k & NODE_MASK) not in guessed), None)
            if pick is None:
                if not gcomplete:
                    nchain = j
                    break
                continue
            guessed.add(NODE_MASK - (pick & NODE_MASK))
            gkey[j] = pick
        # pair keys of owned guesses, max over shards
        pmax = np.zeros(nb, np.int64)
        for j in range(nchain):
            for k in range(j):
                if not gkey[k]:
                    continue
                row = NODE_MASK - (gkey[k] & NODE_MASK) - shard.base
                if 0 <= row < shard.n:
                    v = shard.keys(pods.pods[cursor + j], np.array([row]), seed, seq0 + j, const, w_fit, w_ba,
                                   extra=pods.pods[cursor + k])[0]
                    pmax[j] = max(pmax[j], int(v))
        if eval_range is None:                          # replicas: every guess is local
            t = torch.from_numpy(pmax)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            pmax = t.numpy()
        istar = next((j for j in range(nchain) if pmax[j] > gkey[j]), nchain)
        committed = istar + 1 if istar < nchain else nchain
        inode = NODE_MASK - (int(pmax[istar]) & NODE_MASK) if istar < nchain else -1
        for j in range(committed):
            node = inode if j == istar else (NODE_MASK - (gkey[j] & NODE_MASK) if gkey[j] else -1)
            chosen[cursor + j] = node
            if j < istar and gkey[j]:
                row = node - shard.base
                if 0 <= row < shard.n:
                    shard.bind(row, pods.pods[cursor + j])
                    if node == inode:
                        shard.bind(row, pods.pods[cursor + istar])
        cursor += committed
        seq0 += committed
    return chosen


def num_feasible_nodes_to_find(n: int, pct: int) -> int:
    """numFeasibleNodesToFind."""
    if n < 100 or pct >= 100:
        return n
    p = pct if pct > 0 else max(5, 50 - n // 125)
    return max(n * p // 100, 100)


def window(counts, rank: int, n_total: int, K: int, base: int, n: int, start: int, fail_ok: np.ndarray):
    """k_window_sh: the global cut from every shard's (feasible >= start,
    feasible < start) counts.  Returns (kend, cutslot): this shard keeps its
    feasible nodes at scan position < kend; cutslot = 1 + the cut's scan
    position on the shard that holds it, else 0."""
    T = int(counts.sum())
    all_hi = int(counts[:, 0].sum())
    bhi = int(counts[:rank, 0].sum())
    blo = all_hi + int(counts[:rank, 1].sum())
    fhi, flo = int(counts[rank, 0]), int(counts[rank, 1])
    split = min(n, max(0, start - base))
    if T <= K:
        return n_total, 0
    if bhi <= K < bhi + fhi:
        x = split + int(np.flatnonzero(fail_ok[split:])[K - bhi])
        return base + x - start, base + x - start + 1
    if blo <= K < blo + flo:
        x = int(np.flatnonzero(fail_ok[:split])[K - blo])
        return base + x - start + n_total, base + x - start + n_total + 1
    if blo + flo <= K:
        return n_total, 0
    if bhi + fhi <= K and split < n:
        return base + n - start, 0
    return 0, 0


def schedule_perpod(pods, shard: Shard, rank: int, world: int, dist, n_total: int, seed: int, const: int,
                    w_fit: int, w_ba: int, pct: int):
    """The sharded per-pod cycle (csrc/ksim_kernels.hip §C) for bare pods:
    all-gather of the two run counts -> global window; all-reduce (max) of
    (TB key, cutslot); the owner binds.  Returns (placements, local evals,
    nextStartNodeIndex)."""
    import torch
    K = num_feasible_nodes_to_find(n_total, pct)
    chosen = np.full(pods.n_pods, -1, np.int64)
    rows = np.arange(shard.n)
    g = shard.base + rows
    start, evals = 0, 0
    for j in range(pods.n_pods):
        pod = pods.pods[j]
        keys = shard.keys(pod, rows, seed, j, const, w_fit, w_ba)
        ok = keys != 0
        split = min(shard.n, max(0, start - shard.base))
        mine = torch.tensor([int(ok[split:].sum()), int(ok[:split].sum())], dtype=torch.int64)
        gathered = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(gathered, mine)
        counts = torch.stack(gathered).numpy()
        kend, cutslot = window(counts, rank, n_total, K, shard.base, shard.n, start, ok)
        nf = min(int(counts.sum()), K)
        pos = (g - start) % n_total
        kept = ok & (pos < kend)
        if nf == 1:        # schedulePod: the single feasible node, unscored
            keys = tb_keys(np.zeros(shard.n, np.int64), seed, j, g)
        best = int(keys[kept].max()) if kept.any() else 0
        t = torch.tensor([best, cutslot], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        best, cutslot = int(t[0]), int(t[1])
        evaluated = cutslot if cutslot else n_total
        evals += int((pos < evaluated).sum())
        start = (start + (cutslot - 1 if cutslot else n_total)) % n_total
        if best:
            node = NODE_MASK - (best & NODE_MASK)
            chosen[j] = node
            if shard.base <= node < shard.base + shard.n:
                shard.bind(node - shard.base, pod)
    return chosen, evals, start


def _find_cut(mask: np.ndarray, s: int, k: int) -> int:
    """find_cut (csrc/ksim_adapt.hip): offset from s (circular) of the k-th
    (0-based) feasible node of the boolean node mask, or -1."""
    order = np.concatenate([np.arange(s, len(mask)), np.arange(0, s)])
    idx = np.flatnonzero(mask[order])
    return int(idx[k]) if len(idx) > k else -1


def schedule_adapt(pods, shard: Shard, rank: int, world: int, dist, n_total: int, seed: int, const: int,
                   w_fit: int = 1, w_ba: int = 1, B: int = 16, T: int = 3):
    """The node-sharded ADAPT batch (csrc/ksim_adapt.hip "node-sharded ADAPT
    batch"), rank by rank: each shard's S0 feasibility of its nodes is
    all-gathered into the global bitmap; the scan windows follow from it
    (pod j+1 starts where pod j's scan stopped); each shard lists the top-T of
    the kept nodes it holds; lists all-gathered and merged, the chain run; each
    shard scores the guesses it owns (pair key, and "broken" when the bind
    makes an S0-feasible node at or before the cut infeasible: that pod's
    window would shift); max all-reduce of both; the commit stops before the
    first broken pod and validates the rest as on the P100 path.  Returns
    (global placements, evaluations on this shard, nextStartNodeIndex)."""
    import torch
    P = pods.n_pods
    K = num_feasible_nodes_to_find(n_total, 0)
    chosen = np.full(P, -1, np.int64)
    cursor, seq0, start, evals = 0, 0, 0, 0
    rows = np.arange(shard.n)
    lo, hi = shard.base, shard.base + shard.n
    while cursor < P:
        nb = min(B, P - cursor)
        # S0 bitmaps: this shard's nodes, all-gathered into the global order
        sizes = _shard_sizes(dist, shard.n, world)
        cmax = max(sizes)                          # equal-size all-gather: padded rows (the W words)
        loc = np.zeros((nb, cmax), np.int64)
        for j in range(nb):
            loc[j, :shard.n] = shard.keys(pods.pods[cursor + j], rows, seed, seq0 + j, const, w_fit, w_ba) != 0
        parts = [torch.zeros(nb * cmax, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(parts, torch.from_numpy(loc.reshape(-1)))
        gmask = np.concatenate([x.numpy().reshape(nb, cmax)[:, :sizes[r]] for r, x in enumerate(parts)],
                               axis=1).astype(bool)
        # windows (every rank alike)
        wins, s = [], start
        for j in range(nb):
            cut = _find_cut(gmask[j], s, K)
            wins.append((s, cut))
            s = (s + (cut if cut >= 0 else n_total)) % n_total
        # this shard's kept nodes -> its top-T record per pod
        rec = np.zeros((nb, T + 1), np.int64)
        for j, (s, cut) in enumerate(wins):
            kend = cut if cut >= 0 else n_total
            g = (s + np.arange(kend)) % n_total
            g = g[(g >= lo) & (g < hi)]
            g = g[gmask[j][g]]
            k = shard.keys(pods.pods[cursor + j], g - lo, seed, seq0 + j, const, w_fit, w_ba) if len(g) else \
                np.zeros(0, np.uint64)
            order = np.sort(k[k != 0])[::-1]
            rec[j, :min(T, len(order))] = order[:T].astype(np.int64)
            rec[j, T] = min(T, len(order)) | ((1 if len(order) <= T else 0) << 32)
        gathered = [torch.zeros(nb * (T + 1), dtype=torch.int64) for _ in range(world)]
        dist.all_gather(gathered, torch.from_numpy(rec.reshape(-1)))
        gr = [x.numpy().reshape(nb, T + 1) for x in gathered]
        guessed, gkey, nchain = set(), [0] * nb, nb
        for j in range(nb):
            lists = [gr[r][j, :gr[r][j, T] & 0xFFFFFFFF] for r in range(world)]
            comps = [bool(gr[r][j, T] >> 32) for r in range(world)]
            glist, gcomplete = global_merge(lists, comps, T)
            pick = next((k for k in glist if NODE_MASK - (k & NODE_MASK) not in guessed), None)
            if pick is None:
                if not gcomplete:
                    nchain = j
                    break
                continue
            guessed.add(NODE_MASK - (pick & NODE_MASK))
            gkey[j] = pick
        # owned guesses: pair keys and broken flags, max over shards
        px = np.zeros(2 * nb, np.int64)
        for j in range(nchain):
            s, cut = wins[j]
            kend = cut if cut >= 0 else n_total
            for k in range(j):
                if not gkey[k]:
                    continue
                node = NODE_MASK - (gkey[k] & NODE_MASK)
                if not lo <= node < hi:
                    continue
                off = (node - s) % n_total
                if off < kend or off == cut:
                    v = int(shard.keys(pods.pods[cursor + j], np.array([node - lo]), seed, seq0 + j, const, w_fit,
                                       w_ba, extra=pods.pods[cursor + k])[0])
                    if cut >= 0 and gmask[j][node] and v == 0:
                        px[nb + j] = 1
                    if off < kend:
                        px[j] = max(px[j], v)
        t = torch.from_numpy(px)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        px = t.numpy()
        nchain = next((j for j in range(nchain) if px[nb + j]), nchain)
        istar = next((j for j in range(nchain) if px[j] > gkey[j]), nchain)
        committed = istar + 1 if istar < nchain else nchain
        inode = NODE_MASK - (int(px[istar]) & NODE_MASK) if istar < nchain else -1
        for j in range(committed):
            node = inode if j == istar else (NODE_MASK - (gkey[j] & NODE_MASK) if gkey[j] else -1)
            chosen[cursor + j] = node
            s, cut = wins[j]
            g = (s + np.arange(cut + 1 if cut >= 0 else n_total)) % n_total
            evals += int(((g >= lo) & (g < hi)).sum())
            if j < istar and gkey[j] and lo <= node < hi:
                shard.bind(node - lo, pods.pods[cursor + j])
                if node == inode:
                    shard.bind(node - lo, pods.pods[cursor + istar])
        if committed:
            s, cut = wins[committed - 1]
            start = (s + (cut if cut >= 0 else n_total)) % n_total
        cursor += committed
        seq0 += committed
    return chosen, evals, start


def _shard_sizes(dist, n: int, world: int):
    import torch
    t = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(t, torch.tensor([n], dtype=torch.int64))
    return [int(x[0]) for x in t]
