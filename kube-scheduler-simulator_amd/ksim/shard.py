"""Node sharding of one simulated cluster across GPUs.

Nodes are split into contiguous ranges of nodeTree order (global positions are
kept: tie-break keys and placements use them).  ``partition`` is the split
every rank computes identically; ``ShardedEngine`` wires one rank's engine
handle: shard snapshot, RCCL communicator (unique id from rank 0 over
torch.distributed), and the per-batch exchanges inside ksim_schedule_loaded.
"""
from __future__ import annotations

from typing import List, Tuple


def adapt_chunk(n_total: int, world: int) -> int:
    """Shard size of the 64-aligned layout: ceil(ceil(N / R) / 64) * 64 nodes
    (the engine's adapt_shard_chunk; the last shard holds the rest)."""
    q = -(-n_total // world)
    return -(-q // 64) * 64


def partition(n_total: int, world: int) -> List[Tuple[int, int]]:
    """Contiguous (base, count) per rank.  The 64-aligned layout (adapt_chunk)
    whenever every shard stays non-empty: the node-sharded ADAPT batch path
    needs it (its shards exchange whole 64-node bitmap words); otherwise the
    first n_total % world ranks get one node more."""
    if world < 1 or n_total < world:
        raise ValueError("need at least one node per shard")
    chunk = adapt_chunk(n_total, world)
    if (world - 1) * chunk < n_total:
        return [(r * chunk, min(chunk, n_total - r * chunk)) for r in range(world)]
    q, r = divmod(n_total, world)
    out, base = [], 0
    for i in range(world):
        cnt = q + (1 if i < r else 0)
        out.append((base, cnt))
        base += cnt
    return out


def broadcast_unique_id(dist, rank: int) -> bytes:
    """Rank 0's ncclUniqueId to every rank (any torch.distributed backend)."""
    from .engine import comm_unique_id
    obj = [comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    return obj[0]


def sharded_engine(cluster, prof, rank: int, world: int, device: int, uid: bytes):
    """This rank's engine: shard snapshot of ``cluster`` + RCCL communicator."""
    from .engine import Engine
    base, cnt = partition(cluster.n_nodes, world)[rank]
    eng = Engine(device)
    eng.set_shard(base, cluster.n_nodes)
    eng.set_profile(prof)
    eng.set_cluster(cluster.shard(base, cnt))
    eng.comm_init(rank, world, uid)
    return eng


def replicated_engine(cluster, prof, rank: int, world: int, device: int, uid: bytes):
    """This rank's engine in replicated sharding (ksim_set_eval_range): the
    whole snapshot (a few MB even at 100k nodes, next to 288 GB of HBM), the
    batch top-T over this rank's range of ``partition``, one all-gather per
    batch over RCCL."""
    from .engine import Engine
    lo, cnt = partition(cluster.n_nodes, world)[rank]
    eng = Engine(device)
    eng.set_profile(prof)
    eng.set_cluster(cluster)
    eng.set_eval_range(lo, lo + cnt)
    eng.comm_init(rank, world, uid)
    return eng
