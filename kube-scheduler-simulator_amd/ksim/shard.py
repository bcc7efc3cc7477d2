"""Node sharding of one simulated cluster across GPUs.

Nodes are split into contiguous ranges of nodeTree order (global positions are
kept: tie-break keys and placements use them).  ``partition`` is the split
every rank computes identically; ``ShardedEngine`` wires one rank's engine
handle: shard snapshot, RCCL communicator (unique id from rank 0 over
torch.distributed), and the per-batch exchanges inside ksim_schedule_loaded.
"""
from __future__ import annotations

from typing import List, Tuple


def partition(n_total: int, world: int) -> List[Tuple[int, int]]:
    """Contiguous (base, count) per rank; the first n_total % world ranks get one more."""
    if world < 1 or n_total < world:
        raise ValueError("need at least one node per shard")
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
