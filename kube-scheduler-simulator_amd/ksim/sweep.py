"""Policy sweeps (BASELINE config 5): independent score-weight
vectors over one snapshot and queue, the vectors split over GPUs as replicas.

The reference applies each sweep point by a profile restart
(simulator/server/handler/schedulerconfig.go:40-60 -> scheduler.go:70-87) and
reads the placements back; here each engine re-runs the queue under one vector
after another (ksim_set_profile keeps the captured batch graphs, ksim_load_pods
reuses the queue buffers) and the per-vector placements are gathered to rank 0
at the end (C4: one all-gather of int32 [vectors][pods], no data-path
collective during the sweep).

Vector v runs on rank v % world; within a rank, engine j of J takes the rank's
vectors j, j + J, ...  ``gather_placements`` undoes both splits.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np


def rank_vectors(n_vectors: int, rank: int, world: int) -> List[int]:
    """Global indices of the weight vectors rank ``rank`` sweeps."""
    return list(range(rank, n_vectors, world))


def gather_placements(local: np.ndarray, rank: int, world: int, n_vectors: int, dist=None,
                      device: Optional[str] = None, n_pods: Optional[int] = None) -> Optional[np.ndarray]:
    """All ranks' [local vectors][pods] placement rows -> the [n_vectors][pods]
    matrix in global vector order on rank 0 (None elsewhere).  ``dist``: the
    torch.distributed module of an initialized process group (RCCL on GPU
    tensors, gloo on CPU); None for one process.  ``n_pods``: the queue length,
    which every rank must send alike (a rank with no vectors has no rows to read
    it from); taken from ``local`` when omitted."""
    local = np.ascontiguousarray(local, np.int32)
    if n_pods is None:
        n_pods = local.shape[1] if local.ndim == 2 and local.shape[0] else 0
    if local.size == 0:
        local = np.zeros((0, n_pods), np.int32)
    if dist is None or world == 1:
        out = np.full((n_vectors, n_pods), -3, np.int32)
        out[rank_vectors(n_vectors, 0, 1)] = local
        return out
    import torch
    rows = -(-n_vectors // world)                      # every rank sends the same shape
    buf = np.full((rows, n_pods), -3, np.int32)
    buf[:local.shape[0]] = local
    t = torch.from_numpy(buf)
    if device is not None:
        t = t.to(device)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    if rank != 0:
        return None
    out = np.full((n_vectors, n_pods), -3, np.int32)
    for r, part in enumerate(parts):
        idx = rank_vectors(n_vectors, r, world)
        out[idx] = part.cpu().numpy()[:len(idx)]
    return out


def placement_digest(placements: np.ndarray) -> str:
    """A short digest of a placement matrix (reported by bench.py)."""
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(placements, np.int32).tobytes()).hexdigest()[:16]


def order_engine_results(results: Sequence[Sequence[np.ndarray]], n_local: int) -> np.ndarray:
    """Engine j's placement rows (its vectors j, j + J, ... of the rank's list)
    -> [n_local][pods] in the rank's order."""
    J = len(results)
    rows = [None] * n_local
    for j, res in enumerate(results):
        for k, row in enumerate(res):
            rows[j + k * J] = row
    return np.stack(rows) if rows else np.zeros((0, 0), np.int32)
