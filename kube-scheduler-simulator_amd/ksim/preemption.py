"""Host side of DefaultPreemption: the bound-pod table the
engine's PostFilter dry run reads (ksim_bound_pods), built from the pods bound
in a snapshot.  Requests follow NodeInfo's Requested (the same
computePodResourceRequest the encoder uses)."""
from __future__ import annotations

from typing import Dict, Sequence

import numpy as np

from . import abi
from .encode import pod_requests
from .model import Pod


def bound_table(cluster, bound: Sequence[Pod], start_time: Dict[str, int]) -> abi.BoundPods:
    """ksim_bound_pods for ``bound`` (pods whose node is in ``cluster``), in list order."""
    pos = {n: i for i, n in enumerate(cluster.node_names)}
    rows = [p for p in bound if p.node_name in pos]
    node = np.array([pos[p.node_name] for p in rows], np.int32)
    prio = np.array([p.priority for p in rows], np.int32)
    start = np.array([start_time[p.name] for p in rows], np.int64)
    req = np.zeros((len(rows), abi.PREEMPT_REQ), np.int64)
    for i, p in enumerate(rows):
        r = pod_requests(p)
        req[i, 0] = r.get("cpu", 0)
        req[i, 1] = r.get("memory", 0)
        req[i, 2] = r.get("ephemeral-storage", 0)
        for k, name in enumerate(cluster.scalar_names):
            req[i, 3 + k] = r.get(name, 0)
    return abi.BoundPods(node, prio, start, req)
