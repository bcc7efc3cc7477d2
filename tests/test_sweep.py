"""Policy-sweep placement gather (ksim/sweep.py) on CPU:
the engine / rank splits of the weight vectors and the all-gather to rank 0
on world_size 2 and 3 ``gloo`` process groups."""
import multiprocessing as mp
import socket

import numpy as np
import pytest

from ksim import sweep


def _rows(v, n_pods):
    """Stand-in placements of global vector v (distinct per vector and pod)."""
    return (np.arange(n_pods, dtype=np.int32) * 7 + v * 1000) % 5000 - (v % 3 == 0)


def test_order_engine_results_and_single_process():
    n_vectors, n_pods, J = 11, 13, 4
    local = sweep.rank_vectors(n_vectors, 0, 1)
    results = [[_rows(local[k], n_pods) for k in range(j, len(local), J)] for j in range(J)]
    rows = sweep.order_engine_results(results, len(local))
    out = sweep.gather_placements(rows, 0, 1, n_vectors)
    np.testing.assert_array_equal(out, np.stack([_rows(v, n_pods) for v in range(n_vectors)]))


def _worker(rank, world, port, n_vectors, n_pods, q):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        mine = sweep.rank_vectors(n_vectors, rank, world)
        J = 3                                            # engines per rank
        results = [[_rows(mine[k], n_pods) for k in range(j, len(mine), J)] for j in range(J)]
        rows = sweep.order_engine_results(results, len(mine))
        out = sweep.gather_placements(rows, rank, world, n_vectors, dist, n_pods=n_pods)
        q.put((rank, None if out is None else out.tolist()))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,n_vectors", [(2, 9), (3, 10), (3, 2)])
def test_gather_placements_gloo(world, n_vectors):
    n_pods = 17
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_vectors, n_pods, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert all(got[r] is None for r in range(1, world))
    np.testing.assert_array_equal(np.array(got[0], np.int32),
                                  np.stack([_rows(v, n_pods) for v in range(n_vectors)]))
