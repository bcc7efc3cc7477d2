"""The node-sharded protocol on world_size-2/3 ``gloo`` process groups (CPU).

oracle/shard_model.py restates per rank what the sharded HIP path does
between its two exchanges; placements must equal the C oracle's on the whole
cluster.  Also covers the partition every rank computes and the unique-id
broadcast helper's wiring (bench.py's N > 1 plumbing)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from ksim.shard import partition


def test_partition_tiles_cluster():
    from ksim.shard import adapt_chunk
    for n, w in [(10, 3), (5000, 8), (100000, 8), (7, 7), (1031, 3), (65, 4)]:
        parts = partition(n, w)
        assert parts[0][0] == 0 and sum(c for _, c in parts) == n
        assert all(parts[i][0] + parts[i][1] == parts[i + 1][0] for i in range(w - 1))
        assert all(c > 0 for _, c in parts)
        chunk = adapt_chunk(n, w)
        if (w - 1) * chunk < n:      # the 64-aligned layout (sharded ADAPT batch path)
            assert all(b == r * chunk for r, (b, _) in enumerate(parts))
        else:                        # too few nodes for it: balanced to one node
            assert max(c for _, c in parts) - min(c for _, c in parts) <= 1
    assert partition(100000, 8)[1] == (12544, 12544) and partition(100000, 8)[7] == (87808, 12192)
    with pytest.raises(ValueError):
        partition(3, 4)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_nodes, n_pods, seed, T, B, weights, replicated=False):
    import sys
    root = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
    sys.path[:0] = [root, os.path.join(root, "kube-scheduler-simulator_amd")]
    import torch.distributed as dist
    from ksim import gen, profile
    from ksim.shard import partition
    from oracle import shard_model
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        cluster, pods = gen.config2(n_nodes=n_nodes, n_pods=n_pods, seed=seed)
        sp = profile.SchedulerProfile(percentage_of_nodes_to_score=100)
        if weights:
            sp = sp.with_weights(weights)
        w = {p.name: (p.weight or 1) for p in sp.score_plugins()}
        const = 100 * w["TaintToleration"] + 100 * w["PodTopologySpread"]
        base, cnt = partition(n_nodes, world)[rank]
        if replicated:                                   # whole cluster, this rank's evaluation range
            shard = shard_model.Shard(cluster, 0, n_nodes)
            rng = (base, base + cnt)
        else:
            shard = shard_model.Shard(cluster, base, cnt)
            rng = None
        chosen = shard_model.schedule(pods, shard, rank, world, dist, n_nodes, sp.tiebreak_seed, const,
                                      w["NodeResourcesFit"], w["NodeResourcesBalancedAllocation"], B=B, T=T,
                                      eval_range=rng)
        if replicated:                                   # every replica holds the oracle's node state
            from oracle.oracle import Oracle
            ora = Oracle(cluster, profile.compile_profile(sp))
            ora.schedule(pods)
            np.testing.assert_array_equal(shard.req_cpu, ora.node_state()["req_cpu"])
        if rank == 0:
            from oracle.oracle import Oracle
            ochosen, _ = Oracle(cluster, profile.compile_profile(sp)).schedule(pods)
            np.testing.assert_array_equal(chosen, ochosen)
        # every rank must hold the same placements
        import torch
        t = torch.from_numpy(chosen.astype(np.int64))
        ref = t.clone()
        dist.broadcast(ref, src=0)
        assert torch.equal(t, ref)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_nodes,n_pods,T,B,weights", [
    (2, 60, 500, 3, 16, None),
    (3, 40, 400, 2, 24, {"NodeResourcesBalancedAllocation": 10}),
    (2, 12, 700, 4, 32, None),          # pods stop fitting: unschedulable pods
])
def test_sharded_protocol_gloo(world, n_nodes, n_pods, T, B, weights):
    mp.spawn(_worker, args=(world, _free_port(), n_nodes, n_pods, 7, T, B, weights), nprocs=world, join=True)


@pytest.mark.parametrize("world,n_nodes,n_pods,T,B", [(2, 60, 500, 3, 16), (3, 40, 400, 2, 24)])
def test_replicated_protocol_gloo(world, n_nodes, n_pods, T, B):
    """Replicated sharding (ksim_set_eval_range): one all-gather per batch, no
    pair-key all-reduce, every replica ends with the oracle's node state."""
    mp.spawn(_worker, args=(world, _free_port(), n_nodes, n_pods, 7, T, B, None, True), nprocs=world, join=True)


def test_replicated_protocol_gloo_config4_world8():
    """The eight-replica exchange bench.py --gpus 8 --config 4 runs (one
    all-gather of the ranges' top-T records per batch), on config 4's
    generator at a CPU-sized scale."""
    from ksim import gen
    mp.spawn(_worker, args=(8, _free_port(), 240, 400, gen.SEEDS[4], 4, 32, None, True), nprocs=8, join=True)


def _worker_perpod(rank, world, port, n_nodes, n_pods, seed, pct):
    import sys
    root = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
    sys.path[:0] = [root, os.path.join(root, "kube-scheduler-simulator_amd")]
    import torch
    import torch.distributed as dist
    from ksim import gen, profile
    from ksim.shard import partition
    from oracle import shard_model
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        cluster, pods = gen.config2(n_nodes=n_nodes, n_pods=n_pods, seed=seed)
        sp = profile.SchedulerProfile(percentage_of_nodes_to_score=pct)
        w = {p.name: (p.weight or 1) for p in sp.score_plugins()}
        const = 100 * w["TaintToleration"] + 100 * w["PodTopologySpread"]
        base, cnt = partition(n_nodes, world)[rank]
        shard = shard_model.Shard(cluster, base, cnt)
        chosen, evals, start = shard_model.schedule_perpod(pods, shard, rank, world, dist, n_nodes, sp.tiebreak_seed,
                                                           const, w["NodeResourcesFit"],
                                                           w["NodeResourcesBalancedAllocation"], pct)
        t = torch.tensor([evals], dtype=torch.int64)
        dist.all_reduce(t)
        if rank == 0:
            from oracle.oracle import Oracle
            ora = Oracle(cluster, profile.compile_profile(sp))
            ochosen, ost = ora.schedule(pods)
            np.testing.assert_array_equal(chosen, ochosen)
            assert int(t[0]) == ost.evals and start == ora.next_start
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_nodes,n_pods,pct", [
    (2, 250, 400, 0),      # ADAPT: K = 100 of 250, cuts inside and across shards
    (3, 301, 300, 0),
    (3, 12, 500, 100),     # P100, pods stop fitting
])
def test_sharded_perpod_gloo(world, n_nodes, n_pods, pct):
    """The sharded per-pod cycle's window / argmax exchanges across processes."""
    mp.spawn(_worker_perpod, args=(world, _free_port(), n_nodes, n_pods, 9, pct), nprocs=world, join=True)


def _worker_adapt(rank, world, port, n_nodes, n_pods, seed, T, B):
    import sys
    root = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
    sys.path[:0] = [root, os.path.join(root, "kube-scheduler-simulator_amd")]
    import torch
    import torch.distributed as dist
    from ksim import gen, profile
    from ksim.shard import partition
    from oracle import shard_model
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        cluster, pods = gen.config2(n_nodes=n_nodes, n_pods=n_pods, seed=seed)
        sp = profile.SchedulerProfile(percentage_of_nodes_to_score=0)
        w = {p.name: (p.weight or 1) for p in sp.score_plugins()}
        const = 100 * w["TaintToleration"] + 100 * w["PodTopologySpread"]
        base, cnt = partition(n_nodes, world)[rank]
        shard = shard_model.Shard(cluster, base, cnt)
        chosen, evals, start = shard_model.schedule_adapt(pods, shard, rank, world, dist, n_nodes, sp.tiebreak_seed,
                                                          const, w["NodeResourcesFit"],
                                                          w["NodeResourcesBalancedAllocation"], B=B, T=T)
        t = torch.tensor([evals], dtype=torch.int64)
        dist.all_reduce(t)
        if rank == 0:
            from oracle.oracle import Oracle
            ora = Oracle(cluster, profile.compile_profile(sp))
            ochosen, ost = ora.schedule(pods)
            np.testing.assert_array_equal(chosen, ochosen)
            assert int(t[0]) == ost.evals and start == ora.next_start
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_nodes,n_pods,T,B", [
    (2, 250, 500, 3, 16),     # ADAPT: K = 100 of 250, windows across the shard boundary
    (3, 301, 400, 4, 24),
    (2, 130, 1500, 3, 32),    # pods stop fitting: fewer than K feasible, unschedulable pods
])
def test_sharded_adapt_batch_gloo(world, n_nodes, n_pods, T, B):
    """The node-sharded ADAPT batch protocol (bitmap all-gather, global windows,
    shard records, pair keys + broken flags under one max all-reduce) across
    processes, against the C oracle on the whole cluster."""
    mp.spawn(_worker_adapt, args=(world, _free_port(), n_nodes, n_pods, 11, T, B), nprocs=world, join=True)
