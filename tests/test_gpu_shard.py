"""Node-sharded batch path on the GPU, bit-exact vs the oracle
on the whole cluster.  One MI355X: the in-process shard group exercises the
full exchange protocol (candidate all-gather, pair-key max all-reduce, owner
binds); the RCCL communicator is exercised with world = 1."""
import numpy as np
import pytest

from ksim import engine, gen, profile
from ksim.engine import Engine, group_schedule_loaded
from ksim.shard import partition
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu


def _prof(weights=None, seed=0x4B53494D):
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=100, tiebreak_seed=seed)
    if weights:
        sp = sp.with_weights(weights)
    return profile.compile_profile(sp)


def _group(cluster, pods, prof, world):
    engines = []
    for base, cnt in partition(cluster.n_nodes, world):
        e = Engine(0)
        e.set_shard(base, cluster.n_nodes)
        e.set_profile(prof)
        e.set_cluster(cluster.shard(base, cnt))
        e.load_pods(pods)
        engines.append(e)
    return engines


def _node_state(engines):
    parts = [e.node_state() for e in engines]
    return {k: np.concatenate([p[k] for p in parts]) for k in parts[0]}


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_group_config2_slice(world):
    cluster, pods = gen.config2(n_nodes=2000, n_pods=6000)
    prof = _prof()
    engines = _group(cluster, pods, prof, world)
    chosen, st = group_schedule_loaded(engines, 0, pods.n_pods)
    assert engines[0].diag()["graph_captures"] >= 1      # batches replayed as hipGraphs of 16
    ora = Oracle(cluster, prof)
    ochosen, ost = ora.schedule(pods, nthreads=8)
    np.testing.assert_array_equal(chosen, ochosen)
    assert st.evals == ost.evals and st.scheduled == ost.scheduled
    es, os_ = _node_state(engines), ora.node_state()
    for k in es:
        np.testing.assert_array_equal(es[k], os_[k])


@pytest.mark.parametrize("n_nodes,world", [(9, 2), (65, 4), (300, 3), (1031, 8)])
def test_group_ragged_until_full(n_nodes, world):
    """Ragged shards, pods that stop fitting (unschedulable), batches cut short."""
    cluster, _ = gen.config2(n_nodes=n_nodes, n_pods=1)
    pods = gen.bare_pods(n_nodes * 120 + 37, seed=99)    # > 110 pods per node: some never fit
    prof = _prof()
    engines = _group(cluster, pods, prof, world)
    chosen, st = group_schedule_loaded(engines, 0, pods.n_pods)
    ochosen, ost = Oracle(cluster, prof).schedule(pods)
    np.testing.assert_array_equal(chosen, ochosen)
    assert st.unschedulable == ost.unschedulable and st.unschedulable > 0


def test_group_truncation_and_cuts():
    cluster, _ = gen.config2(n_nodes=300, n_pods=1)
    pods = gen.bare_pods(4000, seed=17, cpu_steps=20, mem_steps=2)
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=100)
    w = {p.name: (10 if p.name == "NodeResourcesBalancedAllocation" else 1) for p in sp.score_plugins()}
    prof = profile.compile_profile(sp.with_weights(w))
    engines = _group(cluster, pods, prof, 4)
    chosen, st = group_schedule_loaded(engines, 0, pods.n_pods)
    ochosen, _ = Oracle(cluster, prof).schedule(pods)
    np.testing.assert_array_equal(chosen, ochosen)
    cluster2, _ = gen.config2(n_nodes=40, n_pods=1)
    cluster2.alloc_cpu[:] = 64000
    cluster2.alloc_mem[:] = 256 << 30
    pods2 = gen.bare_pods(3000, seed=5, cpu_steps=1, mem_steps=1)
    engines = _group(cluster2, pods2, _prof(), 3)
    chosen, st = group_schedule_loaded(engines, 0, pods2.n_pods)
    np.testing.assert_array_equal(chosen, Oracle(cluster2, _prof()).schedule(pods2)[0])
    # identical pods on 40 nodes: batches end early (an exhausted candidate
    # list, or a pod whose best node was bound earlier in its batch)
    assert st.truncations > 0 or st.batches > 2 * (pods2.n_pods // 256)


def test_rccl_world1():
    """ksim_comm_init + the RCCL exchange calls with a single rank."""
    cluster, pods = gen.config2(n_nodes=1500, n_pods=6000)
    prof = _prof()
    uid = engine.comm_unique_id()
    e = Engine(0)
    e.set_shard(0, cluster.n_nodes)
    e.set_profile(prof)
    e.set_cluster(cluster)
    e.comm_init(0, 1, uid)
    e.load_pods(pods)
    chosen, st = e.schedule_loaded(0, pods.n_pods)
    assert e.diag()["graph_captures"] >= 1               # RCCL collectives captured in the batch graphs
    ochosen, ost = Oracle(cluster, prof).schedule(pods, nthreads=8)
    np.testing.assert_array_equal(chosen, ochosen)
    assert st.evals == ost.evals


# ---- sharded per-pod cycle (ADAPT window, per-node normalized scores, topology) ----

def _check_group(cluster, pods, prof, world):
    engines = _group(cluster, pods, prof, world)
    chosen, st = group_schedule_loaded(engines, 0, pods.n_pods)
    ora = Oracle(cluster, prof)
    ochosen, ost = ora.schedule(pods, nthreads=8)
    np.testing.assert_array_equal(chosen, ochosen)
    assert st.evals == ost.evals and st.scheduled == ost.scheduled and st.unschedulable == ost.unschedulable
    for e in engines:
        assert e.next_start == ora.next_start
    es, os_ = _node_state(engines), ora.node_state()
    for k in es:
        np.testing.assert_array_equal(es[k], os_[k])
    return engines, ora


@pytest.mark.parametrize("pct,world", [(0, 2), (100, 3), (0, 8)])
def test_group_perpod_config1(pct, world):
    """Taints, node affinity, per-node-varying normalized scores; ADAPT windows
    that cut inside and across shards; P100 runs mixing batch and per-pod pods."""
    cluster, pods = gen.config1()
    _check_group(cluster, pods, _prof_pct(pct), world)


@pytest.mark.parametrize("world", [2, 5])
def test_group_adapt_config2(world):
    cluster, pods = gen.config2(n_nodes=1200, n_pods=1500)
    _check_group(cluster, pods, _prof_pct(0), world)


@pytest.mark.parametrize("pct,world", [(0, 2), (100, 4), (0, 8)])
def test_group_config3(pct, world):
    """PodTopologySpread + InterPodAffinity: domain sums exchanged, global
    critical paths, IgnoredNodes and pair registrations over the global kept list."""
    cluster, pods = gen.config3(n_nodes=600, pods_per_node=10, n_incoming=700, seed=21, zone_anti_every=50)
    engines, ora = _check_group(cluster, pods, _prof_pct(pct), world)
    np.testing.assert_array_equal(np.concatenate([e.class_count() for e in engines], axis=1), ora.class_count())
    # the 700 topology pods ran as graphs of 128 sharded cycles on the leader
    assert engines[0].diag()["graph_captures"] >= 1


def test_rccl_world1_perpod():
    cluster, pods = gen.config3(n_nodes=500, pods_per_node=10, n_incoming=400, seed=22)
    prof = _prof_pct(0)
    e = Engine(0)
    e.set_shard(0, cluster.n_nodes)
    e.set_profile(prof)
    e.set_cluster(cluster)
    e.comm_init(0, 1, engine.comm_unique_id())
    e.load_pods(pods)
    g0 = e.diag()["graph_captures"]
    chosen, st = e.schedule_loaded(0, pods.n_pods)
    ochosen, ost = Oracle(cluster, prof).schedule(pods, nthreads=8)
    np.testing.assert_array_equal(chosen, ochosen)
    assert st.evals == ost.evals
    # RCCL collectives captured with the cycles' kernels (graphs of 128 cycles)
    assert e.diag()["graph_captures"] > g0


def _prof_pct(pct, seed=0x4B53494D):
    return profile.compile_profile(profile.SchedulerProfile(percentage_of_nodes_to_score=pct, tiebreak_seed=seed))


def _adapt_prof(seed=0x4B53494D):
    return profile.compile_profile(profile.SchedulerProfile(percentage_of_nodes_to_score=0, tiebreak_seed=seed))


@pytest.mark.parametrize("n_nodes,world", [(2000, 2), (3000, 4), (5000, 8), (1031, 3)])
def test_group_adapt_batch(n_nodes, world):
    """ADAPT (the simulator's default) on node shards: the sharded ADAPT batch
    path (bitmap all-gather, global windows, shard records, broken flags in
    the max all-reduce) matches the oracle on the whole cluster, including
    nextStartNodeIndex and the evaluation count."""
    cluster, pods = gen.config2(n_nodes=n_nodes, n_pods=3000)
    prof = _adapt_prof()
    assert partition(n_nodes, world)[1][0] % 64 == 0          # the aligned layout
    engines = _group(cluster, pods, prof, world)
    chosen, st = group_schedule_loaded(engines, 0, pods.n_pods)
    ora = Oracle(cluster, prof)
    ochosen, ost = ora.schedule(pods, nthreads=8)
    np.testing.assert_array_equal(chosen, ochosen)
    assert st.evals == ost.evals and st.scheduled == ost.scheduled
    assert st.batches > 0 and st.perpod_cycles == 0             # the batch path ran
    assert all(e.next_start == ora.next_start for e in engines)
    es, os_ = _node_state(engines), ora.node_state()
    for k in es:
        np.testing.assert_array_equal(es[k], os_[k])


def test_group_adapt_until_full():
    """ADAPT shards while pods stop fitting: windows that wrap, fewer than K
    feasible nodes, unschedulable pods."""
    cluster, _ = gen.config2(n_nodes=700, n_pods=1)
    pods = gen.bare_pods(700 * 112, seed=7)
    prof = _adapt_prof()
    engines = _group(cluster, pods, prof, 4)
    chosen, st = group_schedule_loaded(engines, 0, pods.n_pods)
    ora = Oracle(cluster, prof)
    ochosen, ost = ora.schedule(pods, nthreads=8)
    np.testing.assert_array_equal(chosen, ochosen)
    assert (chosen == -1).sum() > 0 and st.evals == ost.evals
    assert engines[0].diag()["graph_captures"] >= 1      # ADAPT batches replayed as hipGraphs of 16


def test_rccl_world1_adapt():
    """The RCCL exchange calls of the sharded ADAPT batch with a single rank."""
    cluster, pods = gen.config2(n_nodes=1500, n_pods=6000)
    prof = _adapt_prof()
    e = Engine(0)
    e.set_shard(0, cluster.n_nodes)
    e.set_profile(prof)
    e.set_cluster(cluster)
    e.comm_init(0, 1, engine.comm_unique_id())
    e.load_pods(pods)
    chosen, st = e.schedule_loaded(0, pods.n_pods)
    ochosen, ost = Oracle(cluster, prof).schedule(pods, nthreads=8)
    np.testing.assert_array_equal(chosen, ochosen)
    assert st.evals == ost.evals and st.batches > 0
    assert e.diag()["graph_captures"] >= 1


# ---- replicated sharding (ksim_set_eval_range): whole snapshot per handle ----------

def _replicas(cluster, pods, prof, world):
    engines = []
    for lo, cnt in partition(cluster.n_nodes, world):
        e = Engine(0)
        e.set_profile(prof)
        e.set_cluster(cluster)
        e.set_eval_range(lo, lo + cnt)
        e.load_pods(pods)
        engines.append(e)
    return engines


@pytest.mark.parametrize("n_nodes,world", [(2000, 2), (1031, 3), (5000, 8)])
def test_group_replicated(n_nodes, world):
    """Each replica evaluates its node range in the batch top-T; one exchange
    per batch (no pair-key all-reduce); every replica binds every placement
    and ends with the oracle's whole node state."""
    cluster, pods = gen.config2(n_nodes=n_nodes, n_pods=6000)
    prof = _prof()
    engines = _replicas(cluster, pods, prof, world)
    chosen, st = group_schedule_loaded(engines, 0, pods.n_pods)
    ora = Oracle(cluster, prof)
    ochosen, ost = ora.schedule(pods, nthreads=8)
    np.testing.assert_array_equal(chosen, ochosen)
    assert st.evals == ost.evals and st.scheduled == ost.scheduled
    assert engines[0].diag()["graph_captures"] >= 1
    os_ = ora.node_state()
    for e in engines:
        es = e.node_state()
        for k in es:
            np.testing.assert_array_equal(es[k], os_[k])


def test_group_replicated_config4():
    """Config 4's cluster (100,000 nodes) over eight replicas, each keying its
    12,500-node range (bench.py --gpus 8 --config 4's protocol): the oracle's
    placements and every replica's node state."""
    cluster, pods = gen.config4(n_nodes=100000, n_pods=2500)
    prof = _prof()
    engines = _replicas(cluster, pods, prof, 8)
    chosen, st = group_schedule_loaded(engines, 0, pods.n_pods)
    ora = Oracle(cluster, prof)
    ochosen, ost = ora.schedule(pods, nthreads=8)
    np.testing.assert_array_equal(chosen, ochosen)
    assert st.evals == ost.evals and st.scheduled == ost.scheduled
    os_ = ora.node_state()
    for e in engines:
        es = e.node_state()
        for k in es:
            np.testing.assert_array_equal(es[k], os_[k])


def test_group_replicated_mixed_paths():
    """Pods the batch path cannot take (taints, node affinity: per-pod cycles)
    run whole on every replica between replicated batches."""
    cluster, pods = gen.config1(n_nodes=300, n_pods=3000)
    prof = _prof()
    engines = _replicas(cluster, pods, prof, 3)
    chosen, st = group_schedule_loaded(engines, 0, pods.n_pods)
    ochosen, _ = Oracle(cluster, prof).schedule(pods, nthreads=8)
    np.testing.assert_array_equal(chosen, ochosen)


def test_rccl_world1_replicated():
    cluster, pods = gen.config2(n_nodes=1500, n_pods=6000)
    prof = _prof()
    e = Engine(0)
    e.set_profile(prof)
    e.set_cluster(cluster)
    e.set_eval_range(0, cluster.n_nodes)
    e.comm_init(0, 1, engine.comm_unique_id())
    e.load_pods(pods)
    chosen, st = e.schedule_loaded(0, pods.n_pods)
    ochosen, ost = Oracle(cluster, prof).schedule(pods, nthreads=8)
    np.testing.assert_array_equal(chosen, ochosen)
    assert st.evals == ost.evals and e.diag()["graph_captures"] >= 1


@pytest.mark.parametrize("n_nodes,world,n_apps", [(900, 2, 64), (1031, 3, 6), (2000, 8, 64)])
def test_group_replicated_config3(n_nodes, world, n_apps):
    """Replicated topology batches (config 3): each replica filters / scores
    its node range; the per-pod counters and extrema, the top-T records with
    the extremum holders, and the pair maxima are exchanged; every replica
    commits every placement and every class add, ending with the oracle's
    node state and class counts."""
    from ksim.encode import encode_cluster, encode_pods
    from ksim.model import LabelSelector
    nodes, bound, inc = gen.config3_objects(n_nodes=n_nodes, pods_per_node=4, n_incoming=1500, seed=world,
                                            zone_anti_every=50)
    rng = np.random.default_rng(world)
    for k, p in enumerate(inc):
        app = f"a{int(rng.integers(0, n_apps))}"
        p.labels["app"] = app
        if n_apps < 64 and k % 2:                   # node-local uses only: these runs cross
            p.topology_spread = [c for c in p.topology_spread if c.when_unsatisfiable == "ScheduleAnyway"]
        for c in p.topology_spread:
            c.label_selector = LabelSelector({"app": app})
        for w in p.pod_anti_affinity_preferred:
            w.term.label_selector = LabelSelector({"app": app})
    cluster, _ = encode_cluster(nodes, bound)
    pods = encode_pods(cluster, inc)
    prof = _prof()
    engines = _replicas(cluster, pods, prof, world)
    chosen, st = group_schedule_loaded(engines, 0, pods.n_pods)
    ora = Oracle(cluster, prof)
    ochosen, ost = ora.schedule(pods, nthreads=8)
    np.testing.assert_array_equal(chosen, ochosen)
    assert st.scheduled == ost.scheduled and st.perpod_cycles == 0 and st.batches < pods.n_pods
    os_ = ora.node_state()
    for e in engines:
        es = e.node_state()
        for k in es:
            np.testing.assert_array_equal(es[k], os_[k], err_msg=k)
        np.testing.assert_array_equal(e.class_count(), ora.class_count())


def test_rccl_world1_replicated_config3():
    from ksim.encode import encode_cluster, encode_pods
    nodes, bound, inc = gen.config3_objects(n_nodes=700, pods_per_node=4, n_incoming=1200, seed=13)
    cluster, _ = encode_cluster(nodes, bound)
    pods = encode_pods(cluster, inc)
    prof = _prof()
    e = Engine(0)
    e.set_profile(prof)
    e.set_cluster(cluster)
    e.set_eval_range(0, cluster.n_nodes)
    e.comm_init(0, 1, engine.comm_unique_id())
    e.load_pods(pods)
    chosen, st = e.schedule_loaded(0, pods.n_pods)
    ochosen, ost = Oracle(cluster, prof).schedule(pods, nthreads=8)
    np.testing.assert_array_equal(chosen, ochosen)
    assert st.perpod_cycles == 0 and st.batches < pods.n_pods
