"""The static-class table (DevPods::stab, csrc/ksim_engine.cpp ensure_stab,
csrc/ksim_batch.hip k_static_table / stab_fast_keys) against the one-by-one
oracle: the table follows a profile whose static filter list changes, a node
removed from the device snapshot, and a queue with more static classes than
the table holds (the class-less pods' runs take the generic keys).  Config 1's
object distribution: taints (NoSchedule and PreferNoSchedule), tolerations,
required and preferred node affinity with per-pod weights."""
import copy

import numpy as np
import pytest

from ksim import gen, profile
from ksim.encode import encode_cluster, encode_pods
from ksim.engine import Engine
from oracle.oracle import Oracle
from test_gpu_deltas import _drop_node

pytestmark = pytest.mark.gpu


def _state_eq(eng, ora):
    es, os_ = eng.node_state(), ora.node_state()
    for k in es:
        np.testing.assert_array_equal(es[k], os_[k], err_msg=k)


def _without_filter(sp, name):
    sp = copy.deepcopy(sp)
    sp.plugins["filter"].enabled = [p for p in sp.plugins["filter"].enabled
                                    if profile.original_name(p.name) != name]
    return sp


def test_profile_change_rebuilds_table():
    """The table is built under the default profile, then the TaintToleration
    filter leaves the profile: the same queue from the same snapshot must see
    tainted nodes as feasible (the verdicts come from the rebuilt table)."""
    nodes, objs = gen.config1_objects(n_nodes=900, n_pods=3000)
    cluster, _ = encode_cluster(nodes)
    pods = encode_pods(cluster, objs)
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=100)
    eng = Engine(0)
    eng.set_profile(profile.compile_profile(sp))
    eng.set_cluster(cluster)
    eng.load_pods(pods)
    a, st = eng.schedule_loaded(0, pods.n_pods)
    b, _ = Oracle(cluster, profile.compile_profile(sp)).schedule(pods, nthreads=8)
    np.testing.assert_array_equal(a, b)
    assert st.perpod_cycles == 0 and st.batches > 0
    prof2 = profile.compile_profile(_without_filter(sp, "TaintToleration"))
    eng.set_profile(prof2)                       # (drops the queue: the plans follow the profile)
    eng.load_pods(pods)
    eng.reset_cluster()
    eng.set_pod_seq(0)
    a2, _ = eng.schedule_loaded(0, pods.n_pods)
    ora2 = Oracle(cluster, prof2)
    b2, _ = ora2.schedule(pods, nthreads=8)
    np.testing.assert_array_equal(a2, b2)
    _state_eq(eng, ora2)
    assert (a2 != a).any()                       # the filter change reached the keys


def test_remove_node_rebuilds_table():
    """Half the queue, then a node the run filled leaves the device snapshot:
    the table's rows shrink with the node columns."""
    nodes, objs = gen.config1_objects(n_nodes=700, n_pods=2400)
    cluster, _ = encode_cluster(nodes)
    pods = encode_pods(cluster, objs)
    prof = profile.compile_profile(profile.SchedulerProfile(percentage_of_nodes_to_score=100))
    eng = Engine(0)
    eng.set_profile(prof)
    eng.set_cluster(cluster)
    ora = Oracle(cluster, prof)
    eng.load_pods(pods)
    a, _ = eng.schedule_loaded(0, 1200)
    b, _ = ora.schedule(pods, 0, 1200)
    np.testing.assert_array_equal(a, b)
    victim = int(np.bincount(a[a >= 0]).argmax())
    eng.remove_node(victim)
    d, old_pos = _drop_node(cluster, victim)
    ora.upsert_nodes(d, old_pos)
    eng.load_pods(pods)
    a, _ = eng.schedule_loaded(1200, 1200)
    b, _ = ora.schedule(pods, 1200, 1200)
    np.testing.assert_array_equal(a, b)
    _state_eq(eng, ora)


def test_more_classes_than_the_table_holds():
    """4,500 pods naming distinct nodes (spec.nodeName: one static class each)
    interleaved with config 1's pods: past 4,096 classes the remaining pods
    have none, and the runs holding them take the generic keys."""
    nodes, objs = gen.config1_objects(n_nodes=5000, n_pods=2000)
    named = []
    for k in range(4500):
        p = copy.deepcopy(objs[k % len(objs)])
        p.name = f"named-{k:05d}"
        p.node_name = nodes[(7 * k) % len(nodes)].name
        named.append(p)
    queue = []
    for k in range(max(len(objs), len(named))):
        if k < len(named):
            queue.append(named[k])
        if k < len(objs):
            queue.append(objs[k])
    cluster, _ = encode_cluster(nodes)
    pods = encode_pods(cluster, queue)
    prof = profile.compile_profile(profile.SchedulerProfile(percentage_of_nodes_to_score=100))
    eng = Engine(0)
    eng.set_profile(prof)
    eng.set_cluster(cluster)
    chosen, st = eng.schedule_batch(pods)
    ora = Oracle(cluster, prof)
    ochosen, ost = ora.schedule(pods, nthreads=8)
    np.testing.assert_array_equal(chosen, ochosen)
    assert st.evals == ost.evals
    _state_eq(eng, ora)
