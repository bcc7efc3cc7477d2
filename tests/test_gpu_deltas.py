"""Node informer deltas on the GPU: a cluster whose nodes
carry 60 label keys and hugepages resources is scheduled half way, nodes are
added / updated / removed (ksim.ingest.NodeCache -> ksim_upsert_nodes, and
ksim_remove_node on the device snapshot alone), and the rest of the queue runs;
placements, node state and count classes match the oracle given the same
deltas (whose replay tests/test_node_deltas.py pins against a fresh start)."""
import numpy as np
import pytest

from ksim import gen, profile
from ksim.encode import encode_cluster, encode_pods
from ksim.engine import Engine
from ksim.ingest import NodeCache
from ksim.model import Container, Node, NodeSelectorTerm, Pod, Requirement
from oracle.oracle import Oracle
from test_node_deltas import _apply

pytestmark = pytest.mark.gpu


def _same(eng, ora):
    es, os_ = eng.node_state(), ora.node_state()
    for k in es:
        np.testing.assert_array_equal(es[k], os_[k], err_msg=k)
    np.testing.assert_array_equal(eng.class_count(), ora.class_count())
    np.testing.assert_array_equal(eng.nb_alloc(), ora.nb_alloc())
    assert eng.next_start == ora.next_start


@pytest.mark.parametrize("pct", [0, 100])
def test_node_deltas_mid_run(pct):
    nodes, bound, pending, deltas = gen.delta_objects(n_nodes=600, n_pods=1800)
    cache = NodeCache(nodes, bound)
    c0 = cache.cluster
    pods = encode_pods(c0, pending)
    assert c0.n_label_cols >= 50 and "hugepages-2Mi" in c0.scalar_names
    prof = profile.compile_profile(profile.SchedulerProfile(percentage_of_nodes_to_score=pct), c0.scalar_names)
    eng = Engine(0)
    eng.set_profile(prof)
    eng.set_cluster(c0)
    ora = Oracle(c0, prof)
    half = 900
    eng.load_pods(pods)
    a, _ = eng.schedule_loaded(0, half)
    b, _ = ora.schedule(pods, 0, half)
    np.testing.assert_array_equal(a, b)
    _same(eng, ora)
    _apply(cache, deltas)
    c1, old_pos, pods1 = cache.commit(pending)
    assert c1.n_scalar == c0.n_scalar + 1 and (old_pos == -1).sum() == len(deltas[0])
    eng.upsert_nodes(c1, old_pos)
    ora.upsert_nodes(c1, old_pos)
    _same(eng, ora)
    eng.load_pods(pods1)
    a, st = eng.schedule_loaded(half, pods1.n_pods - half)
    b, _ = ora.schedule(pods1, half)
    np.testing.assert_array_equal(a, b)
    _same(eng, ora)
    assert (a >= 0).sum() > 300 and st.perpod_cycles > 0
    # reset: back to the delta's snapshot (the table), then the same run again
    eng.reset_cluster()
    eng.set_next_start(ora.next_start)
    ora2 = Oracle(c1, prof)
    ora2.set_next_start(ora.next_start)
    eng.set_pod_seq(half)
    ora2.set_pod_seq(half)
    a2, _ = eng.schedule_loaded(half, pods1.n_pods - half)
    b2, _ = ora2.schedule(pods1, half)
    np.testing.assert_array_equal(a2, b2)


def _drop_node(c, pos):
    """The host snapshot without node ``pos`` (node columns sliced)."""
    import copy
    keep = np.array([i for i in range(c.n_nodes) if i != pos], np.int64)
    d = copy.copy(c)
    d.n_nodes = c.n_nodes - 1
    for f in ("alloc_cpu", "alloc_mem", "alloc_eph", "alloc_pods", "req_cpu", "req_mem", "req_eph",
              "nz_cpu", "nz_mem", "num_pods", "flags", "nb_limit", "nb_alloc"):
        setattr(d, f, np.ascontiguousarray(getattr(c, f)[keep]))
    for f in ("alloc_scalar", "req_scalar", "taints", "labels", "class_count"):
        setattr(d, f, np.ascontiguousarray(getattr(c, f)[:, keep]))
    d.node_names = [c.node_names[i] for i in keep]
    return d, keep.astype(np.int32)


def test_remove_node_on_device():
    nodes, bound, pending, _ = gen.delta_objects(n_nodes=400, n_pods=900)
    c, _ = encode_cluster(nodes, bound)
    pods = encode_pods(c, pending)
    prof = profile.compile_profile(profile.SchedulerProfile(percentage_of_nodes_to_score=0), c.scalar_names)
    eng = Engine(0)
    eng.set_profile(prof)
    eng.set_cluster(c)
    ora = Oracle(c, prof)
    eng.load_pods(pods)
    a, _ = eng.schedule_loaded(0, 400)
    b, _ = ora.schedule(pods, 0, 400)
    np.testing.assert_array_equal(a, b)
    victim = int(np.bincount(a[a >= 0]).argmax())              # a node the run filled
    eng.remove_node(victim)
    d, old_pos = _drop_node(c, victim)
    ora.upsert_nodes(d, old_pos)
    assert eng.n_nodes == d.n_nodes
    eng.load_pods(pods)
    a, _ = eng.schedule_loaded(400, 500)
    b, _ = ora.schedule(pods, 400, 500)
    np.testing.assert_array_equal(a, b)
    _same(eng, ora)


def test_engine_set_before_pods_resyncs():
    """set_cluster before the pods were encoded: the label columns the pods
    add reach the device (Engine._sync) and the cycles match the oracle."""
    nodes = [Node(f"n{i}", {"zone": f"z{i % 3}", "tier": "abc"[i % 3], "rack": f"r{i % 5}"}, [],
                  {"cpu": "8", "memory": "16Gi", "pods": "20"}) for i in range(30)]
    c, _ = encode_cluster(nodes)
    prof = profile.compile_profile(profile.SchedulerProfile(percentage_of_nodes_to_score=100))
    eng = Engine(0)
    eng.set_profile(prof)
    eng.set_cluster(c)
    assert c.n_label_cols == 0
    plist = [Pod(f"p{j}", containers=[Container({"cpu": "500m"})],
                 required_terms=[NodeSelectorTerm([Requirement("tier", "In", ["b", "c"])])],
                 node_selector={"rack": f"r{j % 5}"}) for j in range(40)]
    pods = encode_pods(c, plist)
    ora = Oracle(c, prof)
    for i in range(pods.n_pods):
        e, o = eng.eval_pod(pods, i), ora.cycle(pods, i)
        assert e["chosen"] == o["chosen"]
        if e["chosen"] >= 0:
            assert nodes[0].labels["tier"] != c.label_values[c.label_col("tier")][c.labels[c.label_col("tier"), e["chosen"]]]
    _same(eng, ora)
