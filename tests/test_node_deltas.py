"""Node informer deltas and on-demand label columns on the CPU (SURVEY §8(f) 2;
VERDICT r1 item 6): ksim.ingest.NodeCache re-encodes the snapshot after node
add / update / remove events, the oracle replays its binds on top of it
(ksim_oracle_upsert_nodes, the restatement of ksim_upsert_nodes), and the run
continues exactly as a scheduler started from scratch on the new snapshot with
the pods placed so far bound to their nodes."""
import copy

import numpy as np
import pytest

from ksim import abi, gen, profile
from ksim.encode import EncodeError, encode_cluster, encode_pods
from ksim.ingest import NodeCache
from ksim.model import Container, Node, NodeSelectorTerm, Pod, Requirement
from oracle.oracle import Oracle


def _apply(cache, deltas):
    added, updated, removed = deltas
    for n in updated:
        cache.update_node(n)
    for name in removed:
        cache.remove_node(name)
    for n in added:
        cache.add_node(n)


def _fresh(cache, bound, pending, placed, old_names, prof_sp):
    """A scheduler started from scratch on the cache's nodes, with the pods
    placed so far bound (pods placed on a node that left stay out, as upstream
    keeps them on a node outside the tree)."""
    names = {n.name for n in cache.nodes}
    b = list(bound)
    for p, c in zip(pending, placed):
        if c >= 0 and old_names[c] in names:
            q = copy.copy(p)
            q.node_name = old_names[c]
            b.append(q)
    cluster, _ = encode_cluster(cache.nodes, b, extra_scalar=cache.extra_scalar)
    return cluster


def delta_run(pct, half=360, n_pods=720):
    """(oracle chosen before / after the delta, fresh-start chosen after, states)."""
    nodes, bound, pending, deltas = gen.delta_objects(n_pods=n_pods)
    cache = NodeCache(nodes, bound)
    c0 = cache.cluster
    assert c0.n_label_cols == 0                          # columns only once a pod references a key
    pods = encode_pods(c0, pending)
    assert 0 < c0.n_label_cols < 62 + 2
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=pct)
    ora = Oracle(c0, profile.compile_profile(sp, c0.scalar_names))
    first, _ = ora.schedule(pods, 0, half)
    old_names = list(c0.node_names)
    _apply(cache, deltas)
    c1, old_pos, pods1 = cache.commit(pending)
    assert c1.n_scalar == c0.n_scalar + 1 and c1.scalar_names[:c0.n_scalar] == c0.scalar_names
    assert (old_pos == -1).sum() == len(deltas[0])
    ora.upsert_nodes(c1, old_pos)
    ns = ora.next_start
    second, _ = ora.schedule(pods1, half, n_pods - half)
    # the fresh start
    cf = _fresh(cache, bound, pending[:half], first, old_names, sp)
    assert cf.node_names == c1.node_names
    podsf = encode_pods(cf, pending[half:])
    fresh = Oracle(cf, profile.compile_profile(sp, cf.scalar_names))
    fresh.set_next_start(ns)
    fresh.set_pod_seq(half)
    fchosen, _ = fresh.schedule(podsf)
    return first, second, fchosen, ora, fresh, (c0, c1, old_pos, pods, pods1)


@pytest.mark.parametrize("pct", [0, 100])
def test_delta_replay_matches_fresh_start(pct):
    first, second, fchosen, ora, fresh, _ = delta_run(pct)
    np.testing.assert_array_equal(second, fchosen)
    a, b = ora.node_state(), fresh.node_state()
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    assert (first >= 0).sum() > 100 and (second >= 0).sum() > 100 and (second == -1).sum() > 0


def test_next_start_carries_over_mod_n():
    nodes, bound, pending, deltas = gen.delta_objects(n_pods=200)
    cache = NodeCache(nodes, bound)
    pods = encode_pods(cache.cluster, pending)
    ora = Oracle(cache.cluster, profile.compile_profile(profile.SchedulerProfile(percentage_of_nodes_to_score=0)))
    ora.set_next_start(cache.cluster.n_nodes - 1)
    ora.schedule(pods, 0, 1)
    before = ora.next_start
    cache.remove_node(cache.nodes[0].name)
    for n in deltas[2][:3]:
        if n != cache.nodes[0].name and any(x.name == n for x in cache.nodes):
            cache.remove_node(n)
    c1, old_pos, _ = cache.commit(pending)
    ora.upsert_nodes(c1, old_pos)
    assert ora.next_start == before % c1.n_nodes


def test_node_tree_order_on_zone_change():
    """nodeTree.updateNode with a new zone = removeNode + addNode: the node
    goes to the end of its new zone's list (node_tree.go)."""
    mk = lambda name, z: Node(name, {"topology.kubernetes.io/zone": z}, [], {"cpu": "4", "memory": "8Gi", "pods": "10"})
    cache = NodeCache([mk("a1", "a"), mk("b1", "b"), mk("a2", "a"), mk("b2", "b"), mk("a3", "a")])
    assert cache.cluster.node_names == ["a1", "b1", "a2", "b2", "a3"]
    cache.update_node(mk("a1", "b"))
    c1, old_pos, _ = cache.commit([])
    # zones in order of first appearance: b (b1), a (a2); b's list b1 b2 a1, a's list a2 a3
    assert c1.node_names == ["b1", "a2", "b2", "a3", "a1"]
    assert list(old_pos) == [1, 2, 3, 4, 0]


def test_label_columns_on_demand():
    nodes, bound, pending, _ = gen.delta_objects(n_pods=50)
    c, _ = encode_cluster(nodes, bound)
    assert c.n_label_cols == 0
    assert c.label_col("no-such-key") == -1 and c.n_label_cols == 0
    k = c.label_col("example.com/k07")
    assert k == 0 and c.label_keys == ["example.com/k07"]
    vals = c.label_values[0]
    assert vals[0] == "" and sorted(vals[1:]) == ["v0", "v1", "v2"]
    for pos, lb in enumerate(c.node_labels):
        v = lb.get("example.com/k07")
        assert c.labels[0, pos] == (vals.index(v) if v is not None else 0)
    c2 = c.copy_state()
    c2.label_col("example.com/k08")
    assert c.n_label_cols == 1 and c2.n_label_cols == 2    # copies never share a grown column list


def test_label_column_cap():
    keys = [f"k{j:03d}" for j in range(abi.MAX_LABEL_COLS + 1)]
    nodes = [Node("n0", {k: "x" for k in keys}, [], {"cpu": "4", "memory": "8Gi", "pods": "10"})]
    c, _ = encode_cluster(nodes)
    pod = Pod("p", containers=[Container({"cpu": "1"})], node_selector={k: "x" for k in keys})
    with pytest.raises(EncodeError):
        encode_pods(c, [pod])


def test_oracle_made_before_pods_resyncs():
    """An Oracle built before the pods were encoded sees the label columns the
    pods added (Oracle._sync re-sends the snapshot in place)."""
    nodes = [Node(f"n{i}", {"zone": f"z{i % 2}", "tier": "a" if i < 2 else "b"}, [],
                  {"cpu": "4", "memory": "8Gi", "pods": "10"}) for i in range(4)]
    c, _ = encode_cluster(nodes)
    ora = Oracle(c, profile.compile_profile(profile.SchedulerProfile()))
    pods = encode_pods(c, [Pod("p", containers=[Container({"cpu": "1"})],
                               required_terms=[NodeSelectorTerm([Requirement("tier", "In", ["b"])])])])
    r = ora.cycle(pods, 0)
    assert c.node_names[r["chosen"]] in ("n2", "n3")
