"""The drop-in's incremental snapshot on the CPU (the oracle as the device):
ksim.fwsnapshot.SnapshotSync applies informer events through the encoder's
delta calls (ABI 11) and the framework's cycles agree, cycle by cycle, with a
run that re-encodes and re-sends its whole record every cycle."""
import copy

import numpy as np
import pytest

from fwdeltas import FullSync, drive, make_runs, objects, same_node_state
from fwmirror import OracleBackend
from ksim import abi, profile
from ksim.fwsnapshot import SnapshotSync
from ksim.model import Node, Pod, Container
from ksim.nativeenc import NativeEncoder
from oracle.oracle import Oracle


def _oracle(nodes, bound, prof):
    from ksim.nativeenc import encode
    cluster, _ = encode(nodes, bound, [])
    return OracleBackend(Oracle(cluster, prof))


@pytest.mark.parametrize("seed", [11, 12])
def test_incremental_snapshot_matches_full_reencode(seed):
    nodes, bound, incoming = objects(n_nodes=72, pods_per_node=3, n_incoming=140)
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=0)
    prof = profile.compile_profile(sp)
    runs = make_runs([("incremental", _oracle(nodes, bound, prof), False),
                      ("full", _oracle(nodes, bound, prof), True)], nodes, bound, sp, seed)
    events = drive(runs, nodes, bound, incoming, seed=seed)
    assert events > 40
    same_node_state(runs)
    st = runs[0].sync.stats
    assert st["full_encodes"] == 1, st              # the first snapshot only
    assert st["node_deltas"] > 5 and st["pod_adds"] > 10 and st["pod_deletes"] > 10, st
    assert st["reserves"] > 100, st
    assert st["node_rows_in_place"] > 0 and st["node_rows_in_place"] < st["node_deltas"], st


def test_encoder_membership_counts_new_classes():
    """A count class registered after binds counts every pod bound so far:
    the engine's binds (ksim_encoder_bind) and the snapshot's pods, minus
    the unbound ones."""
    from ksim.model import LabelSelector, PodAffinityTerm
    nodes = [Node(name=f"n{i}", labels={"kubernetes.io/hostname": f"n{i}", "topology.kubernetes.io/zone": f"z{i % 2}"},
                  allocatable={"cpu": "8", "memory": "16Gi", "pods": "110"}) for i in range(4)]
    c = Container({"cpu": "100m", "memory": "64Mi"})
    bound = [Pod(name=f"b{i}", labels={"app": "x", "k": str(i)}, containers=[c], node_name=f"n{i % 4}")
             for i in range(6)]
    enc = NativeEncoder()
    cl, _ = enc.encode_cluster(nodes, bound)
    pos = {n: i for i, n in enumerate(cl.node_names)}
    q = [Pod(name=f"q{i}", labels={"app": "x", "k": str(i)}, containers=[c]) for i in range(3)]
    for i, p in enumerate(q):
        enc.encode_pods(cl, [p])
        enc.bind(0, pos[f"n{i}"])
    assert enc.unbind("default", "b0") == pos["n0"]
    assert enc.info().n_members == 6 - 1 + 3
    # a selector on app=x registered now counts the members per node
    probe = Pod(name="probe", containers=[c],
                pod_anti_affinity_required=[PodAffinityTerm("kubernetes.io/hostname", LabelSelector({"app": "x"}))])
    enc.encode_pods(cl, [probe])
    counts = cl.class_count
    want = np.zeros(4, np.int32)
    for p in bound[1:]:
        want[pos[p.node_name]] += 1
    for i in range(3):
        want[pos[f"n{i}"]] += 1
    assert any(np.array_equal(row, want) for row in counts), (counts, want)
    with pytest.raises(Exception):
        enc.unbind("default", "b0")               # not bound any more
    enc.encode_pods(cl, [q[0]])
    with pytest.raises(Exception):
        enc.bind(0, pos["n1"])                    # already bound


def test_encoder_node_delta_positions_and_rows():
    """ksim_encoder_update_nodes: kept nodes keep their snapshot rows under
    their new positions, added nodes start empty, a zone move re-adds the
    node at the end of the add order, a removed node's pods leave."""
    nodes, bound, _ = objects(n_nodes=12, pods_per_node=2, n_incoming=0)
    enc = NativeEncoder()
    cl, _ = enc.encode_cluster(nodes, bound)
    before = {n: (int(cl.req_cpu[i]), int(cl.num_pods[i])) for i, n in enumerate(cl.node_names)}
    members = enc.info().n_members
    moved = copy.copy(nodes[4])
    moved.labels = dict(nodes[4].labels, **{"topology.kubernetes.io/zone": "z9"})
    new = Node(name="fresh", labels={"kubernetes.io/hostname": "fresh", "topology.kubernetes.io/zone": "z1"},
               allocatable={"cpu": "4", "memory": "8Gi", "pods": "10"})
    gone = nodes[7].name
    cl2, old_pos, rows = enc.update_nodes([moved, new], [gone])
    assert rows is None                             # nodes added, removed and moved: the whole table
    assert cl2.n_nodes == 12
    assert gone not in cl2.node_names and "fresh" in cl2.node_names
    for i, n in enumerate(cl2.node_names):
        if n == "fresh":
            assert old_pos[i] == -1 and cl2.req_cpu[i] == 0 and cl2.num_pods[i] == 0
        else:
            assert cl.node_names[old_pos[i]] == n
            assert (int(cl2.req_cpu[i]), int(cl2.num_pods[i])) == before[n]
    assert enc.info().n_members == members - 2      # the removed node's two pods
    # the moved node sits in its own zone: nodeTree order puts the new zone last among zones
    assert cl2.node_labels[cl2.node_names.index(nodes[4].name)]["topology.kubernetes.io/zone"] == "z9"


def test_encoder_updates_rows_in_place():
    """An update that moves no node and needs no new vocabulary changes only
    the updated rows' static columns (ksim_encoder_changed_rows); a new label
    value or taint takes the whole-table path."""
    from ksim.model import Taint
    nodes, bound, _ = objects(n_nodes=12, pods_per_node=2, n_incoming=0)
    nodes[3].taints = [Taint("dedicated", "x", "NoSchedule")]
    enc = NativeEncoder()
    cl, _ = enc.encode_cluster(nodes, bound)
    from ksim.model import LabelSelector, PodAffinityTerm
    probe = Pod(name="probe", containers=[Container({"cpu": "1"})],
                pod_anti_affinity_required=[PodAffinityTerm("kubernetes.io/hostname", LabelSelector({"app": "a1"}))])
    enc.encode_pods(cl, [probe])                    # a hostname label column
    cl = enc.cluster
    before = {k: getattr(cl, k).copy() for k in ("alloc_cpu", "flags", "taints", "labels", "req_cpu", "num_pods")}
    a = copy.copy(nodes[5])
    a.allocatable = dict(a.allocatable, cpu="3")
    a.unschedulable = True
    a.taints = [Taint("dedicated", "x", "NoSchedule")]
    cl2, old_pos, rows = enc.update_nodes([a], [])
    assert rows is not None and list(old_pos) == list(range(cl2.n_nodes))
    p = cl2.node_names.index(a.name)
    assert list(rows) == [p]
    assert cl2.alloc_cpu[p] == 3000 and cl2.flags[p] & abi.NODE_UNSCHEDULABLE and cl2.taints[0][p] != 0
    for k, v in before.items():
        got = getattr(cl2, k)
        mask = np.ones(cl2.n_nodes, bool)
        if k in ("alloc_cpu", "flags", "taints"):
            mask[p] = False
        np.testing.assert_array_equal(np.asarray(got)[..., mask], np.asarray(v)[..., mask], err_msg=k)
    b = copy.copy(nodes[6])
    b.labels = dict(b.labels, **{"kubernetes.io/hostname": "renamed-host"})   # a value the column lacks
    _, _, rows2 = enc.update_nodes([b], [])
    assert rows2 is None
    c2 = copy.copy(nodes[7])
    c2.taints = [Taint("fresh", "y", "NoExecute")]                             # a taint the vocabulary lacks
    _, _, rows3 = enc.update_nodes([c2], [])
    assert rows3 is None
