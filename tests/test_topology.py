"""PodTopologySpread + InterPodAffinity on the CPU:
the C oracle (on the encoder's count classes) against the independent
object-level restatement oracle/objref.py (strings and maps, upstream code
structure), cycle by cycle: every filter outcome and message, every raw and
normalized score, totals and the placement.  This pins the host class
compiler (ksim/topology.py) and the C restatement together."""
import numpy as np
import pytest

from ksim import abi, gen, profile
from ksim.encode import encode_cluster, encode_pods
from ksim.model import (Container, LabelSelector, Node, Pod, PodAffinityTerm, Requirement, Taint, Toleration,
                        TopologySpreadConstraint, WeightedPodAffinityTerm, NodeSelectorTerm)
from ksim.wrapped import filter_message
from oracle.objref import ObjScheduler
from oracle.oracle import Oracle

SCORE_NAMES = ["NodeResourcesBalancedAllocation", "ImageLocality", "InterPodAffinity", "NodeResourcesFit",
               "NodeAffinity", "PodTopologySpread", "TaintToleration"]


def run_both(nodes, bound, pods, pct=0, namespaces=None, hard_w=1, check_state=True):
    cluster, _ = encode_cluster(nodes, bound, namespaces=namespaces)
    enc = encode_pods(cluster, pods)
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=pct, hard_pod_affinity_weight=hard_w)
    prof = profile.compile_profile(sp)
    ora = Oracle(cluster, prof)
    ref = ObjScheduler(nodes, bound, namespaces=namespaces, pct=pct, seed=sp.tiebreak_seed,
                       hard_pod_affinity_weight=hard_w)
    forder = sp.filter_order()
    names = cluster.node_names
    chosen = []
    for i, pod in enumerate(pods):
        o = ora.cycle(enc, i)
        r = ref.cycle(pod)
        where = f"pod {i} ({pod.name})"
        # filter outcomes
        for pos, name in enumerate(names):
            fp = int(o["fail_plugin"][pos])
            if fp == abi.NOT_EVALUATED:
                assert name not in r["filter"], f"{where}: {name} evaluated only by objref"
                continue
            pl, msg = r["filter"][name]
            if fp == abi.PASSED:
                assert pl is None, f"{where}: {name} oracle passed, objref {pl}: {msg}"
            else:
                assert pl == forder[fp], f"{where}: {name} oracle {forder[fp]} objref {pl}"
                assert msg == filter_message(cluster, forder[fp], int(o["fail_detail"][pos])), (where, name)
        assert o["n_feasible"] == r["n_feasible"], where
        if o["n_feasible"] > 1:
            for k, pl in enumerate(SCORE_NAMES):
                for pos in np.nonzero(o["scored"])[0]:
                    name = names[pos]
                    assert o["raw"][k][pos] == r["raw"][pl][name], f"{where}: raw {pl} on {name}"
                    assert o["norm"][k][pos] == r["norm"][pl][name], f"{where}: norm {pl} on {name}"
                    assert o["total"][pos] == r["total"][name], f"{where}: total on {name}"
        got = names[o["chosen"]] if o["chosen"] >= 0 else None
        assert got == r["chosen"], f"{where}: oracle {got} objref {r['chosen']}"
        chosen.append(got)
    return cluster, enc, ora, chosen


@pytest.mark.parametrize("pct", [0, 100])
def test_config3_small_vs_objref(pct):
    nodes, bound, pods = gen.config3_objects(n_nodes=30, pods_per_node=4, n_incoming=80, seed=7, zone_anti_every=5)
    _, _, _, chosen = run_both(nodes, bound, pods, pct)
    assert len(set(chosen)) > 5


def _node(i, zone="z0", taints=(), extra=None, cpu="8"):
    labels = {"kubernetes.io/hostname": f"n{i}", "topology.kubernetes.io/zone": zone}
    labels.update(extra or {})
    return Node(f"n{i}", labels, list(taints), {"cpu": cpu, "memory": "32Gi", "pods": "110"})


def _pod(name, labels=None, node="", ns="default", **kw):
    return Pod(name, namespace=ns, labels=dict(labels or {}), node_name=node,
               containers=[Container({"cpu": "100m", "memory": "128Mi"})], **kw)


def test_required_pod_affinity_first_pod_and_followers():
    """satisfyPodAffinity: with no matching pod anywhere, a pod that matches
    its own affinity terms may go anywhere (the first of a series); later pods
    must follow it; a pod that does not match its own terms is unschedulable."""
    nodes = [_node(i, f"z{i % 3}") for i in range(9)]
    term = PodAffinityTerm("topology.kubernetes.io/zone", LabelSelector({"app": "db"}))
    pods = [_pod(f"db{i}", {"app": "db"}, pod_affinity_required=[term]) for i in range(4)]
    pods.append(_pod("web", {"app": "web"}, pod_affinity_required=[
        PodAffinityTerm("topology.kubernetes.io/zone", LabelSelector({"app": "cache"}))]))
    _, _, _, chosen = run_both(nodes, [], pods)
    zones = {n.name: n.labels["topology.kubernetes.io/zone"] for n in nodes}
    assert len({zones[c] for c in chosen[:4]}) == 1
    assert chosen[4] is None


def test_required_anti_affinity_and_existing_anti():
    nodes = [_node(i, f"z{i % 2}") for i in range(6)]
    bound = [_pod("e0", {"app": "x"}, node="n0", pod_anti_affinity_required=[
        PodAffinityTerm("topology.kubernetes.io/zone", LabelSelector({"app": "y"}))])]
    pods = [_pod("y0", {"app": "y"}),                                    # blocked from zone z0 by e0
            _pod("x1", {"app": "z"}, pod_anti_affinity_required=[       # avoids hosts with app=x
                PodAffinityTerm("kubernetes.io/hostname", LabelSelector({"app": "x"}))]),
            _pod("y1", {"app": "y"}, pod_anti_affinity_required=[
                PodAffinityTerm("kubernetes.io/hostname", LabelSelector({"app": "y"}))])]
    run_both(nodes, bound, pods)


def test_spread_policies_missing_labels_and_ignored_nodes():
    """nodeAffinityPolicy Honor vs Ignore, nodeTaintsPolicy Honor, a node
    without the zone label (missing required label for hard constraints,
    IgnoredNodes for soft ones), an empty selector (counts nothing but
    self-matches) and minDomains (feature gate off in v1.26: ignored)."""
    nodes = [_node(i, f"z{i % 3}") for i in range(8)]
    nodes.append(Node("nolabel", {"kubernetes.io/hostname": "nolabel"}, [], {"cpu": "8", "memory": "32Gi",
                                                                            "pods": "110"}))
    nodes[1].taints = [Taint("dedicated", "gpu", "NoSchedule")]
    nodes[2].labels["pool"] = "b"
    bound = [_pod(f"e{i}", {"app": "s"}, node=f"n{i % 4}") for i in range(6)]
    sel = LabelSelector({"app": "s"})
    pods = []
    for i in range(12):
        kw = {}
        if i % 3 == 0:
            kw["node_selector"] = {"pool": "b"}
        pods.append(_pod(f"s{i}", {"app": "s"}, tolerations=[Toleration("dedicated", "Equal", "gpu", "NoSchedule")],
                         topology_spread=[
                             TopologySpreadConstraint(1, "topology.kubernetes.io/zone", "DoNotSchedule", sel,
                                                      min_domains=5,
                                                      node_affinity_policy="Ignore" if i % 2 else None,
                                                      node_taints_policy="Honor" if i % 4 == 1 else None),
                             TopologySpreadConstraint(1, "topology.kubernetes.io/zone", "ScheduleAnyway", sel),
                             TopologySpreadConstraint(3, "kubernetes.io/hostname", "ScheduleAnyway",
                                                      LabelSelector() if i % 5 == 0 else sel)], **kw))
    soft_only = [_pod(f"t{i}", {"app": "s"}, topology_spread=[
        TopologySpreadConstraint(1, "topology.kubernetes.io/zone", "ScheduleAnyway", sel)]) for i in range(6)]
    run_both(nodes, bound, pods + soft_only)


def test_preferred_terms_namespaces_and_hard_weight():
    """IPA scoring: incoming preferred (anti-)affinity, existing pods' required
    affinity (hardPodAffinityWeight) and preferred terms, namespaces lists and
    namespaceSelector (empty = all namespaces, labelled = resolved)."""
    nodes = [_node(i, f"z{i % 3}") for i in range(9)]
    namespaces = {"default": {}, "prod": {"env": "prod"}, "dev": {"env": "dev"}}
    bound = [
        _pod("e0", {"app": "db"}, node="n0", ns="prod", pod_affinity_required=[
            PodAffinityTerm("topology.kubernetes.io/zone", LabelSelector({"app": "web"}), namespaces=["default"])]),
        _pod("e1", {"app": "db"}, node="n4", ns="dev", pod_affinity_preferred=[WeightedPodAffinityTerm(
            30, PodAffinityTerm("kubernetes.io/hostname", LabelSelector({"app": "web"}),
                                namespace_selector=LabelSelector()))]),
        _pod("e2", {"app": "cache"}, node="n5", pod_anti_affinity_preferred=[WeightedPodAffinityTerm(
            70, PodAffinityTerm("topology.kubernetes.io/zone", LabelSelector({"app": "web"})))]),
        _pod("e3", {"app": "db"}, node="n8", ns="prod"),
    ]
    pods = [
        _pod("w0", {"app": "web"}),
        _pod("w1", {"app": "web"}, pod_affinity_preferred=[WeightedPodAffinityTerm(
            20, PodAffinityTerm("topology.kubernetes.io/zone", LabelSelector({"app": "db"}),
                                namespace_selector=LabelSelector({"env": "prod"})))]),
        _pod("w2", {"app": "web"}, pod_anti_affinity_preferred=[WeightedPodAffinityTerm(
            40, PodAffinityTerm("kubernetes.io/hostname", LabelSelector({"app": "web"})))]),
        _pod("w3", {"app": "web"}, ns="dev"),
    ]
    for hw in (1, 0, 7):
        run_both(nodes, bound, pods, namespaces=namespaces, hard_w=hw)


def test_class_counts_follow_binds():
    """After the run the oracle's count classes equal a recount from scratch
    (encoder adds applied at every bind == NodeInfo.AddPod)."""
    nodes, bound, pods = gen.config3_objects(n_nodes=12, pods_per_node=3, n_incoming=30, seed=3, zone_anti_every=4)
    cluster, enc, ora, chosen = run_both(nodes, bound, pods)
    placed = []
    for p, c in zip(pods, chosen):
        if c is not None:
            q = Pod(**{**p.__dict__, "node_name": c})
            placed.append(q)
    again, _ = encode_cluster(nodes, bound + placed)
    encode_pods(again, pods)
    got = ora.class_count()
    want = {k: again.class_count[i] for i, k in enumerate(again.topo.keys)}
    assert set(want) == set(cluster.topo.keys)
    for i, k in enumerate(cluster.topo.keys):
        np.testing.assert_array_equal(got[i], want[k], err_msg=str(k))


def test_invalid_selector_rejected():
    nodes = [_node(0)]
    bad = _pod("bad", {"app": "x"}, topology_spread=[TopologySpreadConstraint(
        1, "topology.kubernetes.io/zone", "DoNotSchedule", LabelSelector({}, [Requirement("app", "In", [])]))])
    cluster, _ = encode_cluster(nodes)
    with pytest.raises(ValueError):
        encode_pods(cluster, [bad])


# ---- NodePorts: HostPortInfo as count classes -------------------

def _port_pod(name, ports, node="", **kw):
    from ksim.model import ContainerPort
    return Pod(name, node_name=node, containers=[
        Container({"cpu": "100m", "memory": "128Mi"}, [ContainerPort(*p) for p in ports])], **kw)


def test_node_ports_conflicts_vs_objref():
    """0.0.0.0 conflicts with the (protocol, port) pair on every ip, a specific ip
    with itself and 0.0.0.0; protocols differ; hostPort 0 is no host port;
    bound pods' ports and earlier queue pods' binds both count."""
    nodes = [_node(i, f"z{i % 2}") for i in range(4)]
    bound = [_port_pod("b0", [(80, "TCP", "")], node="n0"),
             _port_pod("b1", [(80, "TCP", "10.0.0.1"), (53, "UDP", "")], node="n1"),
             _port_pod("b2", [(8080, "TCP", "10.0.0.2")], node="n2")]
    pods = [_port_pod("p0", [(80, "TCP", "")]),                # conflicts n0 (0.0.0.0) and n1 (10.0.0.1)
            _port_pod("p1", [(80, "TCP", "10.0.0.3")]),        # conflicts n0 (0.0.0.0) only
            _port_pod("p2", [(53, "TCP", "")]),                # UDP 53 on n1 does not conflict
            _port_pod("p3", [(53, "UDP", "10.0.0.9")]),        # n1 holds UDP 53 on 0.0.0.0
            _port_pod("p4", [(8080, "TCP", "10.0.0.2"), (0, "TCP", "")]),
            _port_pod("p5", [(80, "TCP", ""), (53, "UDP", "")]),
            _port_pod("p6", [(9000, "", "")])]                 # empty protocol -> TCP
    pods += [_port_pod(f"q{i}", [(7000 + i % 3, "TCP", "")]) for i in range(8)]   # fill: later pods conflict
    for pct in (0, 100):
        run_both(nodes, bound, pods, pct=pct)


def test_node_ports_config1_mixed():
    """Config-1 objects with host ports on a third of the pods (per-pod path),
    the rest batchable: the C oracle equals the object-level restatement."""
    from ksim.model import ContainerPort
    nodes, pods = gen.config1_objects(n_nodes=30, n_pods=240)
    for i, p in enumerate(pods):
        if i % 3 == 0:
            p.containers[0].ports = [ContainerPort(8000 + i % 5, "TCP", "" if i % 2 else "10.1.0.%d" % (i % 4))]
    run_both(nodes, [], pods, pct=0, check_state=False)


# ---- ImageLocality -------------------------------------------------

def test_image_locality_vs_objref():
    """Node image lists with sizes around the 23 MB / 1000 MB x containers
    thresholds, images spread over some nodes, untagged names (":latest"),
    multi-container pods, pods whose images no node has."""
    mb = 1024 * 1024
    nodes = []
    for i in range(12):
        n = _node(i, f"z{i % 3}")
        imgs = []
        if i % 2 == 0:
            imgs.append((["nginx:latest", "docker.io/library/nginx:latest"], 180 * mb))
        if i % 3 == 0:
            imgs.append((["redis:7"], 40 * mb + i))
        if i % 4 == 1:
            imgs.append((["big/model:v1"], 3000 * mb))
        if i == 5:
            imgs.append((["tiny:1"], 5 * mb))
        n.images = imgs
        nodes.append(n)

    def ipod(name, images):
        return Pod(name, containers=[Container({"cpu": "100m", "memory": "64Mi"}, image=im) for im in images])
    pods = [ipod("a", ["nginx"]), ipod("b", ["redis:7", "nginx:latest"]), ipod("c", ["big/model:v1"]),
            ipod("d", ["tiny:1"]), ipod("e", ["absent:1"]), ipod("f", ["big/model:v1", "redis:7", "nginx"]),
            ipod("g", ["docker.io/library/nginx"])]
    pods = pods * 3
    for pct in (0, 100):
        run_both(nodes, [], pods, pct=pct)
