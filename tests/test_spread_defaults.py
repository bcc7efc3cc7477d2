"""PodTopologySpread default constraints: the reference
pins PodTopologySpreadArgs defaultingType System
(/root/reference/simulator/scheduler/plugin/plugins_test.go:992-997) and runs
the Deployment / ReplicaSet controllers
(/root/reference/simulator/controller/controller.go:79-80), so upstream's
buildDefaultConstraints applies the system soft constraints (hostname maxSkew
3, zone maxSkew 5, ScheduleAnyway) to every pod a Service / ReplicaSet /
ReplicationController / StatefulSet selects, and PreScore runs with
requireAllTopologies = false for them; defaultingType List applies the args'
defaultConstraints (hard ones in Filter too).

CPU: the C oracle on the encoder's compile (ksim.topology.SpreadDefaults)
against oracle/objref.py's own DefaultSelector / buildDefaultConstraints,
cycle by cycle, on clusters where some nodes lack the zone or hostname label
(where requireAllTopologies matters).  Parity against Go stays unpinned."""
import numpy as np
import pytest

from ksim import abi, profile
from ksim.encode import encode_cluster, encode_pods
from ksim.model import (Container, Controller, LabelSelector, Node, Pod, Requirement, Service,
                        TopologySpreadConstraint)
from ksim.topology import SpreadDefaults
from ksim.wrapped import filter_message
from oracle.objref import ObjScheduler
from oracle.oracle import Oracle

SCORE_NAMES = ["NodeResourcesBalancedAllocation", "ImageLocality", "InterPodAffinity", "NodeResourcesFit",
               "NodeAffinity", "PodTopologySpread", "TaintToleration"]
ZONE, HOST = "topology.kubernetes.io/zone", "kubernetes.io/hostname"


def mixed_nodes(n=30, seed=3):
    """Nodes with both labels, without a zone (every 4th), without a hostname
    (every 7th), with neither (the simulator's UI node template has no labels)."""
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        labels = {"pool": "ab"[i % 2]}
        if i % 4 != 3:
            labels[ZONE] = f"z{i % 3}"
        if i % 7 != 5:
            labels[HOST] = f"n{i}"
        out.append(Node(f"n{i}", labels, [], {"cpu": str(int(rng.choice([8, 16, 32]))), "memory": "64Gi",
                                              "pods": "110"}))
    return out


WORKLOADS = (
    [Service("web", "default", {"app": "web"}), Service("web-fe", "default", {"app": "web", "tier": "fe"}),
     Service("nil", "default", None), Service("all", "other", {}), Service("db", "default", {"app": "db"})],
    [Controller("ReplicaSet", "web-7f9", "default",
                LabelSelector({"app": "web"}, [Requirement("pod-template-hash", "In", ["7f9"])])),
     Controller("ReplicaSet", "api-1", "default", LabelSelector({}, [Requirement("app", "Exists")])),
     Controller("ReplicationController", "cache", "default", {"app": "cache"}),
     Controller("StatefulSet", "db", "default", LabelSelector({"app": "db"})),
     Controller("ReplicaSet", "nilsel", "default", None)])


def workload_pods(n=90, seed=5, bound_nodes=None):
    rng = np.random.default_rng(seed)
    kinds = [
        ({"app": "web", "tier": "fe", "pod-template-hash": "7f9"}, ("apps/v1", "ReplicaSet", "web-7f9")),
        ({"app": "web", "pod-template-hash": "7f9"}, ("apps/v1", "ReplicaSet", "web-7f9")),
        ({"app": "api"}, ("apps/v1", "ReplicaSet", "api-1")),
        ({"app": "cache"}, ("v1", "ReplicationController", "cache")),
        ({"app": "db"}, ("apps/v1", "StatefulSet", "db")),
        ({"app": "lone"}, None),                                   # selected by nothing: no defaults
        ({"app": "orphan"}, ("apps/v1", "ReplicaSet", "missing")),  # owner not found: no defaults
        ({"app": "x"}, ("apps/v1", "ReplicaSet", "nilsel")),        # nil RS selector: no requirements
        ({"app": "web"}, ("extensions/v1beta1", "ReplicaSet", "web-7f9")),   # other group version
    ]
    out = []
    for i in range(n):
        labels, owner = kinds[int(rng.integers(0, len(kinds)))]
        p = Pod(f"p{i}", labels=dict(labels), owner=owner,
                containers=[Container({"cpu": f"{int(rng.integers(1, 20)) * 100}m", "memory": "512Mi"})])
        if i % 13 == 6:                                            # own constraints: no defaults, requireAll
            p.topology_spread = [TopologySpreadConstraint(1, ZONE, "ScheduleAnyway", LabelSelector(dict(labels)))]
        if bound_nodes is not None:
            p.node_name = bound_nodes[int(rng.integers(0, len(bound_nodes)))]
        out.append(p)
    return out


def run_both(nodes, bound, pods, sp: profile.SchedulerProfile):
    services, controllers = WORKLOADS
    spread = SpreadDefaults(sp.spread, services, controllers)
    cluster, _ = encode_cluster(nodes, bound)
    enc = encode_pods(cluster, pods, spread=spread)
    prof = profile.compile_profile(sp, cluster.scalar_names)
    ora = Oracle(cluster, prof)
    ref = ObjScheduler(nodes, bound, pct=sp.percentage_of_nodes_to_score, seed=sp.tiebreak_seed,
                       spread=sp.spread, services=services, controllers=controllers)
    forder = sp.filter_order()
    names = cluster.node_names
    chosen = []
    for i, pod in enumerate(pods):
        o = ora.cycle(enc, i)
        r = ref.cycle(pod)
        where = f"pod {i} ({pod.name})"
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
    return enc, chosen


def test_default_selector():
    services, controllers = WORKLOADS
    sd = SpreadDefaults(profile.PodTopologySpreadArgs(), services, controllers)
    web = Pod("a", labels={"app": "web", "tier": "fe", "pod-template-hash": "7f9"},
              owner=("apps/v1", "ReplicaSet", "web-7f9"))
    sel = sd.default_selector(web)
    assert sel.match_labels == {"app": "web", "tier": "fe"}
    assert [(r.key, r.operator, r.values) for r in sel.match_expressions] == \
        [("app", "In", ["web"]), ("pod-template-hash", "In", ["7f9"])]
    cons, sysdef = sd.constraints(web)
    assert sysdef and [(c.topology_key, c.max_skew, c.when_unsatisfiable) for c in cons] == \
        [(HOST, 3, "ScheduleAnyway"), (ZONE, 5, "ScheduleAnyway")]
    assert sd.default_selector(Pod("b", labels={"app": "lone"})) is None
    assert sd.default_selector(Pod("c", labels={"app": "x"}, owner=("apps/v1", "ReplicaSet", "nilsel"))) is None
    assert sd.default_selector(Pod("d", labels={"app": "cache"},
                                   owner=("v1", "ReplicationController", "cache"))).match_labels == {"app": "cache"}
    own = Pod("e", labels={"app": "web"}, topology_spread=[TopologySpreadConstraint(1, ZONE)])
    assert sd.constraints(own) == ([own.topology_spread[0]], False)
    assert SpreadDefaults(profile.PodTopologySpreadArgs("List", []), services, controllers).constraints(web) == \
        ([], False)


@pytest.mark.parametrize("pct", [0, 100])
def test_system_defaults_vs_objref(pct):
    nodes = mixed_nodes()
    bound = workload_pods(60, seed=11, bound_nodes=[n.name for n in nodes])
    pods = workload_pods(120, seed=5)
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=pct)
    enc, chosen = run_both(nodes, bound, pods, sp)
    flags = enc.pods["topo_flags"]
    assert (flags & abi.POD_PTS_SYSTEM_DEFAULT).any() and not (flags & abi.POD_PTS_SYSTEM_DEFAULT).all()
    assert sum(c is not None for c in chosen) > 100


def test_system_defaults_on_label_less_nodes():
    """The UI template's nodes carry no labels: every default constraint key is
    missing, so no node is ignored and none gets credit (every PTS score 0,
    normalized 100 -- what a bare pod gets)."""
    nodes = [Node(f"n{i}", {}, [], {"cpu": "4", "memory": "32Gi", "pods": "110"}) for i in range(12)]
    pods = workload_pods(40, seed=2)
    enc, chosen = run_both(nodes, [], pods, profile.SchedulerProfile(percentage_of_nodes_to_score=100))
    assert sum(c is not None for c in chosen) > 30


@pytest.mark.parametrize("pct", [0, 100])
def test_list_defaults_vs_objref(pct):
    """defaultingType List: hard default constraints filter (missing required
    label / skew), soft ones score with requireAllTopologies = true."""
    args = profile.PodTopologySpreadArgs("List", [
        TopologySpreadConstraint(2, ZONE, "DoNotSchedule"),
        TopologySpreadConstraint(1, HOST, "ScheduleAnyway", node_taints_policy="Honor"),
        TopologySpreadConstraint(4, "pool", "ScheduleAnyway", node_affinity_policy="Ignore")])
    profile.validate_spread_args(args)
    nodes = mixed_nodes(24, seed=9)
    bound = workload_pods(30, seed=12, bound_nodes=[n.name for n in nodes])
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=pct, spread=args)
    enc, chosen = run_both(nodes, bound, workload_pods(80, seed=7), sp)
    assert sum(c is not None for c in chosen) > 40
