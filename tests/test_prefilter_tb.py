"""NodeAffinity's PreFilterResult and selectHost over
full int64 totals (the TB pair order), on the CPU: the C oracle (on the
encoder's node lists) against the object-level restatement oracle/objref.py,
cycle by cycle, and the PreFilter records of ksim.wrapped.record_cycle
against wrappedplugin.go:459-486 / store.go:517-530."""
import numpy as np
import pytest

from ksim import abi, gen, profile
from ksim.encode import encode_cluster, encode_pods, prefilter_node_names
from ksim.model import Container, Node, NodeSelectorTerm, Pod, Requirement
from ksim.resultstore import Store
from ksim.wrapped import ERR_NODE_AFFINITY_CONFLICT, filter_message, record_cycle
from oracle.objref import ObjScheduler
from oracle.oracle import Oracle

SCORE_NAMES = ["NodeResourcesBalancedAllocation", "ImageLocality", "InterPodAffinity", "NodeResourcesFit",
               "NodeAffinity", "PodTopologySpread", "TaintToleration"]


def _check_cycles(nodes, pods, sp, weights=None, extender=None, bound=()):
    """Oracle vs objref, cycle by cycle: filter outcomes, scores, totals,
    placement, status and nextStartNodeIndex.  Returns the oracle results."""
    cluster, _ = encode_cluster(nodes, bound)
    enc = encode_pods(cluster, pods)
    ora = Oracle(cluster, profile.compile_profile(sp))
    ref = ObjScheduler(nodes, bound, pct=sp.percentage_of_nodes_to_score, seed=sp.tiebreak_seed, weights=weights)
    forder, names = sp.filter_order(), cluster.node_names
    out = []
    for i, pod in enumerate(pods):
        if extender is not None:
            fail, score = extender
            by = {n: (int(f), int(s)) for n, f, s in zip(names, fail, score)}
            o = ora.cycle(enc, i, fail, score)
            r = ref.cycle(pod, extender=lambda kept: ({n for n in kept if by[n][0]}, {n: by[n][1] for n in kept}))
        else:
            o, r = ora.cycle(enc, i), ref.cycle(pod)
        where = f"pod {i} ({pod.name})"
        for pos, name in enumerate(names):
            fp = int(o["fail_plugin"][pos])
            if fp == abi.NOT_EVALUATED:
                assert name not in r["filter"], f"{where}: {name} evaluated only by objref"
                continue
            pl, msg = r["filter"][name]
            if fp == abi.PASSED:
                assert pl is None, f"{where}: {name} oracle passed, objref {pl}"
            elif fp == abi.FAIL_EXTENDER:
                assert pl == "extender", where
            else:
                assert pl == forder[fp], f"{where}: {name} oracle {forder[fp]} objref {pl}"
                assert msg == filter_message(cluster, forder[fp], int(o["fail_detail"][pos])), (where, name)
        assert o["n_feasible"] == r["n_feasible"], where
        assert (o["status"] == abi.STATUS_ERROR) == (r["error"] is not None), where
        if o["n_feasible"] > 1 and o["status"] == abi.STATUS_SCHEDULED:
            for pos in np.nonzero(o["scored"])[0]:
                assert o["total"][pos] == r["total"][names[pos]], f"{where}: total on {names[pos]}"
        got = names[o["chosen"]] if o["chosen"] >= 0 else None
        assert got == r["chosen"], f"{where}: oracle {got} objref {r['chosen']}"
        assert o["next_start"] == ref.next_start, f"{where}: nextStartNodeIndex"
        out.append(o)
    return cluster, enc, out


@pytest.mark.parametrize("pct", [0, 100])
def test_prefilter_node_names_vs_objref(pct):
    nodes, pods = gen.prefilter_objects(n_nodes=300, n_pods=360)
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=pct)
    cluster, enc, outs = _check_cycles(nodes, pods, sp)
    flags = enc.pods["flags"]
    restricted = (flags & abi.POD_NODE_NAMES) != 0
    assert restricted.sum() > 60
    statuses = {int(o["status"]) for o, rs in zip(outs, restricted) if rs}
    assert {abi.STATUS_SCHEDULED, abi.STATUS_UNSCHEDULABLE, abi.STATUS_ERROR} <= statuses
    # ADAPT: a restricted scan longer than its window cuts (K < R)
    if pct == 0:
        assert any(rs and o["status"] == abi.STATUS_SCHEDULED and o["k_to_find"] < int(enc.pods["nn_count"][i])
                   and o["n_processed"] < int(enc.pods["nn_count"][i])
                   for i, (o, rs) in enumerate(zip(outs, restricted)))


def test_prefilter_node_names_encoding():
    """nodeaffinity.PreFilter's set: union over terms of the intersection of each
    term's metadata.name In fields; a term without one (or no required
    terms) means every node; NotIn is not a restriction."""
    f = lambda op, *v: Requirement("metadata.name", op, list(v))   # noqa: E731
    p = Pod("p", required_terms=[NodeSelectorTerm(match_fields=[f("In", "a", "b"), f("In", "b", "c")]),
                                 NodeSelectorTerm(match_fields=[f("In", "d")])])
    assert prefilter_node_names(p) == ["b", "d"]
    p.required_terms.append(NodeSelectorTerm([Requirement("x", "Exists")]))
    assert prefilter_node_names(p) is None
    assert prefilter_node_names(Pod("q")) is None
    assert prefilter_node_names(Pod("q", required_terms=[NodeSelectorTerm(match_fields=[f("NotIn", "a")])])) is None
    assert prefilter_node_names(Pod("q", required_terms=[NodeSelectorTerm(match_fields=[f("In", "a"),
                                                                                          f("In", "b")])])) == []


def test_prefilter_records():
    """wrappedPlugin.PreFilter records NodeAffinity's status and result
    (sorted NodeNames); conflicting terms end RunPreFilterPlugins and every
    node gets that status (PostFilter lists them all); no Filter records."""
    nodes = [Node(f"n{i}", {"kubernetes.io/hostname": f"n{i}"}, [], {"cpu": "4", "memory": "8Gi", "pods": "110"})
             for i in range(4)]
    f = lambda *v: Requirement("metadata.name", "In", list(v))   # noqa: E731
    pods = [Pod("ok", containers=[Container({"cpu": "1"})],
                required_terms=[NodeSelectorTerm(match_fields=[f("n2")]), NodeSelectorTerm(match_fields=[f("n1")])]),
            Pod("conflict", containers=[Container({"cpu": "1"})],
                required_terms=[NodeSelectorTerm(match_fields=[f("n2"), f("n3")])])]
    cluster, _ = encode_cluster(nodes)
    enc = encode_pods(cluster, pods)
    sp = profile.SchedulerProfile()
    ora = Oracle(cluster, profile.compile_profile(sp))
    st = Store({})
    r0 = ora.cycle(enc, 0)
    record_cycle(st, cluster, sp, "default", "ok", r0, enc.prefilter_names[0])
    d0 = st.results["default/ok"]
    assert d0.pre_filter_status["NodeAffinity"] == "success"
    assert d0.pre_filter_result["NodeAffinity"] == ["n1", "n2"]
    assert set(d0.filter) == {"n1", "n2"}
    r1 = ora.cycle(enc, 1)
    assert r1["status"] == abi.STATUS_UNSCHEDULABLE and r1["n_evaluated"] == 0
    record_cycle(st, cluster, sp, "default", "conflict", r1, enc.prefilter_names[1])
    d1 = st.results["default/conflict"]
    assert d1.pre_filter_status["NodeAffinity"] == ERR_NODE_AFFINITY_CONFLICT
    assert "NodeAffinity" not in d1.pre_filter_result and not d1.filter


def test_large_weights_exact_totals():
    """Score weights whose 100 x sum exceeds 2^20 (a one-word key's total
    field): selectHost still orders by the full int64 total."""
    nodes, pods = gen.config1_objects(n_nodes=120, n_pods=150)
    w = {"NodeResourcesBalancedAllocation": 900001, "ImageLocality": 1, "InterPodAffinity": 7,
         "NodeResourcesFit": 1234567, "NodeAffinity": 40000, "PodTopologySpread": 2, "TaintToleration": 3}
    for pct in (0, 100):
        sp = profile.SchedulerProfile(percentage_of_nodes_to_score=pct).with_weights(w)
        _, _, outs = _check_cycles(nodes, pods, sp, weights=w)
        assert max(int(o["total"].max()) for o in outs) >= 1 << 20


def test_extender_scores_beyond_key_field():
    """Extender totals far outside [0, 2^20), negative ones included."""
    nodes, pods = gen.config1_objects(n_nodes=90, n_pods=120)
    cluster, _ = encode_cluster(nodes)
    from test_extender import extender_model
    fail, score = extender_model(cluster.node_names)
    score = (score - 150) * 10000 * 37          # weight x 10^4 scale, both signs
    _check_cycles(nodes, pods, profile.SchedulerProfile(percentage_of_nodes_to_score=100),
                  extender=(fail, score))


@pytest.mark.parametrize("pct", [0, 100])
def test_edge_quantities_vs_objref(pct):
    """Allocatable 0, overcommitted nodes, quantities past 2^52 and 2^56
    (Go's wrapping int64 product in leastRequestedScore), weight 0 -> 1."""
    nodes, bound, pods = gen.edge_objects()
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=pct)
    _check_cycles(nodes, pods, sp, bound=bound)
    w = {"NodeResourcesBalancedAllocation": 0, "ImageLocality": 0, "InterPodAffinity": 0,
         "NodeResourcesFit": 3, "NodeAffinity": 0, "PodTopologySpread": 0, "TaintToleration": 0}
    sp0 = profile.SchedulerProfile(percentage_of_nodes_to_score=pct).with_weights(w)
    cluster, enc, outs = _check_cycles(nodes, pods, sp0, weights=w, bound=bound)
    assert any(o["status"] == abi.STATUS_UNSCHEDULABLE for o in outs)
