"""Go-harness fixtures (golden vectors item 4; tests/golden/go/).

WHAT THESE PIN: every recorded cycle in tests/golden/go/*.json.gz is an output
of oracle/objref.py, the builder's own object-level restatement
(tools/make_go_fixtures.py), not of the reference's Go plugins.  They are
objref REGRESSION PINS: they hold the C oracle, the encoders and the engine to
objref's answers.  No case counts as parity with upstream until
oracle/go/main.go has written its <case>.go.json.gz (test_go_harness_output),
which needs Go and the k8s.io/kubernetes v1.26.2 module, absent here.

Each fixture is a scheduling run as Kubernetes v1 documents plus the cycles the
object-level restatement records for it.  Here, on the CPU:

1. the documents parse back (model.node_from_dict / pod_from_dict) and the
   object-level restatement reproduces the recorded cycles (the fixture is in
   step with oracle/objref.py);
2. the C oracle, through the host encoder, reproduces every recorded filter
   outcome, score, total, placement and nextStartNodeIndex;
3. when oracle/go/main.go has been run on a box with Go and the
   k8s.io/kubernetes v1.26.2 module cache (it writes <case>.go.json.gz next to
   the fixture), its cycles must equal the recorded ones.  That is the pin
   against the reference's plugins; without the file the case is skipped and
   parity stays "unpinned vs Go".

Round 5 added cases for what rounds 3-4 built (tests/gofixture.py reads them):
plugin args (MostAllocated with an extended resource and ignoredResources,
RequestedToCapacityRatio, addedAffinity), PodTopologySpread System / List
default constraints on workload-owned pods, nominated pods, DefaultPreemption's
dry run and bound-PV volume filters.  Cycles with a PodNominator or a PostFilter
replay on objref here; the C oracle's nominated / preemption calls are held to
objref by tests/test_nominated.py and tests/test_preemption.py.
"""
import glob
import gzip
import json
import os

import pytest

from ksim import abi, profile
from ksim.encode import encode_cluster, encode_pods
from ksim.model import node_from_dict, pod_from_dict
from ksim.wrapped import filter_message
from oracle.oracle import Oracle

import gofixture

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURES = sorted(p for p in glob.glob(os.path.join(HERE, "golden", "go", "*.json.gz"))
                  if not p.endswith(".go.json.gz"))
SCORE_NAMES = ["NodeResourcesBalancedAllocation", "ImageLocality", "InterPodAffinity", "NodeResourcesFit",
               "NodeAffinity", "PodTopologySpread", "TaintToleration"]


def _load(path):
    with gzip.open(path, "rb") as f:
        return json.loads(f.read())


def _objects(doc):
    nodes = [node_from_dict(d) for d in doc["nodes"]]
    bound = [pod_from_dict(d) for d in doc["boundPods"]]
    pods = [pod_from_dict(d) for d in doc["pods"]]
    return nodes, bound, pods


def _cycle(pod_name, res, next_start):
    return {"pod": pod_name, "chosen": res["chosen"], "nextStartNodeIndex": next_start,
            "nFeasible": res["n_feasible"],
            "filter": {n: ("passed" if pl is None else [pl, msg]) for n, (pl, msg) in res["filter"].items()},
            "score": res["raw"], "normalized": res["norm"], "total": res["total"]}


def test_fixtures_present():
    assert len(FIXTURES) >= 13


@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p).split(".")[0] for p in FIXTURES])
def test_fixture_matches_objref(path):
    doc = _load(path)
    nodes, bound, pods = _objects(doc)
    ref = gofixture.objref(doc, nodes, bound)
    assert [ni.node.name for ni in ref.nodes] == [d["metadata"]["name"] for d in doc["nodes"]], "nodeTree order"
    nominated = gofixture.nominated_pods(doc)
    start = {p.name: _seconds(d) for p, d in zip(bound, doc["boundPods"])} if doc.get("preemption") else {}
    order = {p.name: k for k, p in enumerate(bound)}
    for i, (p, exp) in enumerate(zip(pods, doc["expected"])):
        kw = gofixture.cycle_kwargs(doc, i, nominated)
        res = ref.cycle(p, **kw)
        got = json.loads(json.dumps(_cycle(p.name, res, ref.next_start)))
        if "postFilter" in exp:
            node, victims = ref.preempt(p, p.priority, start, order, nominated=kw.get("nominated"))
            got["postFilter"] = {"nominatedNode": node, "victims": victims}
        elif doc.get("preemption") and res["chosen"] is not None:
            start[p.name] = 20000 + i                 # tools/make_go_fixtures.py ASSUMED_START
            order[p.name] = len(order)
        assert got == exp, f"{os.path.basename(path)}: pod {p.name}"


def _seconds(d):
    t = d["status"]["startTime"]                       # 2022-01-01THH:MM:SSZ
    h, m, sec = (int(x) for x in t[11:19].split(":"))
    return h * 3600 + m * 60 + sec


@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p).split(".")[0] for p in FIXTURES])
def test_fixture_matches_c_oracle(path):
    doc = _load(path)
    if not gofixture.plain(doc):
        pytest.skip("PodNominator / PostFilter cycles: objref replays them (test_fixture_matches_objref)")
    cluster, enc, sp, prof = gofixture.encode(doc, encode_cluster, encode_pods)
    ora = Oracle(cluster, prof)
    forder = sp.filter_order()
    snames = [p.name for p in sp.score_plugins()]
    names = cluster.node_names
    for i, exp in enumerate(doc["expected"]):
        o = ora.cycle(enc, i)
        where = f"{os.path.basename(path)}: pod {exp['pod']}"
        for pos, name in enumerate(names):
            fp = int(o["fail_plugin"][pos])
            if fp == abi.NOT_EVALUATED:
                assert name not in exp["filter"], where
            elif fp == abi.PASSED:
                assert exp["filter"][name] == "passed", (where, name)
            else:
                assert exp["filter"][name] == [forder[fp], filter_message(cluster, forder[fp],
                                                                          int(o["fail_detail"][pos]))], (where, name)
        assert o["n_feasible"] == exp["nFeasible"], where
        assert o["next_start"] == exp["nextStartNodeIndex"], where
        if exp["nFeasible"] > 1:
            for k, pl in enumerate(snames):
                for name, raw in exp["score"][pl].items():
                    pos = names.index(name)
                    assert o["raw"][k][pos] == raw, (where, pl, name)
                    assert o["norm"][k][pos] == exp["normalized"][pl][name], (where, pl, name)
            for name, tot in exp["total"].items():
                assert o["total"][names.index(name)] == tot, (where, name)
        got = names[o["chosen"]] if o["chosen"] >= 0 else None
        assert got == exp["chosen"], where


@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p).split(".")[0] for p in FIXTURES])
def test_go_harness_output(path):
    go = path[:-len(".json.gz")] + ".go.json.gz"
    if not os.path.exists(go):
        pytest.skip("no Go harness output (oracle/go needs Go + the k8s.io/kubernetes v1.26.2 module cache)")
    exp = _load(path)["expected"]
    got = _load(go)["cycles"]
    assert len(got) == len(exp)
    for g, e in zip(got, exp):
        assert g == e, f"pod {e['pod']}"
