"""Go-harness fixtures (golden vectors item 4; tests/golden/go/).

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
from oracle.objref import ObjScheduler
from oracle.oracle import Oracle

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
    assert len(FIXTURES) >= 4


@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p).split(".")[0] for p in FIXTURES])
def test_fixture_matches_objref(path):
    doc = _load(path)
    nodes, bound, pods = _objects(doc)
    ref = ObjScheduler(nodes, bound, namespaces=doc["namespaces"], pct=doc["percentageOfNodesToScore"],
                       seed=doc["tiebreakSeed"], hard_pod_affinity_weight=doc["hardPodAffinityWeight"])
    assert [ni.node.name for ni in ref.nodes] == [d["metadata"]["name"] for d in doc["nodes"]], "nodeTree order"
    for p, exp in zip(pods, doc["expected"]):
        got = json.loads(json.dumps(_cycle(p.name, ref.cycle(p), ref.next_start)))
        assert got == exp, f"{os.path.basename(path)}: pod {p.name}"


@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p).split(".")[0] for p in FIXTURES])
def test_fixture_matches_c_oracle(path):
    doc = _load(path)
    nodes, bound, pods = _objects(doc)
    cluster, _ = encode_cluster(nodes, bound, namespaces=doc["namespaces"])
    enc = encode_pods(cluster, pods)
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=doc["percentageOfNodesToScore"],
                                  tiebreak_seed=doc["tiebreakSeed"],
                                  hard_pod_affinity_weight=doc["hardPodAffinityWeight"])
    ora = Oracle(cluster, profile.compile_profile(sp))
    forder = sp.filter_order()
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
            for k, pl in enumerate(SCORE_NAMES):
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
