"""Write the Go-harness fixtures (golden vectors item 4).

Each fixture under tests/golden/go/<case>.json.gz holds one scheduling run as
Kubernetes v1 documents (nodes in nodeTree order, bound pods, pending pods in
queue order, the profile knobs) and, under "expected", what the object-level
restatement (oracle/objref.py) records for every cycle: per-node filter result
("passed" or [plugin, message]), raw and normalized scores per score plugin,
totals, the chosen node and nextStartNodeIndex.

oracle/go/main.go runs the same documents through the upstream in-tree plugins
(k8s.io/kubernetes v1.26.2) and writes <case>.go.json.gz in the same schema;
tests/test_go_fixtures.py compares the two when that file is present.  Until
then the fixtures are self-consistent only ("parity unpinned vs Go").

    python tools/make_go_fixtures.py        # rewrites tests/golden/go/*.json.gz
"""
import gzip
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kube-scheduler-simulator_amd"), os.path.join(ROOT, "tests")]

from ksim import gen, k8sjson  # noqa: E402
from oracle.objref import ObjScheduler  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "go")
SEED = 0x4B53494D


def _cycle_json(pod_name: str, res: dict, next_start: int) -> dict:
    return {
        "pod": pod_name,
        "chosen": res["chosen"],
        "nextStartNodeIndex": next_start,
        "nFeasible": res["n_feasible"],
        "filter": {n: ("passed" if pl is None else [pl, msg]) for n, (pl, msg) in res["filter"].items()},
        "score": res["raw"],
        "normalized": res["norm"],
        "total": res["total"],
    }


def run_case(name: str, nodes, bound, pods, pct: int, namespaces=None) -> dict:
    ref = ObjScheduler(nodes, bound, namespaces=namespaces, pct=pct, seed=SEED)
    doc = {
        "name": name,
        "percentageOfNodesToScore": pct,
        "tiebreakSeed": SEED,
        "hardPodAffinityWeight": 1,
        "namespaces": dict(namespaces or {}),
        "nodes": [k8sjson.node_to_dict(ni.node) for ni in ref.nodes],     # nodeTree order
        "boundPods": k8sjson.pods_to_list(list(bound)),
        "pods": k8sjson.pods_to_list(list(pods)),
        "expected": [],
    }
    for p in pods:
        res = ref.cycle(p)
        doc["expected"].append(_cycle_json(p.name, res, ref.next_start))
    return doc


def cases():
    import test_topology as tt
    nodes, pods = gen.config1_objects(n_nodes=100, n_pods=24)
    yield run_case("config1_p100", nodes, [], pods, 100)
    yield run_case("config1_adapt", nodes, [], pods, 0)
    nodes3, bound3, inc3 = gen.config3_objects(n_nodes=120, pods_per_node=3, n_incoming=30, zone_anti_every=40)
    yield run_case("config3_small_p100", nodes3, bound3, inc3, 100)
    hn = [tt._node(i, f"z{i % 2}") for i in range(6)]
    hb = [tt._pod("e0", {"app": "x"}, node="n0", pod_anti_affinity_required=[
        tt.PodAffinityTerm("topology.kubernetes.io/zone", tt.LabelSelector({"app": "y"}))])]
    hp = [tt._pod("y0", {"app": "y"}), tt._pod("x1", {"app": "z"}, pod_anti_affinity_required=[
        tt.PodAffinityTerm("kubernetes.io/hostname", tt.LabelSelector({"app": "x"}))])]
    yield run_case("ipa_hand_p100", hn, hb, hp, 100)
    # NodeAffinity's PreFilterResult (metadata.name matchFields) restricting the
    # scan; the harness models only sets of known nodes, so conflicting and
    # unknown-name pods are left out
    from ksim.encode import prefilter_node_names
    pn, pp = gen.prefilter_objects(n_nodes=150, n_pods=90)
    known = {n.name for n in pn}
    keep = [p for p in pp if prefilter_node_names(p) != [] and set(prefilter_node_names(p) or ()) <= known]
    yield run_case("prefilter_names_adapt", pn, [], keep, 0)


def main():
    os.makedirs(OUT, exist_ok=True)
    for doc in cases():
        path = os.path.join(OUT, doc["name"] + ".json.gz")
        with gzip.GzipFile(path, "wb", mtime=0) as f:
            f.write(json.dumps(doc, sort_keys=True, separators=(",", ":")).encode())
        print(path, os.path.getsize(path), "bytes,", len(doc["expected"]), "cycles")


if __name__ == "__main__":
    main()
