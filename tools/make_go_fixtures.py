"""Write the Go-harness fixtures (golden vectors item 4).

Each fixture under tests/golden/go/<case>.json.gz holds one scheduling run as
Kubernetes v1 documents (nodes in nodeTree order, bound pods, pending pods in
queue order, the profile knobs) and, under "expected", what the object-level
restatement (oracle/objref.py) records for every cycle: per-node filter result
("passed" or [plugin, message]), raw and normalized scores per score plugin,
totals, the chosen node and nextStartNodeIndex.  THE EXPECTED VALUES ARE
oracle/objref.py OUTPUTS, not Go outputs: a fixture pins nothing until
oracle/go writes its <case>.go.json.gz and tests/test_go_fixtures.py compares.

Optional inputs (round 5; absent = the default profile and none of them):
  profile             a v1beta2 KubeSchedulerProfile (pluginConfig: the plugin
                      args NewPluginConfig merges, plugins.go:103-179)
  services, replicaSets, statefulSets, replicationControllers
                      the objects helper.DefaultSelector reads (PodTopologySpread
                      System / List default constraints)
  pvs, pvcs           PersistentVolumes / claims (VolumeBinding, VolumeZone)
  nominatedPods, cycleInputs
                      the PodNominator before each cycle: {node: [pod names]} and
                      the pod's own status.nominatedNodeName
                      (RunFilterPluginsWithNominatedPods, evaluateNominatedNode)
  preemption          true: an unschedulable cycle also records DefaultPreemption's
                      dry run under "postFilter" (nominated node, victims; offset 0,
                      bound pods' status.startTime)

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
ASSUMED_START = 20000     # status.startTime (seconds after 2022-01-01T00:00:00Z) of pod i once assumed: 20000 + i


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


def run_case(name: str, nodes, bound, pods, pct: int, namespaces=None, extra=None, inputs=None,
             preemption=None) -> dict:
    """extra: the optional documents (profile, services, ..., pvs, pvcs,
    nominatedPods); inputs: per pod, the PodNominator ({node: [pod names]}) and
    the pod's nominated node; preemption: (start_time, order) of the bound pods
    to record DefaultPreemption's dry run after an unschedulable cycle."""
    extra = dict(extra or {})
    doc = {
        "name": name,
        "percentageOfNodesToScore": pct,
        "tiebreakSeed": SEED,
        "hardPodAffinityWeight": 1,
        "namespaces": dict(namespaces or {}),
        "boundPods": k8sjson.pods_to_list(list(bound)),
        "pods": k8sjson.pods_to_list(list(pods)),
        "expected": [],
    }
    doc.update(extra)
    if preemption is not None:
        doc["preemption"] = True
        start, _ = preemption
        for d, p in zip(doc["boundPods"], bound):
            d.setdefault("status", {})["startTime"] = _time(start[p.name])
    import gofixture
    ref = gofixture.objref(doc, nodes, bound)
    doc["nodes"] = [k8sjson.node_to_dict(ni.node) for ni in ref.nodes]     # nodeTree order
    nominated = gofixture.nominated_pods(doc)
    if inputs is not None:
        doc["cycleInputs"] = inputs
    for i, p in enumerate(pods):
        kw = gofixture.cycle_kwargs(doc, i, nominated)
        res = ref.cycle(p, **kw)
        c = _cycle_json(p.name, res, ref.next_start)
        if preemption is not None:
            start, order = preemption
            if res["chosen"] is None:
                node, victims = ref.preempt(p, p.priority, start, order, nominated=kw.get("nominated"))
                c["postFilter"] = {"nominatedNode": node, "victims": victims}
            else:                    # the assumed pod starts after every bound one (oracle/go sets it too)
                start[p.name] = ASSUMED_START + i
                order[p.name] = len(order)
        doc["expected"].append(c)
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
    yield from round5_cases()


def _profile(plugin_config):
    return {"profile": {"schedulerName": "default-scheduler", "pluginConfig": plugin_config}}


def round5_cases():
    """Cases for what rounds 3-4 built."""
    import copy
    import numpy as np
    from ksim.model import (Container, NodeSelectorTerm, Pod, PreferredTerm, Requirement)
    # NodeResourcesFit MostAllocated over cpu, memory and an extended resource,
    # with ignoredResources (the ignored resource is requested, never checked)
    nodes, pods = gen.config1_objects(n_nodes=100, n_pods=30)
    nodes = copy.deepcopy(nodes)
    pods = copy.deepcopy(pods)
    for i, n in enumerate(nodes):
        if i % 3:
            n.allocatable["example.com/gpu"] = str(i % 4)
    for j, p in enumerate(pods):
        if j % 3 == 0:
            p.containers[0].requests["example.com/gpu"] = "1"
        if j % 4 == 1:
            p.containers[0].requests["example.com/fpga"] = "2"
    yield run_case("args_most_allocated_p100", nodes, [], pods, 100, extra=_profile([
        {"name": "NodeResourcesFit", "args": {
            "scoringStrategy": {"type": "MostAllocated", "resources": [
                {"name": "cpu", "weight": 1}, {"name": "memory", "weight": 2},
                {"name": "example.com/gpu", "weight": 3}]},
            "ignoredResources": ["example.com/fpga"]}}]))
    # RequestedToCapacityRatio (a broken-linear shape), ADAPT
    nodes, pods = gen.config1_objects(n_nodes=120, n_pods=30)
    yield run_case("args_rtcr_adapt", nodes, [], pods, 0, extra=_profile([
        {"name": "NodeResourcesFit", "args": {"scoringStrategy": {
            "type": "RequestedToCapacityRatio",
            "resources": [{"name": "cpu", "weight": 2}, {"name": "memory", "weight": 1}],
            "requestedToCapacityRatio": {"shape": [{"utilization": 0, "score": 2},
                                                   {"utilization": 50, "score": 10},
                                                   {"utilization": 100, "score": 0}]}}}}]))
    # NodeAffinityArgs.addedAffinity: required (ANDed into Filter, errReasonEnforced)
    # and preferred (added to Score)
    nodes, pods = gen.config1_objects(n_nodes=100, n_pods=30)
    yield run_case("args_added_affinity_p100", nodes, [], pods, 100, extra=_profile([
        {"name": "NodeAffinity", "args": {"addedAffinity": {
            "requiredDuringSchedulingIgnoredDuringExecution": {"nodeSelectorTerms": [
                {"matchExpressions": [{"key": "pool", "operator": "In", "values": ["a", "b", "c"]}]}]},
            "preferredDuringSchedulingIgnoredDuringExecution": [
                {"weight": 7, "preference": {"matchExpressions": [
                    {"key": "disk", "operator": "In", "values": ["ssd"]}]}}]}}}]))
    # PodTopologySpread System defaults on ReplicaSet / Service / StatefulSet /
    # ReplicationController-owned pods (controller.go:79-80: the simulator runs
    # the Deployment and ReplicaSet controllers), and List defaults
    from test_spread_defaults import WORKLOADS, mixed_nodes, workload_pods
    sn = mixed_nodes(40, seed=4)
    sb = workload_pods(80, seed=12, bound_nodes=[n.name for n in sn])
    sq = workload_pods(30, seed=13)
    yield run_case("spread_system_defaults_adapt", sn, sb, sq, 0, extra=_workloads(*WORKLOADS))
    yield run_case("spread_list_defaults_p100", sn, sb, sq, 100, extra=dict(_workloads(*WORKLOADS), **_profile([
        {"name": "PodTopologySpread", "args": {"defaultingType": "List", "defaultConstraints": [
            {"maxSkew": 2, "topologyKey": "topology.kubernetes.io/zone", "whenUnsatisfiable": "DoNotSchedule"},
            {"maxSkew": 4, "topologyKey": "kubernetes.io/hostname", "whenUnsatisfiable": "ScheduleAnyway"}]}}])))
    # nominated pods: RunFilterPluginsWithNominatedPods (pass 1 with the
    # node's nominated pods of priority >= the pod's) and evaluateNominatedNode
    rng = np.random.default_rng(21)
    nn, _ = gen.config1_objects(n_nodes=60, n_pods=1)
    nq = [Pod(f"q{j}", priority=int(rng.choice([0, 10, 100])),
              containers=[Container({"cpu": f"{int(rng.integers(5, 40)) * 100}m",
                                     "memory": f"{int(rng.integers(1, 12))}Gi"})]) for j in range(30)]
    noms = [Pod(f"nom{k}", priority=int(rng.choice([0, 50, 1000])),
                containers=[Container({"cpu": f"{int(rng.integers(10, 60)) * 100}m",
                                       "memory": f"{int(rng.integers(2, 24))}Gi"})]) for k in range(12)]
    inputs = []
    for j in range(len(nq)):
        nominator = {}
        for k in rng.choice(len(noms), size=int(rng.integers(0, 6)), replace=False):
            nominator.setdefault(nn[int(rng.integers(0, 20))].name, []).append(noms[int(k)].name)
        inputs.append({"nominator": nominator,
                       "nominatedNodeName": nn[int(rng.integers(0, 60))].name if j % 4 == 3 else None})
    yield run_case("nominated_p100", nn, [], nq, 100, extra={"nominatedPods": k8sjson.pods_to_list(noms)},
                   inputs=inputs)
    # DefaultPreemption's dry run on a crowded cluster (unique start times)
    from test_preemption import crowded
    cn, cb, start, order = crowded(n_nodes=30, per_node=5, seed=7)
    start = {name: i * 7 % 10007 for i, name in enumerate(sorted(start))}
    cq = [Pod(f"p{i}", priority=int(rng.choice([0, 5, 50, 500, 5000])),
              containers=[Container({"cpu": f"{int(rng.integers(10, 300)) * 100}m",
                                     "memory": f"{int(rng.integers(4, 40))}Gi"})]) for i in range(30)]
    yield run_case("preemption_p100", cn, cb, cq, 100, preemption=(start, order))
    # VolumeBinding (claims bound to PVs: node affinity) and VolumeZone
    from test_volumes import volume_scenario
    vn, vp, pvs, pvcs = volume_scenario(n_nodes=36, n_pods=40)
    yield run_case("volumes_bound_p100", vn, [], [p for p in vp if p.pvc_claims or True], 100,
                   extra={"pvs": [_pv(v) for v in pvs], "pvcs": [_pvc(c) for c in pvcs]})


def _time(sec: int) -> str:
    return f"2022-01-01T{sec // 3600:02d}:{sec // 60 % 60:02d}:{sec % 60:02d}Z"


def _workloads(services, controllers):
    out = {"services": [], "replicaSets": [], "statefulSets": [], "replicationControllers": []}
    for s in services:
        spec = {} if s.selector is None else {"selector": dict(s.selector)}
        out["services"].append({"apiVersion": "v1", "kind": "Service",
                                "metadata": {"name": s.name, "namespace": s.namespace}, "spec": spec})
    for c in controllers:
        md = {"name": c.name, "namespace": c.namespace}
        if c.kind == "ReplicationController":
            spec = {} if c.selector is None else {"selector": dict(c.selector)}
            out["replicationControllers"].append({"apiVersion": "v1", "kind": c.kind, "metadata": md, "spec": spec})
        else:
            spec = {} if c.selector is None else {"selector": k8sjson._selector(c.selector)}
            key = "replicaSets" if c.kind == "ReplicaSet" else "statefulSets"
            out[key].append({"apiVersion": "apps/v1", "kind": c.kind, "metadata": md, "spec": spec})
    return out


def _pv(v):
    spec = {"capacity": {"storage": str(v.capacity)}, "accessModes": list(v.access_modes) or ["ReadWriteOnce"],
            v.source or "local": {"path": "/data"} if (v.source or "local") in ("local", "hostPath") else {}}
    if v.storage_class:
        spec["storageClassName"] = v.storage_class
    if v.node_affinity is not None:
        spec["nodeAffinity"] = {"required": {"nodeSelectorTerms": [k8sjson._term(t) for t in v.node_affinity]}}
    if v.source == "csi":
        spec["csi"] = {"driver": "csi.example.com", "volumeHandle": v.name}
    md = {"name": v.name}
    if v.labels:
        md["labels"] = dict(v.labels)
    return {"apiVersion": "v1", "kind": "PersistentVolume", "metadata": md, "spec": spec}


def _pvc(c):
    spec = {"volumeName": c.volume_name, "accessModes": list(c.access_modes) or ["ReadWriteOnce"],
            "resources": {"requests": {"storage": str(c.request or 1)}}}
    return {"apiVersion": "v1", "kind": "PersistentVolumeClaim",
            "metadata": {"name": c.name, "namespace": c.namespace}, "spec": spec,
            "status": {"phase": "Bound"} if c.volume_name else {}}


def main():
    os.makedirs(OUT, exist_ok=True)
    for doc in cases():
        path = os.path.join(OUT, doc["name"] + ".json.gz")
        with gzip.GzipFile(path, "wb", mtime=0) as f:
            f.write(json.dumps(doc, sort_keys=True, separators=(",", ":")).encode())
        print(path, os.path.getsize(path), "bytes,", len(doc["expected"]), "cycles")


if __name__ == "__main__":
    main()
