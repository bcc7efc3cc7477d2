"""Snapshot ingest: the reference's import/export documents
and UI object templates (tests/golden/reference/, extracted by
tools/make_ref_fixtures.py) -> engine inputs."""
import copy
import json
import os

import numpy as np
import pytest

from ksim import abi, ingest, profile
from oracle.objref import ObjScheduler
from oracle.oracle import Oracle

GOLD = os.path.join(os.path.dirname(__file__), "golden", "reference")


def _doc(name):
    return json.load(open(os.path.join(GOLD, name)))


def _same_profile(a, b):
    for f in ("n_filter", "n_score", "fit_n_res", "ba_n_res", "hard_pod_affinity_weight", "percentage_of_nodes_to_score"):
        assert getattr(a, f) == getattr(b, f), f
    assert list(a.filter[:a.n_filter]) == list(b.filter[:b.n_filter])
    assert list(a.score[:a.n_score]) == list(b.score[:b.n_score])
    assert list(a.score_weight[:a.n_score]) == list(b.score_weight[:b.n_score])
    assert list(a.fit_res[:a.fit_n_res]) == list(b.fit_res[:b.fit_n_res])
    assert list(a.ba_res[:a.ba_n_res]) == list(b.ba_res[:b.ba_n_res])


@pytest.mark.parametrize("name", ["export_case1.json", "export_case2.json", "import_case1.json"])
def test_reference_documents_profiles(name):
    """The exported default configuration converts to the default profile
    (order, weights, args; percentageOfNodesToScore forced to 0)."""
    snap = ingest.load(_doc(name))
    assert [n for n, _ in snap.profiles] == ["default-scheduler"]
    _same_profile(profile.compile_profile(snap.profiles[0][1]), profile.compile_profile(profile.SchedulerProfile()))
    assert snap.counts["pvs"] == len(_doc(name)["pvs"])


def test_priority_classes_and_queue_order():
    doc = _doc("export_case2.json")
    pc = _doc("template_priorityclass.json")
    pc = dict(pc, metadata={"name": "tmpl"})                 # globalDefault, value 1000
    doc["priorityClasses"] = doc["priorityClasses"] + [pc]
    tmpl = _doc("template_pod.json")
    pods = []
    for i, (prio_kw, ts) in enumerate([({}, "2022-01-01T00:00:03Z"), ({"priorityClassName": "system-node-critical"},
                                       "2022-01-01T00:00:05Z"), ({"priority": 5}, "2022-01-01T00:00:01Z"),
                                      ({}, "2022-01-01T00:00:02Z")]):
        p = copy.deepcopy(tmpl)
        p["metadata"] = {"name": f"p{i}", "namespace": "default", "creationTimestamp": ts}
        p["spec"].update(prio_kw)
        pods.append(p)
    doc["pods"] = pods
    snap = ingest.load(doc)
    assert [p.name for p in snap.pending] == ["p1", "p3", "p0", "p2"]
    assert [p.priority for p in snap.pending] == [2000001000, 1000, 1000, 5]


def _template_cluster(n_nodes=40, n_pods=300, bound_every=4):
    node_t, pod_t = _doc("template_node.json"), _doc("template_pod.json")
    nodes, pods = [], []
    for i in range(n_nodes):
        n = copy.deepcopy(node_t)
        n["metadata"] = {"name": f"node-{i}", "labels": {"kubernetes.io/hostname": f"node-{i}",
                                                         "topology.kubernetes.io/zone": f"z{i % 3}"}}
        n["status"]["allocatable"]["cpu"] = str(4 * (1 + i % 4))
        nodes.append(n)
    for i in range(n_pods):
        p = copy.deepcopy(pod_t)
        p["metadata"] = {"name": f"pod-{i}", "namespace": "default", "labels": {"app": f"a{i % 5}"},
                         "creationTimestamp": "2022-01-01T00:00:00Z"}
        req = p["spec"]["containers"][0]["resources"]["requests"]
        req["cpu"] = f"{100 * (1 + i % 10)}m"
        req["memory"] = f"{1 + i % 8}Gi"
        if i % bound_every == 0 and i < n_pods // 2:
            p["spec"]["nodeName"] = f"node-{(7 * i) % n_nodes}"
        pods.append(p)
    vol = copy.deepcopy(pod_t)
    vol["metadata"] = {"name": "with-pvc", "namespace": "default"}
    vol["spec"]["volumes"] = [{"name": "v", "persistentVolumeClaim": {"claimName": "pvc1"}}]
    pods.append(vol)
    doc = _doc("import_case1.json")
    doc["nodes"], doc["pods"] = nodes, pods
    return doc


@pytest.mark.parametrize("pct", [0, 100])
def test_template_cluster_schedules_like_objref(pct):
    """UI templates (node.yaml / pod.yaml) -> ingest -> C oracle placements
    equal the object-level restatement on the same objects; bound pods fill
    their nodes; the pod with a PVC (the sample's pvc1, bound to the hostPath
    PV pv1) is scheduled with VolumeBinding / VolumeZone (no node affinity, no
    topology labels: every node passes)."""
    snap = ingest.load(_template_cluster())
    assert snap.unsupported == []
    assert len(snap.bound) == 38 and len(snap.pending) == 300 - 38 + 1
    assert [p.name for p in snap.pending if p.pvc_claims] == ["with-pvc"]
    cluster, enc, prof = ingest.encode(snap)
    assert cluster.alloc_cpu.sum() == sum(4000 * (1 + i % 4) for i in range(40))
    assert cluster.req_mem.sum() == sum((1 + i % 8) << 30 for i in range(0, 150, 4))
    sp = copy.deepcopy(snap.profiles[0][1])
    sp.percentage_of_nodes_to_score = pct
    prof = profile.compile_profile(sp, cluster.scalar_names)
    ochosen, _ = Oracle(cluster, prof).schedule(enc)
    ref = ObjScheduler(snap.nodes, snap.bound, namespaces=snap.namespaces, pct=pct, seed=sp.tiebreak_seed,
                       pvs=snap.volumes.pvs.values(), pvcs=snap.volumes.pvcs.values())
    names = cluster.node_names
    for i, pod in enumerate(snap.pending):
        got = ref.cycle(pod)["chosen"]
        assert (names[ochosen[i]] if ochosen[i] >= 0 else None) == got, f"pod {i}"


def test_volume_documents_schedule_like_objref():
    """A document whose PVs (the UI's pv.yaml template) carry node affinity and
    zone labels: pods with claims bound to them are scheduled with
    VolumeBinding / VolumeZone, and placements equal the object-level
    restatement on the same PV / PVC objects.  A claim that does not exist and
    an unbound Immediate claim the PV controller finds no PV for reject their
    pods at PreFilter (unschedulable, not unsupported)."""
    doc = _template_cluster(n_nodes=30, n_pods=60, bound_every=1000)
    pv_t, pvc_t, pod_t = _doc("template_pv.json"), _doc("template_pvc.json"), _doc("template_pod.json")
    pvs, pvcs = [], []
    for k, (aff, zone) in enumerate([(None, "z1"), (["node-3", "node-4"], None), (None, "z0__z2"), (None, None)]):
        pv = copy.deepcopy(pv_t)
        pv["metadata"] = {"name": f"pv-{k}", "labels": ({"topology.kubernetes.io/zone": zone} if zone else {})}
        pv["spec"].pop("claimRef", None)
        if aff:
            pv["spec"]["nodeAffinity"] = {"required": {"nodeSelectorTerms": [{"matchExpressions": [
                {"key": "kubernetes.io/hostname", "operator": "In", "values": aff}]}]}}
        pvs.append(pv)
        pvc = copy.deepcopy(pvc_t)
        pvc["metadata"] = {"name": f"claim-{k}", "namespace": "default"}
        pvc["spec"]["volumeName"] = f"pv-{k}"
        pvcs.append(pvc)
    unbound = copy.deepcopy(pvc_t)
    unbound["metadata"] = {"name": "claim-unbound", "namespace": "default"}
    unbound["spec"].pop("volumeName", None)
    pvcs.append(unbound)
    for i in range(40):
        p = copy.deepcopy(pod_t)
        p["metadata"] = {"name": f"vol-{i}", "namespace": "default", "creationTimestamp": "2022-01-01T00:00:01Z"}
        claim = "claim-unbound" if i == 7 else f"claim-{i % 4}"
        p["spec"]["volumes"] = [{"name": "v", "persistentVolumeClaim": {"claimName": claim}}]
        doc["pods"].append(p)
    doc["pvs"], doc["pvcs"] = pvs, pvcs
    snap = ingest.load(doc)
    assert snap.unsupported == []
    cluster, enc, _ = ingest.encode(snap)
    # claim-1's PV has node affinity (10 pods); with-pvc (pvc1 is not in this
    # document) and vol-7 (claim-unbound) carry a group no node matches
    assert (enc.pods["vb_count"] > 0).sum() == 12 and (enc.pods["vz_count"] > 0).sum() == 20
    sp = copy.deepcopy(snap.profiles[0][1])
    sp.percentage_of_nodes_to_score = 100
    prof = profile.compile_profile(sp, cluster.scalar_names)
    ochosen, _ = Oracle(cluster, prof).schedule(enc)
    ref = ObjScheduler(snap.nodes, snap.bound, namespaces=snap.namespaces, pct=100, seed=sp.tiebreak_seed,
                       pvs=snap.volumes.pvs.values(), pvcs=snap.volumes.pvcs.values())
    names = cluster.node_names
    rejected = []
    for i, pod in enumerate(snap.pending):
        r = ref.cycle(pod)
        got = r["chosen"]
        assert (names[ochosen[i]] if ochosen[i] >= 0 else None) == got, f"pod {i} {pod.name}"
        if "prefilter" in r:
            rejected.append(pod.name)
    assert sorted(rejected) == ["vol-7", "with-pvc"]
    placed = {pod.name: names[ochosen[i]] for i, pod in enumerate(snap.pending) if pod.pvc_claims and ochosen[i] >= 0}
    aff = [placed[f"vol-{i}"] for i in range(1, 40, 4) if f"vol-{i}" in placed]   # pv-1: node-3 / node-4 only
    assert len(aff) >= 2 and set(aff) <= {"node-3", "node-4"}
