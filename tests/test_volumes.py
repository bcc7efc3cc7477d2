"""VolumeBinding and VolumeZone for pods with bound PersistentVolumeClaims
(ksim/volumes.py, ksim_engine.h "Volume groups").

CPU: the C oracle on the encoder's volume groups against the object-level
restatement oracle/objref.py (binder.go checkBoundClaims / CheckNodeAffinity,
volume_zone.go Filter on PV and PVC objects), cycle by cycle: filter outcome
and message per node, placement.  GPU (``gpu``): the engine against the
oracle.  Parity unpinned against Go (restated from v1.26 source, no Go run)."""
import numpy as np
import pytest

from ksim import abi, profile
from ksim.encode import encode_cluster, encode_pods
from ksim.model import (Container, Node, NodeSelectorTerm, PersistentVolume, PersistentVolumeClaim, Pod,
                        Requirement, pod_from_dict, pv_from_dict, pvc_from_dict)
from ksim.volumes import VolumeIndex, label_zones_to_set
from ksim.wrapped import filter_message
from oracle.objref import ObjScheduler
from oracle.oracle import Oracle

ZONE = "topology.kubernetes.io/zone"
REGION = "topology.kubernetes.io/region"
BETA_ZONE = "failure-domain.beta.kubernetes.io/zone"


def volume_scenario(seed=0, n_nodes=48, n_pods=160):
    rng = np.random.default_rng(seed)
    nodes = []
    for i in range(n_nodes):
        labels = {"kubernetes.io/hostname": f"n{i:03d}", "disk": ["ssd", "hdd"][i % 2]}
        if i % 8 != 7:                                        # some nodes carry no topology label
            labels[ZONE] = f"z{i % 3}"
            labels[REGION] = "r0" if i % 3 < 2 else "r1"
        if i % 5 == 0:
            labels[BETA_ZONE] = f"z{i % 3}"
        nodes.append(Node(name=f"n{i:03d}", labels=labels,
                          allocatable={"cpu": "32", "memory": "128Gi", "pods": "110"}))
    pvs, pvcs = [], []

    def pv(name, **kw):
        pvs.append(PersistentVolume(name=name, source=kw.pop("source", "local"), **kw))

    # node affinity: one host, a zone set, a disk type; a matchFields term (never
    # matches: CheckNodeAffinity's node has no name); empty required terms
    pv("pv-host", node_affinity=[NodeSelectorTerm([Requirement("kubernetes.io/hostname", "In", ["n007"])])])
    pv("pv-zone01", node_affinity=[NodeSelectorTerm([Requirement(ZONE, "In", ["z0", "z1"])])])
    pv("pv-ssd-or-z2", node_affinity=[NodeSelectorTerm([Requirement("disk", "In", ["ssd"])]),
                                      NodeSelectorTerm([Requirement(ZONE, "In", ["z2"])])])
    pv("pv-field", node_affinity=[NodeSelectorTerm([], [Requirement("metadata.name", "In", ["n003"])])])
    pv("pv-field-notin", node_affinity=[NodeSelectorTerm([Requirement("disk", "Exists", [])],
                                                         [Requirement("metadata.name", "NotIn", ["n004"])])])
    pv("pv-none", node_affinity=[])
    # topology labels (VolumeZone): one zone, a "__" set, a region, a bad value, a beta key
    pv("pv-lz1", labels={ZONE: "z1"})
    pv("pv-lz02", labels={ZONE: "z0__z2", REGION: "r0"})
    pv("pv-lr1", labels={REGION: "r1"}, source="csi")
    pv("pv-lbad", labels={ZONE: "z1____z2"})
    pv("pv-lbeta", labels={BETA_ZONE: "z0"}, node_affinity=[NodeSelectorTerm([Requirement("disk", "In", ["hdd"])])])
    pv("pv-plain")
    names = [p.name for p in pvs]
    for k, n in enumerate(names):
        pvcs.append(PersistentVolumeClaim(name=f"c-{n}", namespace="default", volume_name=n))
    pods = []
    for j in range(n_pods):
        k = int(rng.integers(0, 3))
        claims = [f"c-{names[x]}" for x in rng.choice(len(names), size=k, replace=False)] if k else []
        if j % 11 == 0:
            claims = ["c-pv-none"]
        pods.append(Pod(name=f"p{j}", containers=[Container({"cpu": "500m", "memory": "1Gi"})], pvc_claims=claims))
    return nodes, pods, pvs, pvcs


def run_both(nodes, pods, pvs, pvcs, pct):
    cluster, _ = encode_cluster(nodes)
    enc = encode_pods(cluster, pods, volumes=VolumeIndex.from_nodes(nodes, pvs, pvcs))
    assert not (enc.pods["flags"] & abi.POD_HAS_VOLUMES).any()
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=pct)
    prof = profile.compile_profile(sp)
    ora = Oracle(cluster, prof)
    ref = ObjScheduler(nodes, [], pct=pct, seed=sp.tiebreak_seed, pvs=pvs, pvcs=pvcs)
    forder = sp.filter_order()
    names = cluster.node_names
    seen = set()
    for i, pod in enumerate(pods):
        o = ora.cycle(enc, i)
        r = ref.cycle(pod)
        for pos, name in enumerate(names):
            fp = int(o["fail_plugin"][pos])
            if fp == abi.NOT_EVALUATED:
                continue
            pl, msg = r["filter"][name]
            if fp == abi.PASSED:
                assert pl is None, f"pod {i} node {name}: oracle passed, objref {pl}: {msg}"
            else:
                seen.add(forder[fp])
                assert pl == forder[fp], f"pod {i} node {name}: oracle {forder[fp]} objref {pl}"
                assert msg == filter_message(cluster, forder[fp], int(o["fail_detail"][pos]))
        got = names[o["chosen"]] if o["chosen"] >= 0 else None
        assert got == r["chosen"], f"pod {i}"
    assert {"VolumeBinding", "VolumeZone"} <= seen
    return cluster, enc, prof


def test_label_zones_to_set():
    assert label_zones_to_set("z0__z1") == ["z0", "z1"]
    assert label_zones_to_set(" z0 ") == ["z0"]
    assert label_zones_to_set("z0____z1") is None


@pytest.mark.parametrize("pct", [0, 100])
def test_volume_filters_vs_objref(pct):
    nodes, pods, pvs, pvcs = volume_scenario()
    run_both(nodes, pods, pvs, pvcs, pct)


def test_unsupported_claims_are_flagged():
    """Volumes counted against node limits and ReadWriteOncePod claims (feature
    gate off in v1.26) are flagged (not scheduled); a missing claim and an
    unbound Immediate claim reject the pod at PreFilter (recorded as
    VolumeBinding's PreFilter status; the engine gets a group no node matches)."""
    nodes, _, pvs, pvcs = volume_scenario()
    pvs = pvs + [PersistentVolume(name="pv-ebs", source="awsElasticBlockStore")]
    pvcs = pvcs + [PersistentVolumeClaim(name="c-ebs", volume_name="pv-ebs"),
                   PersistentVolumeClaim(name="c-unbound"),
                   PersistentVolumeClaim(name="c-rwop", volume_name="pv-plain", access_modes=["ReadWriteOncePod"])]
    pods = [Pod(name=f"x{k}", pvc_claims=[c]) for k, c in enumerate(["c-ebs", "c-unbound", "c-rwop", "c-missing"])]
    pods.append(Pod(name="ok", pvc_claims=["c-pv-plain"]))
    cluster, _ = encode_cluster(nodes)
    enc = encode_pods(cluster, pods, volumes=VolumeIndex.from_nodes(nodes, pvs, pvcs))
    flags = enc.pods["flags"] & abi.POD_HAS_VOLUMES
    assert list(flags != 0) == [True, False, True, False, False]
    assert list(enc.pods["vb_count"] > 0) == [False, True, False, True, False]
    assert [enc.rejection(i) for i in range(5)] == [
        None, ("VolumeBinding", "pod has unbound immediate PersistentVolumeClaims"), None,
        ("VolumeBinding", 'persistentvolumeclaim "c-missing" not found'), None]
    # CSI volumes count against attachable-volumes-* node limits when a node publishes one
    nodes2 = nodes + [Node(name="lim", allocatable={"cpu": "1", "attachable-volumes-csi-x": "10"})]
    enc2 = encode_pods(encode_cluster(nodes2)[0], [Pod(name="c", pvc_claims=["c-pv-lr1"])],
                       volumes=VolumeIndex.from_nodes(nodes2, pvs, pvcs))
    assert enc2.pods["flags"][0] & abi.POD_HAS_VOLUMES


def test_pv_pvc_from_v1_dicts():
    pv = pv_from_dict({"metadata": {"name": "v", "labels": {ZONE: "z1"}},
                       "spec": {"local": {"path": "/d"}, "nodeAffinity": {"required": {"nodeSelectorTerms": [
                           {"matchExpressions": [{"key": "k", "operator": "In", "values": ["a"]}]}]}}}})
    assert pv.source == "local" and pv.labels == {ZONE: "z1"} and pv.node_affinity[0].match_expressions[0].key == "k"
    pvc = pvc_from_dict({"metadata": {"name": "c", "namespace": "ns"}, "spec": {"volumeName": "v"}})
    assert (pvc.namespace, pvc.volume_name) == ("ns", "v")
    pod = pod_from_dict({"metadata": {"name": "p"}, "spec": {"volumes": [
        {"name": "a", "persistentVolumeClaim": {"claimName": "c"}}, {"name": "b", "emptyDir": {}}]}})
    assert pod.pvc_claims == ["c"] and not pod.has_volumes


# ---- device -------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("pct", [0, 100])
def test_volume_filters_engine_vs_oracle(pct):
    from ksim.engine import Engine
    nodes, pods, pvs, pvcs = volume_scenario(seed=3, n_nodes=300, n_pods=900)
    cluster, _ = encode_cluster(nodes)
    enc = encode_pods(cluster, pods, volumes=VolumeIndex.from_nodes(nodes, pvs, pvcs))
    prof = profile.compile_profile(profile.SchedulerProfile(percentage_of_nodes_to_score=pct))
    ora = Oracle(cluster, prof)
    eng = Engine(0)
    eng.set_profile(prof)
    eng.set_cluster(cluster)
    for i in range(60):                                    # compat cycles: every per-node output
        e, o = eng.eval_pod(enc, i), ora.cycle(enc, i)
        for k in ("fail_plugin", "fail_detail", "total"):
            np.testing.assert_array_equal(e[k], o[k], err_msg=f"pod {i} {k}")
        assert e["chosen"] == o["chosen"]
    eng.set_cluster(cluster)                               # a loaded-queue run of every pod
    eng.load_pods(enc)
    chosen, st = eng.schedule_loaded(0, enc.n_pods)
    ochosen, ost = Oracle(cluster, prof).schedule(enc)
    np.testing.assert_array_equal(chosen, ochosen)
    assert st.evals == ost.evals
    eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_volume_filters_sharded(world):
    """Volume pods on the node-sharded per-pod cycle (in-process shard group)."""
    from ksim.engine import Engine, group_schedule_loaded
    from ksim.shard import partition
    nodes, pods, pvs, pvcs = volume_scenario(seed=5, n_nodes=200, n_pods=500)
    cluster, _ = encode_cluster(nodes)
    enc = encode_pods(cluster, pods, volumes=VolumeIndex.from_nodes(nodes, pvs, pvcs))
    prof = profile.compile_profile(profile.SchedulerProfile(percentage_of_nodes_to_score=0))
    engines = []
    for base, cnt in partition(cluster.n_nodes, world):
        e = Engine(0)
        e.set_shard(base, cluster.n_nodes)
        e.set_profile(prof)
        e.set_cluster(cluster.shard(base, cnt))
        e.load_pods(enc)
        engines.append(e)
    chosen, st = group_schedule_loaded(engines, 0, enc.n_pods)
    ochosen, ost = Oracle(cluster, prof).schedule(enc)
    np.testing.assert_array_equal(chosen, ochosen)
    assert st.evals == ost.evals
    for e in engines:
        e.close()
