"""Unbound PersistentVolumeClaims: the PV controller's binding of Immediate
claims (a claim of a class that does not exist is Immediate), VolumeBinding's
static matching and dynamic provisioning of WaitForFirstConsumer claims
(FindPodVolumes, AssumePodVolumes: with no provisioner in the simulator the
pod waits in PreBind and its claims keep the selected node; ``provisioning``
models one), PreFilter rejections (missing claim, unbound Immediate claim)
recorded as VolumeBinding's PreFilter status, and the Filter reasons
(node affinity conflict, bind conflict, both) (ksim/volumes.py; SURVEY §8(f) 1,
/root/reference/simulator/export/export.go:47-49,59-61 carries pvs / pvcs /
storageClasses).

CPU: ksim.ingest.schedule_queue on the C oracle (the encoder's volume groups
under the bindings the run has made) against the object-level restatement
oracle/objref.py, which restates FindMatchingVolume / FindPodVolumes on the
objects themselves.  GPU (``gpu``): the same queue on the engine against the
oracle.  Parity unpinned against Go (v1.26 source restated, no Go run)."""
import copy

import numpy as np
import pytest

from ksim import profile
from ksim.encode import encode_cluster
from ksim.ingest import schedule_queue
from ksim.model import (Container, LabelSelector, Node, NodeSelectorTerm, PersistentVolume, PersistentVolumeClaim,
                        Pod, Requirement, StorageClass, storage_class_from_dict)
from ksim.volumes import VolumeIndex
from oracle.objref import ObjScheduler
from oracle.oracle import Oracle

ZONE = "topology.kubernetes.io/zone"
HOST = "kubernetes.io/hostname"
GI = 1 << 30


def binding_scenario(seed=0, n_nodes=40, n_pods=150):
    rng = np.random.default_rng(seed)
    nodes = [Node(name=f"n{i:03d}", labels={HOST: f"n{i:03d}", ZONE: f"z{i % 3}"},
                  allocatable={"cpu": "16", "memory": "64Gi", "pods": "110"}) for i in range(n_nodes)]
    classes = [StorageClass("local", "kubernetes.io/no-provisioner", "WaitForFirstConsumer"),
               StorageClass("zonal", "csi.example.com", "WaitForFirstConsumer",
                            [[(ZONE, ["z0", "z1"])], []]),
               StorageClass("fast", "csi.example.com", "WaitForFirstConsumer"),
               StorageClass("imm", "kubernetes.io/no-provisioner", "Immediate"),
               StorageClass("blank", "", "WaitForFirstConsumer")]
    pvs, pvcs = [], []
    for k in range(60):                                  # local PVs: one host each, mixed sizes
        host = f"n{int(rng.integers(0, n_nodes)):03d}"
        pvs.append(PersistentVolume(
            name=f"local-{k:02d}", capacity=int(rng.integers(1, 6)) * GI, storage_class="local",
            access_modes=["ReadWriteOnce"], labels={"tier": ["gold", "silver"][k % 2]},
            node_affinity=[NodeSelectorTerm([Requirement(HOST, "In", [host])])], source="local",
            deleting=(k % 29 == 28)))
    for k in range(12):                                  # zonal PVs
        pvs.append(PersistentVolume(name=f"zonal-{k:02d}", capacity=(k % 3 + 1) * 2 * GI, storage_class="zonal",
                                    access_modes=["ReadWriteOnce", "ReadOnlyMany"],
                                    node_affinity=[NodeSelectorTerm([Requirement(ZONE, "In", [f"z{k % 3}"])])]))
    pvs.append(PersistentVolume(name="imm-a", capacity=2 * GI, storage_class="imm", access_modes=["ReadWriteOnce"]))
    pvs.append(PersistentVolume(name="imm-b", capacity=8 * GI, storage_class="imm", access_modes=["ReadWriteOnce"]))
    # a PV pre-bound to a WaitForFirstConsumer claim (claimRef set, claim unbound)
    pvs.append(PersistentVolume(name="local-pre", capacity=GI, storage_class="local", access_modes=["ReadWriteOnce"],
                                node_affinity=[NodeSelectorTerm([Requirement(HOST, "In", ["n005"])])],
                                claim_ref=("default", "c-pre")))
    pods = []
    for j in range(n_pods):
        claims = []
        for q in range(int(rng.choice([0, 1, 1, 2]))):
            name = f"c-{j}-{q}"
            kind = int(rng.integers(0, 10))
            cls = ["local", "local", "local", "zonal", "zonal", "fast", "imm", "local", "zonal", "local"][kind]
            sel = LabelSelector({"tier": "gold"}) if (cls == "local" and j % 7 == 3) else None
            modes = ["ReadOnlyMany"] if (cls == "zonal" and j % 5 == 4) else ["ReadWriteOnce"]
            pvcs.append(PersistentVolumeClaim(name=name, storage_class=cls, request=int(rng.integers(1, 5)) * GI,
                                              selector=sel, access_modes=modes))
            claims.append(name)
        if j == 10:
            claims.append("c-pre")
        if j == 20:
            claims.append("c-missing")
        if j == 30:
            pvcs.append(PersistentVolumeClaim(name="c-noclass", storage_class="gone"))
            claims.append("c-noclass")
        if j in (40, 41, 60):                           # one provisioned claim, then its later users
            if j == 40:
                pvcs.append(PersistentVolumeClaim(name="c-prov", storage_class="fast", request=GI,
                                                  access_modes=["ReadWriteOnce"]))
            claims.append("c-prov")
        if j == 70:                                     # a class with an empty provisioner cannot provision
            pvcs.append(PersistentVolumeClaim(name="c-noprov", storage_class="blank", request=100 * GI,
                                              access_modes=["ReadWriteOnce"]))
            claims.append("c-noprov")
        if j in (50, 51):                               # the same local claim twice: the second finds it bound
            if j == 50:
                pvcs.append(PersistentVolumeClaim(name="c-shared", storage_class="local", request=GI,
                                                  access_modes=["ReadWriteOnce"]))
            claims.append("c-shared")
        pods.append(Pod(f"p{j:03d}", containers=[Container({"cpu": "1", "memory": "2Gi"})], pvc_claims=claims))
    pvcs.append(PersistentVolumeClaim(name="c-pre", storage_class="local", request=GI, access_modes=["ReadWriteOnce"]))
    return nodes, pods, pvs, pvcs, classes


def _objref(nodes, pvs, pvcs, classes, pct, seed, provisioning=False):
    return ObjScheduler(nodes, [], pct=pct, seed=seed, pvs=pvs, pvcs=pvcs, storage_classes=classes,
                        provisioning=provisioning)


def run_queue(backend_factory, nodes, pods, pvs, pvcs, classes, pct=100, provisioning=False):
    vol = VolumeIndex.from_nodes(nodes, copy.deepcopy(pvs), copy.deepcopy(pvcs), classes, provisioning)
    vol.run_pv_controller()
    cluster, _ = encode_cluster(nodes)
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=pct)
    prof = profile.compile_profile(sp)
    backend = backend_factory(cluster, prof)
    got = schedule_queue(backend, cluster, pods, vol, nodes)
    return got, vol, backend, sp


@pytest.mark.parametrize("seed,pct,prov", [(0, 100, False), (1, 0, False), (2, 100, True), (3, 0, True)])
def test_binding_queue_vs_objref(seed, pct, prov):
    nodes, pods, pvs, pvcs, classes = binding_scenario(seed)
    got, vol, _, sp = run_queue(lambda c, p: Oracle(c, p), nodes, pods, pvs, pvcs, classes, pct, prov)
    ref = _objref(nodes, pvs, pvcs, classes, pct, sp.tiebreak_seed, prov)
    want, rejected = [], 0
    for pod in pods:
        r = ref.cycle(pod)
        want.append(r["chosen"])
        rejected += "prefilter" in r
    assert got == want
    # every path ran: static binds, provisioning, PreFilter rejections, unschedulable pods
    assert rejected >= 2 and None in got
    assert (vol.provisioned > 0) == prov and (len(vol.waiting) > 0) == (not prov)
    bound_static = sum(1 for pv in vol.pvs.values() if pv.claim_ref and not pv.name.startswith("pvc-provisioned"))
    assert bound_static > 10
    # the same bindings (and provisioning nodes) on both sides
    assert {n: pv.claim_ref for n, pv in vol.pvs.items()} == {n: pv.claim_ref for n, pv in ref.pvs.items()}
    assert {k: c.selected_node for k, c in vol.pvcs.items()} == {k: c.selected_node for k, c in ref.pvcs.items()}
    if not prov:                          # the later users of the claim waiting on a node follow it
        users = [got[j] for j in (40, 41, 60)]
        assert users[0] is not None and all(u in (users[0], None) for u in users)


def test_missing_class_claims_are_immediate():
    """IsDelayBindingMode: a class that does not exist is not delay binding, so
    the PV controller binds the claim like an Immediate one (a PV naming the
    same class), or the pod is rejected at PreFilter while it stays unbound."""
    vol = VolumeIndex([PersistentVolume("g", capacity=GI, storage_class="gone", access_modes=["ReadWriteOnce"])],
                      [PersistentVolumeClaim("a", storage_class="gone", request=GI, access_modes=["ReadWriteOnce"]),
                       PersistentVolumeClaim("b", storage_class="gone", request=GI, access_modes=["ReadWriteOnce"])])
    assert vol.run_pv_controller() == 1
    assert vol.pvcs[("default", "a")].volume_name == "g"
    assert vol.prefilter_rejection(Pod("p", pvc_claims=["a"])) is None
    assert vol.prefilter_rejection(Pod("q", pvc_claims=["b"])) == "pod has unbound immediate PersistentVolumeClaims"


def test_prefilter_rejections_and_reasons_recorded():
    """Compat annotations: a missing claim / unbound Immediate claim is
    VolumeBinding's PreFilter status (no Filter entries, every node in
    PostFilter); a node failing both a bound PV's affinity and an unbound
    claim's matching gets both reasons, joined in FindPodVolumes' order."""
    from ksim.encode import encode_pods
    from ksim.resultstore import Store
    from ksim.wrapped import compat_cycle
    nodes = [Node(name=f"n{i}", labels={HOST: f"n{i}", ZONE: f"z{i % 2}"},
                  allocatable={"cpu": "8", "memory": "8Gi", "pods": "10"}) for i in range(4)]
    aff = lambda key, vals: [NodeSelectorTerm([Requirement(key, "In", vals)])]
    pvs = [PersistentVolume("zpv", capacity=GI, storage_class="local", access_modes=["ReadWriteOnce"],
                            node_affinity=aff(ZONE, ["z0"])),
           PersistentVolume("hpv", capacity=GI, storage_class="local", access_modes=["ReadWriteOnce"],
                            node_affinity=aff(HOST, ["n0", "n1"]))]
    pvcs = [PersistentVolumeClaim("bound", storage_class="local", volume_name="zpv", access_modes=["ReadWriteOnce"]),
            PersistentVolumeClaim("wffc", storage_class="local", request=GI, access_modes=["ReadWriteOnce"]),
            PersistentVolumeClaim("imm", request=GI, access_modes=["ReadWriteOnce"])]
    classes = [StorageClass("local", "kubernetes.io/no-provisioner", "WaitForFirstConsumer")]
    vol = VolumeIndex.from_nodes(nodes, pvs, pvcs, classes)
    vol.run_pv_controller()
    pods = [Pod("both", pvc_claims=["bound", "wffc"]), Pod("gone", pvc_claims=["nope"]),
            Pod("immediate", pvc_claims=["imm"])]
    cluster, _ = encode_cluster(nodes)
    enc = encode_pods(cluster, pods, volumes=vol)
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=100)
    ora = Oracle(cluster, profile.compile_profile(sp))
    st = Store(profile.default_score_weights())
    got = [compat_cycle(ora, st, cluster, sp, enc, i)["chosen"] for i in range(3)]
    assert got[1] < 0 and got[2] < 0
    ref = _objref(nodes, pvs, pvcs, classes, 100, sp.tiebreak_seed)
    r = ref.cycle(pods[0])
    assert cluster.node_names[got[0]] == r["chosen"] == "n0"
    res = st.results["default/both"]
    msgs = {n: res.filter[n]["VolumeBinding"] for n in ("n1", "n2", "n3")}
    assert msgs == {n: r["filter"][n][1] for n in msgs}
    assert msgs["n3"] == "node(s) had volume node affinity conflict, node(s) didn't find available persistent " \
                         "volumes to bind"
    assert msgs["n2"] == "node(s) didn't find available persistent volumes to bind"
    assert msgs["n1"] == "node(s) had volume node affinity conflict"
    for name, msg in (("gone", 'persistentvolumeclaim "nope" not found'),
                      ("immediate", "pod has unbound immediate PersistentVolumeClaims")):
        res = st.results["default/" + name]
        assert res.pre_filter_status["VolumeBinding"] == msg and not res.filter
        assert "NodeAffinity" not in res.pre_filter_status      # RunPreFilterPlugins stopped
        assert set(res.post_filter) == {n.name for n in nodes}


def test_pv_controller_binds_immediate_claims():
    vol = VolumeIndex([PersistentVolume("a", capacity=2 * GI, access_modes=["ReadWriteOnce"]),
                       PersistentVolume("b", capacity=1 * GI, access_modes=["ReadWriteOnce"]),
                       PersistentVolume("c", capacity=5 * GI, access_modes=["ReadOnlyMany"]),
                       PersistentVolume("d", capacity=9 * GI, storage_class="slow", access_modes=["ReadWriteOnce"])],
                      [PersistentVolumeClaim("x", request=GI, access_modes=["ReadWriteOnce"]),
                       PersistentVolumeClaim("y", request=GI, access_modes=["ReadWriteOnce"]),
                       PersistentVolumeClaim("z", request=GI, access_modes=["ReadWriteOnce"]),
                       PersistentVolumeClaim("w", request=GI, storage_class="slow", access_modes=["ReadWriteOnce"]),
                       PersistentVolumeClaim("v", request=GI, storage_class="wffc", access_modes=["ReadWriteOnce"])],
                      classes=[StorageClass("slow", "", "Immediate"), StorageClass("wffc", "", "WaitForFirstConsumer")])
    assert vol.run_pv_controller() == 3
    got = {k[1]: c.volume_name for k, c in vol.pvcs.items()}
    assert got == {"x": "b", "y": "a", "z": "", "w": "d", "v": ""}   # smallest first; modes; class; delay


def test_competing_claims_get_an_exact_group():
    """Two claims of one pod whose only PVs on a node are the same PV: the
    node fails (FindPodVolumes' chosenPVs), which per-claim OR groups cannot
    express; the exact group lists the nodes where the whole match succeeds."""
    nodes = [Node(name=f"n{i}", labels={HOST: f"n{i}"}, allocatable={"cpu": "8", "memory": "8Gi", "pods": "10"})
             for i in range(4)]
    aff = lambda h: [NodeSelectorTerm([Requirement(HOST, "In", h)])]
    pvs = [PersistentVolume("big", capacity=4 * GI, storage_class="local", access_modes=["ReadWriteOnce"],
                            node_affinity=aff(["n0", "n1"])),
           PersistentVolume("small", capacity=GI, storage_class="local", access_modes=["ReadWriteOnce"],
                            node_affinity=aff(["n1", "n2"]))]
    pvcs = [PersistentVolumeClaim("a", storage_class="local", request=GI, access_modes=["ReadWriteOnce"]),
            PersistentVolumeClaim("b", storage_class="local", request=GI, access_modes=["ReadWriteOnce"])]
    classes = [StorageClass("local", "kubernetes.io/no-provisioner", "WaitForFirstConsumer")]
    vol = VolumeIndex.from_nodes(nodes, pvs, pvcs, classes)
    pod = Pod("p", containers=[Container({"cpu": "1"})], pvc_claims=["a", "b"])
    vb, _, _ = vol.groups(pod)
    assert len(vb) == 1 and [t.match_fields[0].values[0] for t in vb[0]] == ["n1"]
    got, vol2, _, sp = run_queue(lambda c, p: Oracle(c, p), nodes, [pod], pvs, pvcs, classes)
    ref = _objref(nodes, pvs, pvcs, classes, 100, sp.tiebreak_seed)
    assert got == [ref.cycle(pod)["chosen"]] == ["n1"]
    assert vol2.pvcs[("default", "a")].volume_name == "small" and vol2.pvcs[("default", "b")].volume_name == "big"


def test_storage_class_from_dict():
    sc = storage_class_from_dict({"metadata": {"name": "s"}, "provisioner": "p",
                                  "volumeBindingMode": "WaitForFirstConsumer",
                                  "allowedTopologies": [{"matchLabelExpressions": [{"key": ZONE, "values": ["z1"]}]}]})
    assert (sc.name, sc.provisioner, sc.volume_binding_mode, sc.allowed_topologies) == \
        ("s", "p", "WaitForFirstConsumer", [[(ZONE, ["z1"])]])
    sc = storage_class_from_dict({"metadata": {"name": "d"}, "provisioner": "kubernetes.io/no-provisioner"})
    assert sc.volume_binding_mode == "Immediate" and sc.allowed_topologies == []


# ---- device -------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("seed,pct", [(3, 100), (4, 0)])
def test_binding_queue_engine_vs_oracle(seed, pct):
    from ksim.engine import Engine

    def engine(c, p):
        e = Engine(0)
        e.set_profile(p)
        e.set_cluster(c)
        return e
    nodes, pods, pvs, pvcs, classes = binding_scenario(seed, n_nodes=300, n_pods=700)
    got, vol, eng, _ = run_queue(engine, nodes, pods, pvs, pvcs, classes, pct)
    want, vol_o, ora, _ = run_queue(lambda c, p: Oracle(c, p), nodes, pods, pvs, pvcs, classes, pct)
    assert got == want
    assert {n: pv.claim_ref for n, pv in vol.pvs.items()} == {n: pv.claim_ref for n, pv in vol_o.pvs.items()}
    es, os_ = eng.node_state(), ora.node_state()
    for k in es:
        np.testing.assert_array_equal(es[k], os_[k], err_msg=k)
