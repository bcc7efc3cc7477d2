"""The native snapshot encoder (csrc/ksim_encode.cpp, ksim_encode_nodes /
ksim_encode_pods, ABI 10) against the Python compile it restates
(ksim/encode.py + ksim/topology.py): every node-table, vocabulary and pod-set
array byte for byte, and the host metadata (node order, label / taint /
scalar vocabularies), on the configs' object distributions, the reference's
own sample export documents and UI templates (tests/golden/reference), the
Go-harness documents (tests/golden/go), PodTopologySpread default
constraints, volumes, NetworkBandwidth, NodePorts / ImageLocality,
NodeAffinity PreFilterResult names, plugin args and node informer deltas.
Host code: no GPU."""
import copy
import gzip
import glob
import json
import os

import numpy as np
import pytest

from ksim import abi, gen, ingest, nativeenc, profile
from ksim.encode import EncodeError, encode_cluster, encode_pods
from ksim.model import (Container, ContainerPort, LabelSelector, Node, NodeSelectorTerm, PodAffinityTerm,
                        PreferredTerm, Pod, Requirement, Taint, Toleration, TopologySpreadConstraint,
                        WeightedPodAffinityTerm, node_from_dict, pod_from_dict)
from ksim.topology import SpreadDefaults
from ksim.volumes import VolumeIndex

from native_compare import both, same_cluster, same_pods

HERE = os.path.dirname(__file__)


def test_config1():
    nodes, pods = gen.config1_objects(n_nodes=100, n_pods=1000)
    both(nodes, [], [pods])


def test_config3():
    nodes, bound, inc = gen.config3_objects(n_nodes=600, pods_per_node=5, n_incoming=400, zone_anti_every=37)
    both(nodes, bound, [inc])


def test_queues_in_turn():
    """Label columns and classes accumulate over encode_pods calls on one
    snapshot (ksim/ingest.py schedule_queue re-encodes pods at their turn)."""
    nodes, bound, inc = gen.config3_objects(n_nodes=200, pods_per_node=3, n_incoming=120)
    _, c1 = gen.config1_objects(n_nodes=200, n_pods=50)     # selectors on keys of the config-1 labels
    both(nodes, bound, [inc[:40], c1, inc[40:]])


@pytest.mark.parametrize("errors", [False, True])
def test_network_bandwidth(errors):
    nodes, bound, pods = gen.netbw_objects(node_errors=errors, pod_errors=errors)
    both(nodes, bound, [pods])


def test_prefilter_names():
    nodes, pods = gen.prefilter_objects(n_nodes=300, n_pods=600)
    both(nodes, [], [pods])


def test_edge_quantities():
    nodes, bound, pods = gen.edge_objects()
    both(nodes, bound, [pods])


def test_delta_objects():
    nodes, bound, pending, _ = gen.delta_objects(n_nodes=120, n_pods=300)
    both(nodes, bound, [pending])


def test_ports_images_tolerations():
    """NodePorts classes (any-ip and per-ip), ImageLocality classes, taints
    with every effect, tolerations of every operator."""
    rng = np.random.default_rng(5)
    images = [(["nginx:1.25", "docker.io/nginx:1.25"], 180 * 2 ** 20), (["redis"], 40 * 2 ** 20),
              (["busybox:latest"], 2 * 2 ** 20), (["registry:5000/app"], 900 * 2 ** 20)]
    nodes = []
    for i in range(80):
        taints = [Taint("dedicated", ["gpu", "infra"][i % 2], ["NoSchedule", "NoExecute", "PreferNoSchedule"][i % 3])
                  ] if i % 4 == 0 else []
        nodes.append(Node(f"n{i}", {"kubernetes.io/hostname": f"n{i}", "topology.kubernetes.io/zone": f"z{i % 3}"},
                          taints, {"cpu": "8", "memory": "32Gi", "pods": "110"},
                          images=[images[k] for k in range(4) if (i >> k) & 1]))
    bound, pods = [], []
    for j in range(150):
        ports = [ContainerPort(int(rng.choice([80, 443, 8080])), str(rng.choice(["TCP", "UDP", ""])),
                               str(rng.choice(["", "0.0.0.0", "10.0.0.1"])))] if j % 3 else []
        img = str(rng.choice(["nginx:1.25", "redis", "busybox", "registry:5000/app", "missing:1"]))
        tols = [Toleration("dedicated", str(rng.choice(["", "Equal", "Exists"])), "gpu",
                           str(rng.choice(["", "NoSchedule", "PreferNoSchedule"])))] if j % 2 else []
        p = Pod(f"p{j}", containers=[Container({"cpu": "100m"}, ports, img), Container({}, [], "redis")],
                tolerations=tols)
        if j < 50:
            p.node_name = f"n{j % 80}"
            bound.append(p)
        else:
            pods.append(p)
    both(nodes, bound, [pods])


def test_affinity_terms_and_namespaces():
    """Pod (anti-)affinity with namespaces lists, namespaceSelectors (empty =
    every namespace), nil / empty label selectors, and every selector operator."""
    rng = np.random.default_rng(9)
    nodes = [Node(f"n{i}", {"kubernetes.io/hostname": f"n{i}", "topology.kubernetes.io/zone": f"z{i % 3}",
                            "rack": f"r{i % 5}"}, [], {"cpu": "16", "memory": "64Gi", "pods": "110"})
             for i in range(60)]
    namespaces = {"default": {"team": "a"}, "prod": {"team": "b", "env": "prod"}, "dev": {"team": "a"}}
    sels = [LabelSelector({"app": "web"}), LabelSelector({}, [Requirement("app", "In", ["web", "db"])]),
            LabelSelector({}, [Requirement("tier", "NotIn", ["x"])]), LabelSelector({}, [Requirement("app", "Exists")]),
            LabelSelector({}, [Requirement("gone", "DoesNotExist")]), LabelSelector(), None]
    nss = [LabelSelector({"team": "a"}), LabelSelector(), None, LabelSelector({}, [Requirement("env", "Exists")])]

    keys = ["kubernetes.io/hostname", "topology.kubernetes.io/zone", "rack", "missing"]

    def term(k):
        return PodAffinityTerm(keys[k % 4], sels[k % len(sels)], [] if k % 3 else ["prod"],
                               nss[k % len(nss)] if k % 2 else None)

    def pod(j, bound=False):
        ns = str(rng.choice(["default", "prod"]))
        p = Pod(f"p{j}", ns, {"app": str(rng.choice(["web", "db", "cache"])), "tier": "t"},
                [Container({"cpu": "200m", "memory": "1Gi"})])
        k = int(rng.integers(0, 2))
        if bound:                    # few distinct carried terms: each matching one is a use of the queue's pods
            k = k % 2
            p.namespace = "default"
            if j % 3:
                return p
        if j % 4 == 0:
            p.pod_affinity_required = [term(k), term(k + 1)]
        if j % 4 == 1:
            p.pod_anti_affinity_required = [term(k)]
        if j % 3 == 0:
            p.pod_affinity_preferred = [WeightedPodAffinityTerm(int(rng.integers(0, 100)), term(k + 2))]
        if j % 5 == 0:
            p.pod_anti_affinity_preferred = [WeightedPodAffinityTerm(int(rng.integers(1, 100)), term(k + 3))]
        if j % 6 == 0:
            p.topology_spread = [TopologySpreadConstraint(int(rng.integers(1, 3)), "topology.kubernetes.io/zone",
                                                          "DoNotSchedule", sels[k % 6],
                                                          node_affinity_policy=["Honor", "Ignore", None][j % 3],
                                                          node_taints_policy=["Honor", None][j % 2])]
        return p

    bound = [pod(j, True) for j in range(120)]
    for j, p in enumerate(bound):
        p.node_name = f"n{j % 60}"
    queue = [pod(j) for j in range(120, 200)]
    queue[3].namespace = "dev"                 # namespaces noted while the queue compiles
    queue[7].namespace = "other"
    both(nodes, bound, [queue], cluster_kw={"namespaces": namespaces})


def test_node_affinity_expressions():
    """Every NodeSelectorRequirement operator, values outside the vocabulary,
    numeric Gt / Lt, matchFields, weight-0 preferred terms, nodeSelector on
    unknown keys and values."""
    nodes = [Node(f"n{i}", {"kubernetes.io/hostname": f"n{i}", "disk": ["ssd", "hdd", ""][i % 3],
                            "cores": str(4 * (i % 5)), "bad": ["x", "-3", "+7"][i % 3]},
                  [], {"cpu": "8", "memory": "32Gi", "pods": "110"}) for i in range(40)]
    R = Requirement
    terms = [NodeSelectorTerm([R("disk", "In", ["ssd", "nvme"])]), NodeSelectorTerm([R("disk", "NotIn", ["zzz"])]),
             NodeSelectorTerm([R("disk", "Exists")]), NodeSelectorTerm([R("nokey", "DoesNotExist")]),
             NodeSelectorTerm([R("cores", "Gt", ["7"]), R("bad", "Lt", ["0"])]),
             NodeSelectorTerm([R("cores", "Gt", ["x"])]), NodeSelectorTerm([R("disk", "In", [])]),
             NodeSelectorTerm([], [R("metadata.name", "In", ["n3"])]),
             NodeSelectorTerm([], [R("metadata.name", "NotIn", ["n4"])]),
             NodeSelectorTerm([], [R("metadata.name", "In", ["n1", "n2"])]), NodeSelectorTerm(),
             NodeSelectorTerm([R("disk", "Weird", ["a"])]), NodeSelectorTerm([R("disk", "In", [""])])]
    pods = []
    for j in range(80):
        p = Pod(f"p{j}", containers=[Container({"cpu": "1"})])
        if j % 2:
            p.required_terms = [terms[j % len(terms)], terms[(j * 7) % len(terms)]]
        if j % 9 == 0:
            p.required_terms = []
        p.preferred_terms = [PreferredTerm(j % 3, terms[(j * 5) % len(terms)])]
        if j % 4 == 0:
            p.node_selector = {"disk": ["ssd", "hdd", "", "none"][j % 4], "zzz": "1"}
        if j % 10 == 1:
            p.node_name = ["n5", "nope"][j % 2]
        pods.append(p)
    both(nodes, [], [pods])


def test_plugin_args():
    """NodeAffinityArgs.addedAffinity (required and preferred) and scalar
    resources the nodes do not offer (extra_scalar)."""
    nodes, pods = gen.config1_objects(n_nodes=60, n_pods=200)
    for i, n in enumerate(nodes):
        if i % 2:
            n.allocatable["example.com/gpu"] = str(i % 4)
        n.allocatable["hugepages-2Mi"] = "1Gi"
    for j, p in enumerate(pods):
        if j % 3 == 0:
            p.containers[0].requests["example.com/gpu"] = "1"
        if j % 5 == 0:
            p.init_containers = [Container({"cpu": "3", "example.com/fpga": "1"})]
            p.overhead = {"cpu": "50m", "memory": "10Mi"}
    sp = profile.SchedulerProfile()
    sp.node_affinity = profile.NodeAffinityArgs(
        [NodeSelectorTerm([Requirement("pool", "In", ["a", "b"])])],
        [PreferredTerm(7, NodeSelectorTerm([Requirement("disk", "In", ["ssd"])])),
         PreferredTerm(0, NodeSelectorTerm([Requirement("disk", "In", ["hdd"])]))])
    both(nodes, [], [pods], cluster_kw={"extra_scalar": ["example.com/fpga"]},
         pods_kw={"added_affinity": sp.node_affinity})
    sp.node_affinity = profile.NodeAffinityArgs([], [])
    both(nodes, [], [pods], cluster_kw={"extra_scalar": ["example.com/fpga"]},
         pods_kw={"added_affinity": sp.node_affinity})


@pytest.mark.parametrize("kind", ["system", "list"])
def test_spread_defaults(kind):
    from test_spread_defaults import WORKLOADS, mixed_nodes, workload_pods
    nodes = mixed_nodes(60, seed=4)
    bound = workload_pods(200, seed=12, bound_nodes=[n.name for n in nodes])
    args = profile.PodTopologySpreadArgs()
    if kind == "list":
        args = profile.PodTopologySpreadArgs("List", [
            TopologySpreadConstraint(2, "topology.kubernetes.io/zone", "DoNotSchedule"),
            TopologySpreadConstraint(4, "kubernetes.io/hostname", "ScheduleAnyway", node_taints_policy="Honor")])
    both(nodes, bound, [workload_pods(150, seed=13)], pods_kw={"spread": SpreadDefaults(args, *WORKLOADS)})


@pytest.mark.parametrize("scenario", ["bound", "binding"])
def test_volumes(scenario):
    if scenario == "bound":
        from test_volumes import volume_scenario
        nodes, pods, pvs, pvcs = volume_scenario()
        vol = VolumeIndex.from_nodes(nodes, pvs, pvcs)
    else:
        from test_volume_binding import binding_scenario
        nodes, pods, pvs, pvcs, classes = binding_scenario()
        vol = VolumeIndex.from_nodes(nodes, copy.deepcopy(pvs), copy.deepcopy(pvcs), classes, True)
        vol.run_pv_controller()
    pods = pods + [Pod("inline", containers=[Container({"cpu": "1"})], has_volumes=True)]
    _, _, out = both(nodes, [], [pods], pods_kw={"volumes": vol})
    assert (out[0][1].pods["vb_count"] > 0).any()


def _reference_docs():
    return sorted(glob.glob(os.path.join(HERE, "golden", "reference", "*_case*.json")))


@pytest.mark.parametrize("path", _reference_docs(), ids=os.path.basename)
def test_reference_documents(path):
    """The reference's own import / export samples
    (simulator/docs/api-samples/v1/{export,import}.md) through ingest."""
    snap = ingest.load(json.load(open(path)))
    sp = snap.profiles[0][1]
    kw = ingest._pod_args(sp, snap)
    kw["volumes"] = snap.volumes
    both(snap.nodes, snap.bound, [snap.pending],
         cluster_kw={"namespaces": snap.namespaces, "nb_args": sp.network_bandwidth}, pods_kw=kw)


def test_template_cluster():
    """A cluster of the simulator's UI templates (web/components/lib/templates)."""
    from test_ingest import _template_cluster
    doc = _template_cluster()
    snap = ingest.load(doc)
    both(snap.nodes, snap.bound, [snap.pending], cluster_kw={"namespaces": snap.namespaces},
         pods_kw=dict(ingest._pod_args(snap.profiles[0][1], snap), volumes=snap.volumes))


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(HERE, "golden", "go", "*.json.gz"))),
                         ids=os.path.basename)
def test_go_documents(path):
    """The Go-harness fixtures with their plugin args, workloads, volumes and
    scalar resources (tests/gofixture.py encode's inputs)."""
    import gofixture
    with gzip.open(path, "rb") as f:
        doc = json.loads(f.read())
    nodes, bound, pods = gofixture.objects(doc)
    sp = gofixture.scheduler_profile(doc)
    services, controllers = gofixture.workloads(doc)
    _, _, vol = gofixture.volumes(doc, nodes)
    scalar = sorted({k for p in pods for c in p.containers + p.init_containers for k in c.requests
                     if k not in ("cpu", "memory", "ephemeral-storage", "pods")})
    both(nodes, bound, [pods], cluster_kw={"namespaces": doc["namespaces"], "extra_scalar": scalar},
         pods_kw={"volumes": vol, "added_affinity": sp.node_affinity,
                  "spread": SpreadDefaults(sp.spread, services, controllers)})


def test_node_deltas_keep_classes():
    """A re-encoded snapshot keeps the scalar columns and class ids of the one
    it replaces (ksim/ingest.py NodeCache, ksim_encode_nodes keep_previous)."""
    nodes, bound, pending, (added, updated, removed) = gen.delta_objects(n_nodes=120, n_pods=300)
    pc, _ = encode_cluster(nodes, bound)
    enc = nativeenc.NativeEncoder()
    nc, _ = enc.encode_cluster(nodes, bound)
    same_pods(encode_pods(pc, pending[:150]), enc.encode_pods(nc, pending[:150]))
    cache = ingest.NodeCache(nodes, bound)
    for n in added:
        cache.add_node(n)
    for n in updated:
        cache.update_node(n)
    for name in removed:
        cache.remove_node(name)
    changed = cache.nodes
    pc2, _ = encode_cluster(changed, bound, scalar_order=pc.scalar_names, classes_from=pc.topo)
    nc2, _ = enc.encode_cluster(changed, bound, keep_previous=True)
    same_cluster(pc2, nc2)
    same_pods(encode_pods(pc2, pending[150:]), enc.encode_pods(nc2, pending[150:]))
    same_cluster(pc2, nc2)
    assert pc2.topo.keys[:len(pc.topo.keys)] == pc.topo.keys


@pytest.mark.parametrize("bad", ["taints", "selector", "spread", "quantity", "scalar", "uses"])
def test_errors_match(bad):
    """Inputs the Python compile refuses are refused natively as well."""
    nodes = [Node("n0", {"kubernetes.io/hostname": "n0"}, [], {"cpu": "4", "memory": "8Gi", "pods": "10"})]
    pod = Pod("p", containers=[Container({"cpu": "1"})])
    if bad == "taints":
        nodes[0].taints = [Taint(f"k{i}") for i in range(9)]
    elif bad == "selector":
        pod.pod_anti_affinity_required = [PodAffinityTerm("x", LabelSelector({}, [Requirement("a", "In", [])]))]
    elif bad == "spread":
        pod.topology_spread = [TopologySpreadConstraint(0, "kubernetes.io/hostname")]
    elif bad == "quantity":
        pod.containers[0].requests["memory"] = "12QQ"
    elif bad == "scalar":
        pod.containers[0].requests["example.com/gpu"] = "1"
    else:
        pod.pod_anti_affinity_preferred = [WeightedPodAffinityTerm(1, PodAffinityTerm("k", LabelSelector({"a": str(i)})))
                                           for i in range(17)]
    with pytest.raises(Exception):
        c, _ = encode_cluster(nodes)
        encode_pods(c, [pod])
    e = nativeenc.NativeEncoder()
    with pytest.raises(EncodeError):
        c, _ = e.encode_cluster(nodes)
        e.encode_pods(c, [pod])


def test_quantities():
    """resource.Quantity forms (ksim/model.py quantity_value / milli_value):
    suffixes, exponents, fractions rounded up, signs."""
    qs = ["1", "0", "100m", "1.5", "0.1", "1.0001", "2Ki", "1.5Gi", "3Mi", "1k", "1M", "1G", "1T", "1P",
          "1e3", "1E3", "1.5e-3", "12e+2", ".5", "5.", "-1", "-1.5", "+3", "250u", "7n", " 8 ", "0.000000001"]
    nodes = [Node(f"n{i}", {}, [], {"cpu": q, "memory": q, "ephemeral-storage": q, "pods": "5"})
             for i, q in enumerate(qs)]
    both(nodes, [], [[Pod("p", containers=[Container({"cpu": q, "memory": q})]) for q in qs]])


def test_pool_struct_layout():
    """The pool structs have the header's sizes (ksim_abi_sizeof)."""
    from ksim import engine
    for which, s in enumerate(abi.STRUCT_ORDER):
        assert engine.lib().ksim_abi_sizeof(which) == abi.struct_size(s), which
