"""Deterministic synthetic clusters for BASELINE.json's configs.

SplitMix64 streams with the seeds 0x4B53494D0001..0005.  Config 1 is built as
Node/Pod objects (it exercises the encoder); configs 2/4/5 are emitted straight
into the engine's SoA buffers (vectorised, 100k nodes / 1M pods in seconds).
Node/pod shapes start from the UI templates web/components/lib/templates/
{node,pod}.yaml (cpu 4 / 32Gi / 110 pods; pod 100m / 16Gi).
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np

from . import abi
from .encode import EncodedCluster, EncodedPods, encode_cluster, encode_pods
from .model import (Container, Node, NodeSelectorTerm, Pod, PreferredTerm, Requirement, Taint,
                    Toleration)

M64 = (1 << 64) - 1
GOLDEN = 0x9E3779B97F4A7C15
SEEDS = {1: 0x4B53494D0001, 2: 0x4B53494D0002, 3: 0x4B53494D0003, 4: 0x4B53494D0004,
         5: 0x4B53494D0005}
GI = 1 << 30
MI = 1 << 20


def mix64(z: int) -> int:
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


class Rng:
    """SplitMix64 stream."""

    def __init__(self, seed: int):
        self.s = seed & M64

    def next(self) -> int:
        self.s = (self.s + GOLDEN) & M64
        return mix64(self.s)

    def below(self, n: int) -> int:
        return (self.next() >> 11) % n

    def chance(self, pct: int) -> bool:
        return self.below(100) < pct


def _mix_np(z: np.ndarray) -> np.ndarray:
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def stream(seed: int, tag: int, n: int) -> np.ndarray:
    """n values of the SplitMix64 stream seeded with mix64(seed ^ tag)."""
    s = np.uint64(mix64((seed ^ tag) & M64))
    with np.errstate(over="ignore"):
        idx = np.arange(1, n + 1, dtype=np.uint64)
        return _mix_np(s + idx * np.uint64(GOLDEN))


def below(x: np.ndarray, n: int) -> np.ndarray:
    return ((x >> np.uint64(11)) % np.uint64(n)).astype(np.int64)


# ---- config 1: 100 nodes x 1,000 pods, resources + taints + node affinity ----
POOLS = ["a", "b", "c", "d"]
DISKS = ["ssd", "hdd"]
NOSCHED = [Taint("dedicated", "gpu", "NoSchedule"), Taint("dedicated", "infra", "NoSchedule")]
PREFER = [Taint("spot", "true", "PreferNoSchedule"), Taint("old", "true", "PreferNoSchedule")]


def config1_objects(n_nodes: int = 100, n_pods: int = 1000,
                    seed: int = SEEDS[1]) -> Tuple[List[Node], List[Pod]]:
    r = Rng(seed)
    nodes = []
    for i in range(n_nodes):
        cores = [4, 8, 16, 32][r.below(4)]
        mem = [16, 32, 64, 128][r.below(4)]
        taints = []
        if r.chance(10):
            taints.append(NOSCHED[r.below(2)])
        if r.chance(20):
            taints.append(PREFER[r.below(2)])
        nodes.append(Node(
            name=f"node-{i:05d}",
            labels={"kubernetes.io/hostname": f"node-{i:05d}",
                    "topology.kubernetes.io/zone": f"z{i % 3}",
                    "pool": POOLS[r.below(4)], "disk": DISKS[r.below(2)]},
            taints=taints,
            allocatable={"cpu": str(cores), "memory": f"{mem}Gi", "pods": "110"}))
    pods = []
    all_taints = NOSCHED + PREFER
    for j in range(n_pods):
        cpu = 100 * (1 + r.below(20))
        mem = 128 * (1 << r.below(7))
        p = Pod(name=f"pod-{j:06d}", containers=[Container({"cpu": f"{cpu}m", "memory": f"{mem}Mi"})])
        if r.chance(30):
            t = all_taints[r.below(4)]
            p.tolerations = [Toleration(t.key, "Equal", t.value, t.effect)]
        if r.chance(30):
            k = 1 + r.below(2)
            vals = sorted({POOLS[r.below(4)] for _ in range(k)})
            p.required_terms = [NodeSelectorTerm([Requirement("pool", "In", vals)])]
        if r.chance(30):
            terms = []
            for _ in range(1 + r.below(2)):
                w = 1 + r.below(100)
                if r.chance(50):
                    req = Requirement("pool", "In", [POOLS[r.below(4)]])
                else:
                    req = Requirement("disk", "In", ["ssd"])
                terms.append(PreferredTerm(w, NodeSelectorTerm([req])))
            p.preferred_terms = terms
        pods.append(p)
    return nodes, pods


def config1(n_nodes: int = 100, n_pods: int = 1000, seed: int = SEEDS[1]):
    nodes, pods = config1_objects(n_nodes, n_pods, seed)
    cluster, _ = encode_cluster(nodes)
    return cluster, encode_pods(cluster, pods)


# ---- configs 2/4/5: bare pods, NodeResourcesFit + BalancedAllocation dominated --
def bare_cluster(n_nodes: int, seed: int) -> EncodedCluster:
    """Nodes cpu in {8,16,32,64} cores, memory in {32,64,128,256} Gi, 110 pods,
    3 zones (node i in z{i%3}: nodeTree order is the identity)."""
    N = n_nodes
    cores = np.array([8, 16, 32, 64], np.int64)[below(stream(seed, 1, N), 4)]
    mem = np.array([32, 64, 128, 256], np.int64)[below(stream(seed, 2, N), 4)] * GI
    hostnames = [f"node-{i:06d}" for i in range(N)]
    labels = np.zeros((2, N), np.uint32)
    labels[0] = np.arange(1, N + 1, dtype=np.uint32)          # kubernetes.io/hostname
    labels[1] = (np.arange(N) % 3 + 1).astype(np.uint32)       # topology.kubernetes.io/zone
    z = np.zeros(N, np.int64)
    return EncodedCluster(
        n_nodes=N, n_scalar=0,
        alloc_cpu=cores * 1000, alloc_mem=mem, alloc_eph=z.copy(),
        alloc_pods=np.full(N, 110, np.int32), alloc_scalar=np.zeros((0, N), np.int64),
        req_cpu=z.copy(), req_mem=z.copy(), req_eph=z.copy(), req_scalar=np.zeros((0, N), np.int64),
        nz_cpu=z.copy(), nz_mem=z.copy(), num_pods=np.zeros(N, np.int32),
        flags=np.zeros(N, np.uint32), taints=np.zeros((abi.MAX_NODE_TAINTS, N), np.uint16),
        labels=labels, taint_effect=np.zeros(1, np.uint8),
        label_col_offset=np.array([0, N + 1], np.int32),
        label_num=np.zeros(N + 1 + 4, np.int64), label_num_ok=np.zeros(N + 1 + 4, np.uint8),
        node_names=hostnames,
        label_keys=["kubernetes.io/hostname", "topology.kubernetes.io/zone"],
        label_values=[[""] + hostnames, ["", "z0", "z1", "z2"]],
        taint_vocab=[None], scalar_names=[])


def bare_pods(n_pods: int, seed: int, cpu_steps: int = 10, mem_steps: int = 16) -> EncodedPods:
    """Pods with one container: cpu 100m..1000m (step 100m), memory
    256Mi..4Gi (step 256Mi); requests set, so non-zero == requests."""
    P = n_pods
    cpu = 100 * (1 + below(stream(seed, 11, P), cpu_steps))
    mem = 256 * MI * (1 + below(stream(seed, 12, P), mem_steps))
    pods = np.zeros(P, abi.POD_DTYPE)
    pods["req_cpu"] = cpu
    pods["req_mem"] = mem
    pods["nz_cpu"] = cpu
    pods["nz_mem"] = mem
    pods["node_name"] = -1
    return EncodedPods(pods, np.zeros(0, abi.LABEL_EXPR_DTYPE), np.zeros(0, abi.TERM_DTYPE),
                       [("default", f"pod-{j:07d}") for j in range(P)] if P <= 200000 else [])


def config2(n_nodes: int = 5000, n_pods: int = 50000, seed: int = SEEDS[2]):
    return bare_cluster(n_nodes, seed), bare_pods(n_pods, seed)


def config4(n_nodes: int = 100000, n_pods: int = 1000000, seed: int = SEEDS[4]):
    return bare_cluster(n_nodes, seed), bare_pods(n_pods, seed)


def config5_weights(n: int = 1024, seed: int = SEEDS[5]) -> np.ndarray:
    """1,024 score-weight vectors w in {1..10}^7 (profile Score order)."""
    x = stream(seed, 21, n * 7)
    return (1 + below(x, 10)).reshape(n, 7).astype(np.int32)


# ---- config 3: PodTopologySpread + InterPodAffinity heavy ---------------------
N_APPS = 64


def config3_objects(n_nodes: int = 10000, pods_per_node: int = 10, n_incoming: int = 10000,
                    seed: int = SEEDS[3], zone_anti_every: int = 1000):
    """nodes in 3 zones (round-robin), ``pods_per_node``
    existing pods per node, each with app=a<k> (64 values) carrying a required
    anti-affinity term against a random app (topologyKey hostname; every
    ``zone_anti_every``-th one instead zone-wide against app + tier=critical)
    and a preferred affinity term (zone, weight 1..100) to a random app.
    Incoming pods (app=a<x>, 5 % tier=critical) spread with maxSkew 1 over
    zones (DoNotSchedule) and maxSkew 2 over hostnames (ScheduleAnyway) on
    their own app, and prefer (weight 50) not to share a host with it."""
    from .model import (LabelSelector, PodAffinityTerm, TopologySpreadConstraint, WeightedPodAffinityTerm)
    r = Rng(seed)
    nodes = []
    for i in range(n_nodes):
        cores = [16, 32, 64][r.below(3)]
        mem = [64, 128, 256][r.below(3)]
        nodes.append(Node(
            name=f"node-{i:06d}",
            labels={"kubernetes.io/hostname": f"node-{i:06d}", "topology.kubernetes.io/zone": f"z{i % 3}"},
            allocatable={"cpu": str(cores), "memory": f"{mem}Gi", "pods": "110"}))
    # pods of one workload share their spec's objects (selectors, terms,
    # containers), as the pods of a ReplicaSet do: built once per distinct value
    shared: dict = {}

    def one(key, make):
        x = shared.get(key)
        if x is None:
            x = shared[key] = make()
        return x

    bound = []
    j = 0
    for i in range(n_nodes):
        for _ in range(pods_per_node):
            app = f"a{r.below(N_APPS)}"
            cpu = 100 * (1 + r.below(5))
            mem = 256 * (1 + r.below(8))
            p = Pod(name=f"existing-{j:07d}", labels={"app": app, "tier": "web"},
                    containers=[one(("c", cpu, mem), lambda: Container({"cpu": f"{cpu}m", "memory": f"{mem}Mi"}))],
                    node_name=nodes[i].name)
            target = f"a{r.below(N_APPS)}"
            if zone_anti_every and j % zone_anti_every == zone_anti_every - 1:
                p.pod_anti_affinity_required = [one(("za", target), lambda: PodAffinityTerm(
                    "topology.kubernetes.io/zone", LabelSelector({"app": target, "tier": "critical"})))]
            else:
                p.pod_anti_affinity_required = [one(("ha", target), lambda: PodAffinityTerm(
                    "kubernetes.io/hostname", LabelSelector({"app": target})))]
            w, pref = 1 + r.below(100), f"a{r.below(N_APPS)}"
            p.pod_affinity_preferred = [one(("pa", w, pref), lambda: WeightedPodAffinityTerm(w, PodAffinityTerm(
                "topology.kubernetes.io/zone", LabelSelector({"app": pref}))))]
            bound.append(p)
            j += 1
    incoming = []
    for k in range(n_incoming):
        app = f"a{r.below(N_APPS)}"
        tier = "critical" if r.chance(5) else "web"
        cpu = 100 * (1 + r.below(10))
        mem = 256 * (1 + r.below(16))
        sel = LabelSelector({"app": app})
        p = Pod(name=f"pod-{k:07d}", labels={"app": app, "tier": tier},
                containers=[Container({"cpu": f"{cpu}m", "memory": f"{mem}Mi"})],
                topology_spread=[
                    TopologySpreadConstraint(1, "topology.kubernetes.io/zone", "DoNotSchedule", sel),
                    TopologySpreadConstraint(2, "kubernetes.io/hostname", "ScheduleAnyway", sel)],
                pod_anti_affinity_preferred=[WeightedPodAffinityTerm(50, PodAffinityTerm(
                    "kubernetes.io/hostname", LabelSelector({"app": app})))])
        incoming.append(p)
    return nodes, bound, incoming


def config3(n_nodes: int = 10000, pods_per_node: int = 10, n_incoming: int = 10000, seed: int = SEEDS[3],
            zone_anti_every: int = 1000):
    nodes, bound, incoming = config3_objects(n_nodes, pods_per_node, n_incoming, seed, zone_anti_every)
    cluster, _ = encode_cluster(nodes, bound)
    return cluster, encode_pods(cluster, incoming)


# ---- NetworkBandwidth scenarios (the simulator's out-of-tree plugin) ----------
NB_LIMITS = ["1G", "2G", "5G", "10G", "1Gi", "2500M", "750M", "1500000k"]
NB_REQS = ["50M", "100M", "250M", "400M", "1G", "120Mi", "0.5G", "1500m", "1e8"]


def netbw_objects(n_nodes: int = 120, n_pods: int = 300, seed: int = SEEDS[1] ^ 0x4E42,
                  node_errors: bool = False, pod_errors: bool = False,
                  n_bound: int = 60) -> Tuple[List[Node], List[Pod], List[Pod]]:
    """config1-shaped nodes with network-limit annotations, bound pods holding
    request annotations (the nodes' allocated amounts), and pending pods whose
    requests come from the request annotations or the *-bandwidth fallbacks.
    ``node_errors``: some nodes lack the limit or carry an unparsable one;
    ``pod_errors``: some pods request nothing or carry an unparsable request."""
    from .netbw import EGRESS_BANDWIDTH, INGRESS_BANDWIDTH, NetworkBandwidthArgs
    a = NetworkBandwidthArgs()
    nodes, pods = config1_objects(n_nodes, n_pods + n_bound, seed)
    r = Rng(seed ^ 0xB0)
    for n in nodes:
        if node_errors and r.chance(4):
            continue                                         # no limit annotation
        if node_errors and r.chance(3):
            n.annotations[a.node_limit_annotation] = "ten-gigabit"
        else:
            n.annotations[a.node_limit_annotation] = NB_LIMITS[r.below(len(NB_LIMITS))]
    bound, pending = pods[:n_bound], pods[n_bound:]
    for p in bound:
        p.node_name = nodes[r.below(n_nodes)].name
        p.tolerations, p.required_terms, p.preferred_terms = [], None, []
        if r.chance(70):
            p.annotations[a.ingress_request_annotation] = NB_REQS[r.below(len(NB_REQS))]
        if r.chance(50):
            p.annotations[a.egress_request_annotation] = NB_REQS[r.below(len(NB_REQS))]
        if r.chance(10):
            p.annotations[a.egress_request_annotation] = "lots"      # skipped by getNodeAllocatedAmount
        if r.chance(20):
            p.annotations[INGRESS_BANDWIDTH] = NB_REQS[r.below(len(NB_REQS))]   # not counted as allocated
    for p in pending:
        k = r.below(4)
        if k == 0:
            p.annotations[a.ingress_request_annotation] = NB_REQS[r.below(len(NB_REQS))]
        elif k == 1:
            p.annotations[INGRESS_BANDWIDTH] = NB_REQS[r.below(len(NB_REQS))]
        elif k == 2:
            p.annotations[a.egress_request_annotation] = NB_REQS[r.below(len(NB_REQS))]
            p.annotations[INGRESS_BANDWIDTH] = NB_REQS[r.below(len(NB_REQS))]
        else:
            p.annotations[EGRESS_BANDWIDTH] = NB_REQS[r.below(len(NB_REQS))]
        if pod_errors and r.chance(3):
            p.annotations = {}                                 # requests nothing: Skip -> Error
        elif pod_errors and r.chance(3):
            p.annotations[a.egress_request_annotation] = "fast"
    return nodes, bound, pending


def prefilter_objects(n_nodes: int = 300, n_pods: int = 600, seed: int = SEEDS[1] ^ 0x50464E) \
        -> Tuple[List[Node], List[Pod]]:
    """config1-shaped nodes and pods, a third of them with required node
    affinity on metadata.name matchFields, so NodeAffinity's PreFilterResult
    restricts their scan: one name; two names as two
    ORed terms; a long list of single-name terms (more than
    numFeasibleNodesToFind's window under ADAPT); a term that also carries
    label expressions; intersecting fields; conflicting fields (no node);
    an unknown node name (the cycle errors); a two-value requirement (the
    PreFilter set holds it, the Filter's field selector cannot parse it); a
    NotIn field (no restriction)."""
    nodes, pods = config1_objects(n_nodes, n_pods, seed)
    r = Rng(seed ^ 0x77)
    names = [n.name for n in nodes]

    def field(op, *vals):
        return Requirement("metadata.name", op, list(vals))

    for j, p in enumerate(pods):
        if j % 3:
            continue
        k = r.below(10)
        a, b = names[r.below(n_nodes)], names[r.below(n_nodes)]
        if k == 0:
            p.required_terms = [NodeSelectorTerm(match_fields=[field("In", a)])]
        elif k == 1:
            p.required_terms = [NodeSelectorTerm(match_fields=[field("In", a)]),
                                NodeSelectorTerm(match_fields=[field("In", b)])]
        elif k == 2:
            many = sorted({names[r.below(n_nodes)] for _ in range(min(n_nodes, 180))})
            p.required_terms = [NodeSelectorTerm(match_fields=[field("In", x)]) for x in many]
        elif k == 3:
            p.required_terms = [NodeSelectorTerm([Requirement("pool", "In", [POOLS[r.below(4)]])],
                                                 [field("In", a)]),
                                NodeSelectorTerm(match_fields=[field("In", b)])]
        elif k == 4:
            p.required_terms = [NodeSelectorTerm(match_fields=[field("In", a), field("In", a)])]
        elif k == 5:
            c = names[(names.index(a) + 1) % n_nodes]
            p.required_terms = [NodeSelectorTerm(match_fields=[field("In", a), field("In", c)])]
        elif k == 6:
            p.required_terms = [NodeSelectorTerm(match_fields=[field("In", "node-missing")]),
                                NodeSelectorTerm(match_fields=[field("In", a)])]
        elif k == 7:
            p.required_terms = [NodeSelectorTerm(match_fields=[field("In", a, b)])]
        elif k == 8:
            p.required_terms = [NodeSelectorTerm(match_fields=[field("NotIn", a)])]
        else:
            p.required_terms = [NodeSelectorTerm(match_fields=[field("In", a)]),
                                NodeSelectorTerm([Requirement("disk", "In", ["ssd"])])]
    return nodes, pods


def edge_objects(n_pods: int = 160, seed: int = SEEDS[1] ^ 0xED6E) -> Tuple[List[Node], List[Pod], List[Pod]]:
    """Resource edge cases the plugin arithmetic must get right (SURVEY
    Appendix A): allocatable 0, requested above allocatable (bound pods
    overcommit a node), allowed pods 0, quantities at and past 2^52 (the exact
    division path) and past 2^56 (leastRequestedScore's int64 product wraps
    in Go), BestEffort pods (non-zero defaults), init containers.  Returns
    (nodes, bound pods, pending pods)."""
    r = Rng(seed)

    def node(i, cpu, mem, pods="110"):
        return Node(f"edge-{i:02d}", {"kubernetes.io/hostname": f"edge-{i:02d}",
                                      "topology.kubernetes.io/zone": f"z{i % 2}"},
                    [], {"cpu": cpu, "memory": mem, "pods": pods})

    nodes = [node(0, "0", "0"), node(1, "4", "8Gi"), node(2, "4", "4Pi"), node(3, "100000000000", "1Ei"),
             node(4, "5000000000000", "3Ei"), node(5, "8", "16Gi", pods="0"), node(6, "16", "64Gi"),
             node(7, "32", "128Gi"), node(8, "8", "32Gi"), node(9, "64", "4Pi"), node(10, "2", "1Gi"),
             node(11, "4503599627370", "8191Pi")]
    bound = [Pod(f"over-{k}", node_name="edge-01", containers=[Container({"cpu": "3", "memory": "6Gi"})])
             for k in range(2)]
    bound.append(Pod("big", node_name="edge-03", containers=[Container({"cpu": "1000", "memory": "300Pi"})]))
    mems = ["0", "64Mi", "1Gi", "6Gi", "2Pi", "700Pi", "1Ei"]
    cpus = ["0", "100m", "1", "3", "2000", "4000000000000"]
    pending = []
    for j in range(n_pods):
        k = r.below(6)
        if k == 0:
            c = Container({})                                         # BestEffort: 100m / 200Mi non-zero
        else:
            c = Container({"cpu": cpus[r.below(len(cpus))], "memory": mems[r.below(len(mems))]})
        p = Pod(f"edge-pod-{j:04d}", containers=[c])
        if r.chance(15):
            p.init_containers = [Container({"cpu": cpus[r.below(len(cpus))], "memory": mems[r.below(len(mems))]})]
        pending.append(p)
    return nodes, bound, pending


def delta_objects(n_nodes: int = 240, n_pods: int = 720, n_keys: int = 60, seed: int = SEEDS[1] ^ 0xDE17A):
    """A cluster for node informer deltas (ksim.ingest.NodeCache): nodes carry
    ``n_keys`` label keys (example.com/k00.., three values, each present on 80 %
    of the nodes) plus hostname / zone (4 zones) and hugepages-2Mi / -1Gi
    allocatable; bound pods; pending pods with node selectors, required and
    preferred terms over those keys, hugepages requests, a zone spread and a
    hostname anti-affinity on their app.  Returns (nodes, bound, pending,
    deltas) with deltas = (added nodes, updated nodes, removed names): added
    nodes carry a new label key and a new scalar resource, updates change
    label values and (for some) the zone, removals hit nodes holding pods."""
    from .model import LabelSelector, PodAffinityTerm, TopologySpreadConstraint
    r = Rng(seed)
    keys = [f"example.com/k{j:02d}" for j in range(n_keys)]

    def node(name, zone):
        labels = {"kubernetes.io/hostname": name, "topology.kubernetes.io/zone": f"z{zone}"}
        for k in keys:
            if r.chance(80):
                labels[k] = f"v{r.below(3)}"
        alloc = {"cpu": str([8, 16, 32][r.below(3)]), "memory": f"{[32, 64, 128][r.below(3)]}Gi", "pods": "110"}
        if r.chance(50):
            alloc["hugepages-2Mi"] = f"{1 + r.below(4)}Gi"
        if r.chance(25):
            alloc["hugepages-1Gi"] = f"{2 + r.below(3)}Gi"
        return Node(name, labels, [], alloc)

    nodes = [node(f"dn-{i:05d}", i % 4) for i in range(n_nodes)]

    def pod(name):
        app = f"app{r.below(12)}"
        req = {"cpu": f"{100 * (1 + r.below(20))}m", "memory": f"{256 * (1 + r.below(16))}Mi"}
        if r.chance(30):
            req["hugepages-2Mi"] = f"{256 * (1 + r.below(4))}Mi"
        if r.chance(10):
            req["hugepages-1Gi"] = "1Gi"
        p = Pod(name, labels={"app": app}, containers=[Container(req)])
        if r.chance(40):
            p.node_selector = {keys[r.below(n_keys)]: f"v{r.below(3)}" for _ in range(1 + r.below(2))}
        if r.chance(20):
            k = keys[r.below(n_keys)]
            op = ["In", "NotIn", "Exists", "DoesNotExist"][r.below(4)]
            vals = [f"v{r.below(3)}"] if op in ("In", "NotIn") else []
            p.required_terms = [NodeSelectorTerm([Requirement(k, op, vals)])]
        if r.chance(25):
            p.preferred_terms = [PreferredTerm(1 + r.below(100), NodeSelectorTerm(
                [Requirement(keys[r.below(n_keys)], "In", [f"v{r.below(3)}"])]))]
        if r.chance(25):
            p.topology_spread = [TopologySpreadConstraint(2, "topology.kubernetes.io/zone", "DoNotSchedule",
                                                          LabelSelector({"app": app}))]
        if r.chance(15):
            p.pod_anti_affinity_required = [PodAffinityTerm("kubernetes.io/hostname", LabelSelector({"app": app}))]
        return p

    bound = []
    for j in range(n_nodes // 2):
        p = pod(f"bound-{j:05d}")
        p.node_selector, p.required_terms, p.topology_spread = {}, None, []
        p.node_name = nodes[r.below(n_nodes)].name
        bound.append(p)
    pending = [pod(f"dpod-{j:05d}") for j in range(n_pods)]

    added = []
    for i in range(n_nodes // 10):
        n = node(f"dn-new-{i:04d}", r.below(5))                       # a fifth zone appears
        n.labels["example.com/new"] = f"v{r.below(2)}"
        if r.chance(50):
            n.allocatable["example.com/fpga"] = "2"
        added.append(n)
    updated = []
    for i in r_sample(r, n_nodes, n_nodes // 20):
        old = nodes[i]
        labels = dict(old.labels)
        for k in keys[:8]:
            labels[k] = f"v{r.below(3)}"
        if i % 3 == 0:
            labels["topology.kubernetes.io/zone"] = f"z{(int(labels['topology.kubernetes.io/zone'][1:]) + 1) % 4}"
        updated.append(Node(old.name, labels, list(old.taints), dict(old.allocatable)))
    held = sorted({p.node_name for p in bound})
    removed = [held[r.below(len(held))] for _ in range(n_nodes // 40)]
    removed += [nodes[r.below(n_nodes)].name for _ in range(n_nodes // 40)]
    removed = sorted(set(removed) - {n.name for n in updated})
    return nodes, bound, pending, (added, updated, removed)


def r_sample(r: Rng, n: int, k: int) -> List[int]:
    """k distinct indices below n from the stream r."""
    out: List[int] = []
    while len(out) < min(k, n):
        x = r.below(n)
        if x not in out:
            out.append(x)
    return out
