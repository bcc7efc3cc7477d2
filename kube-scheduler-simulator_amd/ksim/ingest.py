"""Snapshot ingest: the simulator's import/export document -> engine inputs
(SURVEY §8(f) 2).

The reference moves whole cluster states as ``ResourcesForImport`` /
``ResourcesForExport`` JSON (simulator/export/export.go:43-65): pods, nodes,
pvs, pvcs, storageClasses, priorityClasses, schedulerConfig, namespaces.  This
module turns one such document into what the engine runs:

* nodes in nodeTree order (ksim.encode), bound pods (``spec.nodeName`` set)
  added to their node's aggregates and count classes like NodeInfo.AddPod;
* the pending pods in scheduling-queue order: PrioritySort (higher
  ``.spec.priority`` first, the priority resolved from ``priorityClassName`` /
  the globalDefault class as the Priority admission plugin does), ties by
  creationTimestamp then document order;
* the scheduler profiles of ``schedulerConfig`` converted the way the simulator
  does it (scheduler.go:199-249 convertConfigurationForSimulator): plugins merged
  over the in-tree defaults (plugins.go:185-288), plugin args over the defaults
  (plugins.go:103-179), every non-profile field reset to the default, so
  percentageOfNodesToScore is 0 (ADAPT) whatever the document says.

PVs, PVCs and StorageClasses feed VolumeBinding, VolumeZone and
VolumeRestrictions (ksim.volumes): the PV controller's binding of Immediate
claims at load, bound claims by PV node affinity / topology labels, unbound
WaitForFirstConsumer claims by static matching or dynamic provisioning, and
ReadWriteOncePod claims in use; ``schedule_queue`` runs a queue whose pods take
PVs as they bind.  Pods with volumes the engine does not model (inline disks,
CSI inline, ephemeral, PVs counted against node volume limits) are reported in
``unsupported`` and left out of the queue.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import profile as prof_mod
from .model import (Controller, Node, Pod, Service, controller_from_dict, node_from_dict, pod_from_dict, pv_from_dict,
                    pvc_from_dict, service_from_dict, storage_class_from_dict)
from .volumes import VolumeIndex, VolumeUnsupported
from .netbw import NetworkBandwidthArgs


@dataclass
class Snapshot:
    nodes: List[Node]
    bound: List[Pod]
    pending: List[Pod]                       # scheduling-queue order
    namespaces: Dict[str, Dict[str, str]]
    profiles: List[Tuple[str, prof_mod.SchedulerProfile]]   # (schedulerName, profile)
    unsupported: List[Tuple[str, str, str]] = field(default_factory=list)   # (namespace, name, why)
    volumes: Optional[VolumeIndex] = None    # the document's PVs / PVCs (VolumeBinding, VolumeZone)
    counts: Dict[str, int] = field(default_factory=dict)
    # Services and controllers that select pods (PodTopologySpread default
    # constraints, helper.DefaultSelector).  Not part of the reference's
    # export document: a host fills them from its listers (optional keys
    # "services", "replicationControllers", "replicaSets", "statefulSets").
    services: List[Service] = field(default_factory=list)
    controllers: List[Controller] = field(default_factory=list)


# ---- priority (admission: priority from PriorityClass) -------------------------------
def _priority(spec: dict, classes: Dict[str, int], default: int) -> int:
    if spec.get("priority") is not None:
        return int(spec["priority"])
    name = spec.get("priorityClassName") or ""
    if name:
        if name not in classes:
            raise ValueError(f"priorityClassName {name!r} not found")
        return classes[name]
    return default


def _priority_classes(items: List[dict]) -> Tuple[Dict[str, int], int]:
    classes, default = {}, 0
    # the built-in classes the apiserver always has (scheduling/v1 SystemPriorityClasses)
    classes["system-node-critical"] = 2000001000
    classes["system-cluster-critical"] = 2000000000
    for pc in items or []:
        name = (pc.get("metadata") or {}).get("name", "")
        classes[name] = int(pc.get("value") or 0)
        if pc.get("globalDefault"):
            default = int(pc.get("value") or 0)
    return classes, default


# ---- scheduler configuration ---------------------------------------------------------
def _plugin_set(d: Optional[dict]) -> prof_mod.PluginSet:
    d = d or {}
    return prof_mod.PluginSet([prof_mod.Plugin(p["name"], int(p.get("weight") or 0)) for p in d.get("enabled") or []],
                              [prof_mod.Plugin(p["name"]) for p in d.get("disabled") or []])


_EXT_JSON = {"queueSort": "queueSort", "preFilter": "preFilter", "filter": "filter", "postFilter": "postFilter",
             "preScore": "preScore", "score": "score", "reserve": "reserve", "permit": "permit",
             "preBind": "preBind", "bind": "bind", "postBind": "postBind"}


class UnsupportedArgs(ValueError):
    """A pluginConfig argument the engine does not implement (refused, never dropped)."""


def _check_keys(plugin: str, args: dict, known: Sequence[str]) -> None:
    for k in args:
        if k not in known and k not in ("kind", "apiVersion"):
            raise UnsupportedArgs(f"{plugin} args: {k!r} not supported by the engine")


def _fit_args(args: dict, cur: prof_mod.FitArgs) -> prof_mod.FitArgs:
    """NodeResourcesFitArgs decoded over the current (default) object: a field
    the document sets replaces it, a nested object is merged field by field
    (json.Unmarshal into the typed default, plugins.go:131-136)."""
    _check_keys("NodeResourcesFit", args, ("ignoredResources", "ignoredResourceGroups", "scoringStrategy"))
    fit = prof_mod.FitArgs(cur.strategy, list(cur.resources), None if cur.shape is None else list(cur.shape),
                           list(cur.ignored_resources), list(cur.ignored_resource_groups))
    if "ignoredResources" in args:
        fit.ignored_resources = [str(x) for x in args["ignoredResources"] or []]
    if "ignoredResourceGroups" in args:
        fit.ignored_resource_groups = [str(x) for x in args["ignoredResourceGroups"] or []]
    if "scoringStrategy" in args:
        ss = args["scoringStrategy"]
        if ss is None:                                  # nil: SetDefaults_NodeResourcesFitArgs
            return prof_mod.FitArgs(ignored_resources=fit.ignored_resources,
                                    ignored_resource_groups=fit.ignored_resource_groups)
        _check_keys("NodeResourcesFit scoringStrategy", ss, ("type", "resources", "requestedToCapacityRatio"))
        if ss.get("type"):
            fit.strategy = str(ss["type"])
        if "resources" in ss:
            fit.resources = [(r["name"], int(r.get("weight") or 1)) for r in ss["resources"] or []]
            if not fit.resources:                       # empty: the default set (SetDefaults)
                fit.resources = [("cpu", 1), ("memory", 1)]
        if ss.get("requestedToCapacityRatio") is not None:
            rt = ss["requestedToCapacityRatio"]
            _check_keys("requestedToCapacityRatio", rt, ("shape",))
            fit.shape = [(int(x.get("utilization") or 0), int(x.get("score") or 0)) for x in rt.get("shape") or []]
    return fit


def _node_affinity_args(args: dict) -> prof_mod.NodeAffinityArgs:
    from .model import _term, PreferredTerm
    _check_keys("NodeAffinity", args, ("addedAffinity",))
    aa = args.get("addedAffinity") or {}
    _check_keys("NodeAffinity addedAffinity", aa, ("requiredDuringSchedulingIgnoredDuringExecution",
                                                   "preferredDuringSchedulingIgnoredDuringExecution"))
    out = prof_mod.NodeAffinityArgs()
    req = aa.get("requiredDuringSchedulingIgnoredDuringExecution")
    if req is not None:
        terms = [_term(t) for t in req.get("nodeSelectorTerms") or []]
        if not terms:                                   # ValidateNodeAffinityArgs -> ValidateNodeSelector
            raise ValueError("NodeAffinityArgs.addedAffinity: must have at least one node selector term")
        out.required = terms
    for pt in aa.get("preferredDuringSchedulingIgnoredDuringExecution") or []:
        w = int(pt.get("weight") or 0)
        if not 1 <= w <= 100:                           # ValidatePreferredSchedulingTerms
            raise ValueError("NodeAffinityArgs.addedAffinity: preferred term weight must be in the range 1-100")
        out.preferred.append(PreferredTerm(w, _term(pt.get("preference") or {})))
    return out


def _spread_args(args: dict, cur: prof_mod.PodTopologySpreadArgs) -> prof_mod.PodTopologySpreadArgs:
    from .model import _spread
    _check_keys("PodTopologySpread", args, ("defaultConstraints", "defaultingType"))
    out = prof_mod.PodTopologySpreadArgs(cur.defaulting_type, list(cur.default_constraints))
    if args.get("defaultingType"):
        out.defaulting_type = str(args["defaultingType"])
    if "defaultConstraints" in args:
        out.default_constraints = []
        for d in args["defaultConstraints"] or []:
            _check_keys("PodTopologySpread defaultConstraints", d, ("maxSkew", "topologyKey", "whenUnsatisfiable",
                                                                     "labelSelector", "minDomains",
                                                                     "nodeAffinityPolicy", "nodeTaintsPolicy",
                                                                     "matchLabelKeys"))
            if d.get("matchLabelKeys"):
                raise UnsupportedArgs("PodTopologySpread defaultConstraints: matchLabelKeys not supported")
            out.default_constraints.append(_spread(d))
    prof_mod.validate_spread_args(out)
    return out


def _preemption_args(args: dict, cur: prof_mod.PreemptionArgs) -> prof_mod.PreemptionArgs:
    _check_keys("DefaultPreemption", args, ("minCandidateNodesPercentage", "minCandidateNodesAbsolute"))
    out = prof_mod.PreemptionArgs(cur.min_candidate_nodes_percentage, cur.min_candidate_nodes_absolute)
    if args.get("minCandidateNodesPercentage") is not None:
        out.min_candidate_nodes_percentage = int(args["minCandidateNodesPercentage"])
    if args.get("minCandidateNodesAbsolute") is not None:
        out.min_candidate_nodes_absolute = int(args["minCandidateNodesAbsolute"])
    return out


def profile_from_config(p: dict) -> prof_mod.SchedulerProfile:
    """One v1beta2 KubeSchedulerProfile -> the converted SchedulerProfile.
    NewPluginConfig (plugins.go:103-179): each in-tree plugin's args are the
    default object with the document's fields decoded over it.  Every arg is
    implemented or refused (UnsupportedArgs), none is dropped."""
    plugins = {}
    for key, ext in _EXT_JSON.items():
        if key in (p.get("plugins") or {}):
            plugins[ext] = _plugin_set(p["plugins"][key])
    sp = prof_mod.SchedulerProfile(plugins=prof_mod.convert_for_simulator(plugins))
    for pc in p.get("pluginConfig") or []:
        name, args = pc.get("name", ""), pc.get("args") or {}
        if name == "NodeResourcesFit":
            sp.fit = _fit_args(args, sp.fit)
        elif name == "NodeResourcesBalancedAllocation":
            _check_keys(name, args, ("resources",))
            if args.get("resources"):
                sp.balanced = prof_mod.BalancedAllocationArgs([(r["name"], int(r.get("weight") or 1))
                                                               for r in args["resources"]])
        elif name == "InterPodAffinity":
            _check_keys(name, args, ("hardPodAffinityWeight", "ignorePreferredTermsOfExistingPods"))
            if args.get("ignorePreferredTermsOfExistingPods"):
                raise UnsupportedArgs("InterPodAffinity args: ignorePreferredTermsOfExistingPods not supported")
            if args.get("hardPodAffinityWeight") is not None:
                sp.hard_pod_affinity_weight = int(args["hardPodAffinityWeight"])
                if not 0 <= sp.hard_pod_affinity_weight <= 100:   # ValidateInterPodAffinityArgs
                    raise ValueError("InterPodAffinityArgs.hardPodAffinityWeight not in valid range [0, 100]")
        elif name == "NodeAffinity":
            sp.node_affinity = _node_affinity_args(args)
        elif name == "PodTopologySpread":
            sp.spread = _spread_args(args, sp.spread)
        elif name == "DefaultPreemption":
            sp.preemption = _preemption_args(args, sp.preemption)
        elif name == "VolumeBinding":
            # bindTimeoutSeconds bounds PreBind's wait (no placement effect);
            # shape scores capacity only behind the VolumeCapacityPriority gate (off)
            _check_keys(name, args, ("bindTimeoutSeconds", "shape"))
        elif name == "NetworkBandwidth":
            sp.network_bandwidth = NetworkBandwidthArgs.from_config(args)
        elif name in prof_mod.SUPPORTED_FILTER or name in prof_mod.SUPPORTED_SCORE:
            if args and set(args) - {"kind", "apiVersion"}:
                raise UnsupportedArgs(f"{name} takes no args the engine knows: {sorted(args)}")
    sp.percentage_of_nodes_to_score = 0      # non-profile fields are reset to the defaults
    return sp


def profiles_from_config(cfg: Optional[dict]) -> List[Tuple[str, prof_mod.SchedulerProfile]]:
    profiles = (cfg or {}).get("profiles") or [{"schedulerName": "default-scheduler"}]
    return [(p.get("schedulerName") or "default-scheduler", profile_from_config(p)) for p in profiles]


# ---- the document ----------------------------------------------------------------------
def load(doc: dict) -> Snapshot:
    """A ResourcesForImport / ResourcesForExport document (already JSON-decoded)."""
    classes, default_prio = _priority_classes(doc.get("priorityClasses") or [])
    namespaces = {}
    for ns in doc.get("namespaces") or []:
        md = ns.get("metadata") or {}
        namespaces[md.get("name", "")] = dict(md.get("labels") or {})
    nodes = [node_from_dict(n) for n in doc.get("nodes") or []]
    names = {n.name for n in nodes}
    if len(names) != len(nodes):
        raise ValueError("duplicate node names")
    volumes = VolumeIndex.from_nodes(nodes, [pv_from_dict(d) for d in doc.get("pvs") or []],
                                     [pvc_from_dict(d) for d in doc.get("pvcs") or []],
                                     [storage_class_from_dict(d) for d in doc.get("storageClasses") or []])
    volumes.run_pv_controller()               # the simulator's PV controller binds Immediate claims
    bound, pending, unsupported = [], [], []
    keyed = []
    for idx, d in enumerate(doc.get("pods") or []):
        pod = pod_from_dict(d)
        spec = d.get("spec") or {}
        pod.priority = _priority(spec, classes, default_prio)
        namespaces.setdefault(pod.namespace, {})
        if pod.node_name:
            if pod.node_name in names:
                bound.append(pod)
            continue
        if pod.has_volumes:
            unsupported.append((pod.namespace, pod.name, "volumes"))
            continue
        if pod.pvc_claims:
            try:
                volumes.groups(pod)
            except VolumeUnsupported as e:
                unsupported.append((pod.namespace, pod.name, f"volumes: {e}"))
                continue
        ts = (d.get("metadata") or {}).get("creationTimestamp") or ""
        keyed.append((-pod.priority, ts, idx, pod))
    keyed.sort(key=lambda t: t[:3])           # PrioritySort, then queue arrival
    pending = [t[3] for t in keyed]
    volumes.add_users(bound)                  # ReadWriteOncePod claims already in use
    services = [service_from_dict(d) for d in doc.get("services") or []]
    controllers = [controller_from_dict(kind, d) for key, kind in
                   (("replicationControllers", "ReplicationController"), ("replicaSets", "ReplicaSet"),
                    ("statefulSets", "StatefulSet")) for d in doc.get(key) or []]
    return Snapshot(nodes, bound, pending, namespaces, profiles_from_config(doc.get("schedulerConfig")),
                    unsupported, volumes,
                    {k: len(doc.get(k) or []) for k in ("pods", "nodes", "pvs", "pvcs", "storageClasses",
                                                         "priorityClasses", "namespaces", "services",
                                                         "replicaSets")},
                    services, controllers)


def schedule_queue(backend, cluster, pending: Sequence[Pod], volumes: Optional[VolumeIndex] = None,
                   nodes: Optional[Sequence[Node]] = None,
                   profile: Optional[prof_mod.SchedulerProfile] = None,
                   snap: Optional[Snapshot] = None) -> List[Optional[str]]:
    """Schedule ``pending`` in queue order on ``backend`` (a ksim.engine.Engine
    or the oracle: ``schedule_batch`` / ``schedule`` and ``eval_pod`` / ``cycle``)
    whose cluster is ``cluster``; returns each pod's node name (None: not
    scheduled).  Stretches of pods whose volume verdicts cannot change run as
    one loaded queue (the batch paths); a pod with unbound WaitForFirstConsumer
    or ReadWriteOncePod claims is encoded at its turn, under the bindings the
    earlier pods made, runs one cycle, and its volumes are assumed on the chosen
    node (VolumeBinding Reserve / PreBind)."""
    from .encode import encode_pods
    labels = {n.name: n.labels for n in (nodes if nodes is not None else (volumes.nodes if volumes else []) or [])}
    out: List[Optional[str]] = []
    n = len(pending)
    i = 0
    while i < n:
        j = i
        while j < n and not (volumes is not None and volumes.stateful(pending[j])):
            j += 1
        if j > i:
            enc = encode_pods(cluster, pending[i:j], volumes=volumes, **_pod_args(profile, snap))
            run = backend.schedule_batch(enc) if hasattr(backend, "schedule_batch") else backend.schedule(enc)
            out.extend(cluster.node_names[c] if c >= 0 else None for c in run[0])
        if j < n:
            pod = pending[j]
            enc = encode_pods(cluster, [pod], volumes=volumes, **_pod_args(profile, snap))
            r = backend.eval_pod(enc, 0) if hasattr(backend, "eval_pod") else backend.cycle(enc, 0)
            node = cluster.node_names[r["chosen"]] if r["chosen"] >= 0 else None
            if node is not None:
                volumes.assume(pod, labels[node], node)   # False: waiting in PreBind for a provisioner
            out.append(node)
            j += 1
        i = j
    return out


def _pod_args(profile: Optional[prof_mod.SchedulerProfile], snap: Optional[Snapshot] = None) -> dict:
    """The profile-dependent part of the pod compile (encode_pods keywords):
    NodeAffinity's addedAffinity, PodTopologySpread's default constraints."""
    if profile is None:
        return {}
    from .topology import SpreadDefaults
    return {"added_affinity": profile.node_affinity,
            "spread": SpreadDefaults(profile.spread, snap.services if snap else (), snap.controllers if snap else ())}


def encode(snap: Snapshot, profile_index: int = 0):
    """(EncodedCluster, EncodedPods of the pending queue, compiled profile)."""
    from .encode import encode_cluster, encode_pods
    sp = snap.profiles[profile_index][1]
    cluster, _ = encode_cluster(snap.nodes, snap.bound, namespaces=snap.namespaces, nb_args=sp.network_bandwidth)
    pods = encode_pods(cluster, snap.pending, volumes=snap.volumes, **_pod_args(sp, snap))
    return cluster, pods, prof_mod.compile_profile(sp, cluster.scalar_names)


# ---- node informer deltas ---------------------------------------------------------------
class NodeCache:
    """The node side of the scheduler cache between snapshots ([upstream]
    pkg/scheduler/internal/cache/cache.go AddNode / UpdateNode / RemoveNode and
    node_tree.go; the simulator drives them from the node informer of its fake
    cluster).  Nodes are kept in informer add order, which is the nodeTree's
    insertion order: an update that moves a node to another zone re-adds it
    (nodeTree.updateNode = removeNode + addNode), a removed node leaves the tree
    and the pods bound to it leave the snapshot.

    ``commit(pending)`` re-encodes the snapshot (the same scalar columns and
    count classes first, label columns for the keys the pods reference) and returns it with ``old_pos`` for ksim_upsert_nodes, which
    replays the engine's binds since the last snapshot on top of it."""

    def __init__(self, nodes: Sequence[Node], bound: Sequence[Pod] = (),
                 namespaces: Optional[Dict[str, Dict[str, str]]] = None,
                 nb_args: Optional[NetworkBandwidthArgs] = None, extra_scalar: Sequence[str] = ()):
        self.nodes: List[Node] = list(nodes)
        self.bound: List[Pod] = list(bound)
        self.namespaces = namespaces
        self.nb_args = nb_args
        self.extra_scalar = list(extra_scalar)
        self.cluster = self._encode((), None)

    def _encode(self, scalar_order, classes_from):
        from .encode import encode_cluster
        c, _ = encode_cluster(self.nodes, self.bound, extra_scalar=self.extra_scalar,
                              namespaces=self.namespaces, nb_args=self.nb_args, scalar_order=scalar_order,
                              classes_from=classes_from)
        return c

    def _index(self, name: str) -> int:
        for i, n in enumerate(self.nodes):
            if n.name == name:
                return i
        raise KeyError(f"node {name!r} not in the cache")

    def add_node(self, node: Node) -> None:
        if any(n.name == node.name for n in self.nodes):
            raise ValueError(f"node {node.name!r} already in the cache")
        self.nodes.append(node)

    def update_node(self, node: Node) -> None:
        from .encode import zone_key
        i = self._index(node.name)
        if zone_key(self.nodes[i].labels) != zone_key(node.labels):
            del self.nodes[i]
            self.nodes.append(node)
        else:
            self.nodes[i] = node

    def remove_node(self, name: str) -> None:
        del self.nodes[self._index(name)]

    def commit(self, pending: Sequence[Pod]):
        """(new EncodedCluster, old_pos, EncodedPods of ``pending``, encoded
        against the new snapshot; pass the queue still to run)."""
        from .encode import EncodeError, encode_pods
        old = self.cluster
        new = self._encode(old.scalar_names, old.topo)
        pods = encode_pods(new, pending)
        if new.topo.keys[:len(old.topo.keys)] != old.topo.keys:
            raise EncodeError("count classes changed ids across the node delta")
        pos = {name: i for i, name in enumerate(old.node_names)}
        old_pos = np.array([pos.get(name, -1) for name in new.node_names], np.int32)
        self.cluster = new
        return new, old_pos, pods
