"""Minimal Kubernetes object model for the hot path (Node, Pod and the fields
the six north-star plugins read), plus resource.Quantity parsing.

Objects can be built directly or parsed from v1 JSON/YAML dicts (the shape of
``ResourcesForImport`` in simulator/export/export.go:56-65).
"""
from __future__ import annotations

import functools
import math
import re
from dataclasses import dataclass, field
from fractions import Fraction
from typing import Dict, List, Optional, Tuple

# ---- resource.Quantity ----------------------------------------------------
_BIN = {"Ki": 2 ** 10, "Mi": 2 ** 20, "Gi": 2 ** 30, "Ti": 2 ** 40, "Pi": 2 ** 50, "Ei": 2 ** 60}
_DEC = {"n": Fraction(1, 10 ** 9), "u": Fraction(1, 10 ** 6), "m": Fraction(1, 1000), "": 1,
        "k": 10 ** 3, "M": 10 ** 6, "G": 10 ** 9, "T": 10 ** 12, "P": 10 ** 15, "E": 10 ** 18}
_QRE = re.compile(r"^([+-]?(?:\d+\.?\d*|\.\d+))(?:(Ki|Mi|Gi|Ti|Pi|Ei|[numkMGTPE])|[eE]([+-]?\d+))?$")


def parse_quantity(q) -> Fraction:
    """Exact value of a k8s resource.Quantity string (or number)."""
    if isinstance(q, (int, Fraction)):
        return Fraction(q)
    if isinstance(q, float):
        return Fraction(str(q))
    return _parse_quantity_str(str(q))


@functools.lru_cache(maxsize=65536)
def _parse_quantity_str(q: str) -> Fraction:
    # clusters repeat a few quantity strings many times (Fractions are immutable)
    s = q.strip()
    m = _QRE.match(s)
    if not m:
        raise ValueError(f"invalid quantity {q!r}")
    num = Fraction(m.group(1))
    if m.group(2):
        suf = m.group(2)
        num *= _BIN[suf] if suf in _BIN else _DEC[suf]
    elif m.group(3):
        num *= Fraction(10) ** int(m.group(3))
    return num


def quantity_value(q) -> int:
    """resource.Quantity.Value(): rounds up to an integer."""
    if isinstance(q, str):
        return _quantity_value_str(q)
    return math.ceil(parse_quantity(q))


def quantity_milli_value(q) -> int:
    """resource.Quantity.MilliValue(): value*1000 rounded up."""
    if isinstance(q, str):
        return _quantity_milli_str(q)
    return math.ceil(parse_quantity(q) * 1000)


@functools.lru_cache(maxsize=65536)
def _quantity_value_str(q: str) -> int:
    return math.ceil(_parse_quantity_str(q))


@functools.lru_cache(maxsize=65536)
def _quantity_milli_str(q: str) -> int:
    return math.ceil(_parse_quantity_str(q) * 1000)


# ---- objects --------------------------------------------------------------
@dataclass
class Taint:
    key: str
    value: str = ""
    effect: str = "NoSchedule"


@dataclass
class Toleration:
    key: str = ""
    operator: str = ""          # "" == Equal
    value: str = ""
    effect: str = ""

    def tolerates(self, t: Taint) -> bool:
        """k8s.io/api core/v1 Toleration.ToleratesTaint."""
        if self.effect and self.effect != t.effect:
            return False
        if self.key and self.key != t.key:
            return False
        if self.operator in ("", "Equal"):
            return self.value == t.value
        if self.operator == "Exists":
            return True
        return False


@dataclass
class Requirement:
    key: str
    operator: str               # In NotIn Exists DoesNotExist Gt Lt
    values: List[str] = field(default_factory=list)


@dataclass
class NodeSelectorTerm:
    match_expressions: List[Requirement] = field(default_factory=list)
    match_fields: List[Requirement] = field(default_factory=list)


@dataclass
class PreferredTerm:
    weight: int
    term: NodeSelectorTerm


@dataclass
class LabelSelector:
    """metav1.LabelSelector.  A pod-side field holding ``None`` is a nil
    selector (labels.Nothing() after LabelSelectorAsSelector); a LabelSelector
    with no requirements is labels.Everything()."""
    match_labels: Dict[str, str] = field(default_factory=dict)
    match_expressions: List[Requirement] = field(default_factory=list)

    def empty(self) -> bool:
        return not self.match_labels and not self.match_expressions

    def matches(self, labels: Dict[str, str]) -> bool:
        """labels.Selector.Matches of LabelSelectorAsSelector(self).  Invalid
        requirements (an operator this model does not know, or In/NotIn
        without values) make the selector match nothing (the conversion errs
        and callers treat the error as a non-match)."""
        for k, v in self.match_labels.items():
            if labels.get(k) != v:
                return False
        for r in self.match_expressions:
            has = r.key in labels
            if r.operator == "In":
                if not r.values or not has or labels[r.key] not in r.values:
                    return False
            elif r.operator == "NotIn":
                if not r.values:
                    return False
                if has and labels[r.key] in r.values:
                    return False
            elif r.operator == "Exists":
                if r.values or not has:
                    return False
            elif r.operator == "DoesNotExist":
                if r.values or has:
                    return False
            else:
                return False
        return True

    def key(self):
        """Canonical, hashable form (requirement order does not change the
        selector: labels.Requirements are sorted by key)."""
        return (tuple(sorted(self.match_labels.items())),
                tuple(sorted((r.key, r.operator, tuple(sorted(r.values))) for r in self.match_expressions)))


def selector_matches(sel: "Optional[LabelSelector]", labels: Dict[str, str]) -> bool:
    """LabelSelectorAsSelector(sel).Matches(labels): nil -> Nothing."""
    return sel is not None and sel.matches(labels)


@dataclass
class TopologySpreadConstraint:
    """v1.TopologySpreadConstraint (fields read by [upstream] podtopologyspread)."""
    max_skew: int
    topology_key: str
    when_unsatisfiable: str = "DoNotSchedule"      # or ScheduleAnyway
    label_selector: Optional[LabelSelector] = None
    min_domains: Optional[int] = None
    node_affinity_policy: Optional[str] = None     # nil -> Honor
    node_taints_policy: Optional[str] = None       # nil -> Ignore


@dataclass
class PodAffinityTerm:
    """v1.PodAffinityTerm."""
    topology_key: str
    label_selector: Optional[LabelSelector] = None
    namespaces: List[str] = field(default_factory=list)
    namespace_selector: Optional[LabelSelector] = None


@dataclass
class WeightedPodAffinityTerm:
    weight: int
    term: PodAffinityTerm


@dataclass
class ContainerPort:
    """v1.ContainerPort fields NodePorts reads (hostPort 0: not a host port)."""
    host_port: int = 0
    protocol: str = "TCP"
    host_ip: str = ""


@dataclass
class Container:
    requests: Dict[str, str] = field(default_factory=dict)
    ports: List[ContainerPort] = field(default_factory=list)
    image: str = ""

    @property
    def host_ports(self) -> List[int]:
        return [p.host_port for p in self.ports if p.host_port > 0]


@dataclass
class Node:
    name: str
    labels: Dict[str, str] = field(default_factory=dict)
    taints: List[Taint] = field(default_factory=list)
    allocatable: Dict[str, str] = field(default_factory=dict)
    unschedulable: bool = False
    images: List[Tuple[List[str], int]] = field(default_factory=list)   # status.images: (names, sizeBytes)
    annotations: Dict[str, str] = field(default_factory=dict)


@dataclass
class Pod:
    name: str
    namespace: str = "default"
    labels: Dict[str, str] = field(default_factory=dict)
    containers: List[Container] = field(default_factory=list)
    init_containers: List[Container] = field(default_factory=list)
    overhead: Dict[str, str] = field(default_factory=dict)
    node_selector: Dict[str, str] = field(default_factory=dict)
    required_terms: Optional[List[NodeSelectorTerm]] = None   # None: no required affinity
    preferred_terms: List[PreferredTerm] = field(default_factory=list)
    tolerations: List[Toleration] = field(default_factory=list)
    node_name: str = ""
    has_volumes: bool = False          # a volume the engine does not model (inline disks, CSI, ephemeral, ...)
    pvc_claims: List[str] = field(default_factory=list)   # persistentVolumeClaim.claimName of each such volume
    priority: int = 0
    topology_spread: List[TopologySpreadConstraint] = field(default_factory=list)
    pod_affinity_required: List[PodAffinityTerm] = field(default_factory=list)
    pod_affinity_preferred: List[WeightedPodAffinityTerm] = field(default_factory=list)
    pod_anti_affinity_required: List[PodAffinityTerm] = field(default_factory=list)
    pod_anti_affinity_preferred: List[WeightedPodAffinityTerm] = field(default_factory=list)
    annotations: Dict[str, str] = field(default_factory=dict)
    # metav1.GetControllerOf: (apiVersion, kind, name) of the ownerReference with controller: true
    owner: Optional[Tuple[str, str, str]] = None

    def has_pod_affinity(self) -> bool:
        """PodInfo: pods with any (anti)affinity term (NodeInfo.PodsWithAffinity)."""
        return bool(self.pod_affinity_required or self.pod_affinity_preferred or
                    self.pod_anti_affinity_required or self.pod_anti_affinity_preferred)


@dataclass
class PersistentVolume:
    """v1.PersistentVolume fields VolumeBinding / VolumeZone read (bound claims,
    and the static binding of unbound WaitForFirstConsumer claims)."""
    name: str
    labels: Dict[str, str] = field(default_factory=dict)
    node_affinity: Optional[List[NodeSelectorTerm]] = None   # spec.nodeAffinity.required.nodeSelectorTerms
    source: str = ""                                        # the spec key of its volume source (csi, local, ...)
    access_modes: List[str] = field(default_factory=list)
    capacity: int = 0                                       # spec.capacity.storage (bytes)
    storage_class: str = ""                                 # spec.storageClassName
    claim_ref: Optional[Tuple[str, str]] = None             # spec.claimRef (namespace, name)
    volume_mode: str = "Filesystem"                         # spec.volumeMode (nil: Filesystem)
    deleting: bool = False                                  # metadata.deletionTimestamp set


@dataclass
class PersistentVolumeClaim:
    name: str
    namespace: str = "default"
    volume_name: str = ""                                    # spec.volumeName ("" = unbound)
    access_modes: List[str] = field(default_factory=list)
    storage_class: Optional[str] = None                      # spec.storageClassName (None: unset)
    request: int = 0                                         # spec.resources.requests.storage (bytes)
    selector: Optional[LabelSelector] = None                 # spec.selector
    volume_mode: str = "Filesystem"                          # spec.volumeMode (nil: Filesystem)
    selected_node: str = ""                                  # annotation volume.kubernetes.io/selected-node


@dataclass
class StorageClass:
    """storage.k8s.io/v1 StorageClass fields the volume binder reads."""
    name: str
    provisioner: str = ""
    volume_binding_mode: str = "Immediate"                   # or WaitForFirstConsumer
    # allowedTopologies: terms OR-ed, each a list of (key, values) requirements AND-ed
    allowed_topologies: List[List[Tuple[str, List[str]]]] = field(default_factory=list)


# ---- v1 dict parsing --------------------------------------------------------
# Volume sources the volume filter plugins (VolumeRestrictions, *Limits,
# VolumeBinding, VolumeZone) act on; pods with none of them pass all of those.
# persistentVolumeClaim volumes are kept as claims (Pod.pvc_claims); the others
# mark the pod has_volumes (not modelled).
_VOLUME_SOURCES = ("persistentVolumeClaim", "gcePersistentDisk", "awsElasticBlockStore",
                   "azureDisk", "csi", "rbd", "iscsi", "cinder", "ephemeral")
_PV_SOURCES = ("csi", "local", "hostPath", "nfs", "awsElasticBlockStore", "gcePersistentDisk", "azureDisk",
               "azureFile", "cinder", "rbd", "iscsi", "fc", "cephfs", "glusterfs", "portworxVolume",
               "vsphereVolume", "flexVolume", "flocker", "quobyte", "scaleIO", "storageos", "photonPersistentDisk")


def pv_from_dict(d: dict) -> PersistentVolume:
    md, spec = d.get("metadata", {}) or {}, d.get("spec", {}) or {}
    req = ((spec.get("nodeAffinity") or {}).get("required"))
    ref = spec.get("claimRef") or None
    cap = (spec.get("capacity") or {}).get("storage")
    return PersistentVolume(
        name=md.get("name", ""), labels=dict(md.get("labels") or {}),
        node_affinity=None if req is None else [_term(t) for t in (req.get("nodeSelectorTerms") or [])],
        source=next((k for k in _PV_SOURCES if k in spec), ""),
        access_modes=list(spec.get("accessModes") or []),
        capacity=quantity_value(cap) if cap is not None else 0,
        storage_class=spec.get("storageClassName", "") or "",
        claim_ref=None if not ref else (ref.get("namespace", "") or "", ref.get("name", "") or ""),
        volume_mode=spec.get("volumeMode") or "Filesystem",
        deleting=bool(md.get("deletionTimestamp")))


def pvc_from_dict(d: dict) -> PersistentVolumeClaim:
    md, spec = d.get("metadata", {}) or {}, d.get("spec", {}) or {}
    req = ((spec.get("resources") or {}).get("requests") or {}).get("storage")
    return PersistentVolumeClaim(name=md.get("name", ""), namespace=md.get("namespace", "default") or "default",
                                 volume_name=spec.get("volumeName", "") or "",
                                 access_modes=list(spec.get("accessModes") or []),
                                 storage_class=spec.get("storageClassName"),
                                 request=quantity_value(req) if req is not None else 0,
                                 selector=_selector(spec.get("selector")),
                                 volume_mode=spec.get("volumeMode") or "Filesystem",
                                 selected_node=(md.get("annotations") or {}).get("volume.kubernetes.io/selected-node",
                                                                                 "") or "")


def storage_class_from_dict(d: dict) -> StorageClass:
    md = d.get("metadata", {}) or {}
    topo = []
    for t in d.get("allowedTopologies") or []:
        topo.append([(e.get("key", ""), list(e.get("values") or [])) for e in (t.get("matchLabelExpressions") or [])])
    return StorageClass(name=md.get("name", ""), provisioner=d.get("provisioner", "") or "",
                        volume_binding_mode=d.get("volumeBindingMode") or "Immediate", allowed_topologies=topo)

def _req(d) -> Requirement:
    return Requirement(d["key"], d["operator"], list(d.get("values") or []))


def _term(d) -> NodeSelectorTerm:
    return NodeSelectorTerm([_req(x) for x in (d.get("matchExpressions") or [])],
                            [_req(x) for x in (d.get("matchFields") or [])])


def _selector(d) -> Optional[LabelSelector]:
    if d is None:
        return None
    return LabelSelector(dict(d.get("matchLabels") or {}),
                         [_req(x) for x in (d.get("matchExpressions") or [])])


def _pod_term(d) -> PodAffinityTerm:
    return PodAffinityTerm(d.get("topologyKey", ""), _selector(d.get("labelSelector")),
                           list(d.get("namespaces") or []), _selector(d.get("namespaceSelector")))


def _weighted(d) -> WeightedPodAffinityTerm:
    return WeightedPodAffinityTerm(int(d.get("weight", 0)), _pod_term(d.get("podAffinityTerm") or {}))


def _spread(d) -> TopologySpreadConstraint:
    return TopologySpreadConstraint(int(d.get("maxSkew", 1)), d.get("topologyKey", ""),
                                    d.get("whenUnsatisfiable", "DoNotSchedule"),
                                    _selector(d.get("labelSelector")), d.get("minDomains"),
                                    d.get("nodeAffinityPolicy"), d.get("nodeTaintsPolicy"))


def node_from_dict(d: dict) -> Node:
    md, spec, status = d.get("metadata", {}), d.get("spec", {}) or {}, d.get("status", {}) or {}
    return Node(
        name=md.get("name", ""),
        labels=dict(md.get("labels") or {}),
        taints=[Taint(t["key"], t.get("value", ""), t.get("effect", "")) for t in (spec.get("taints") or [])],
        allocatable={k: str(v) for k, v in (status.get("allocatable") or {}).items()},
        unschedulable=bool(spec.get("unschedulable", False)),
        images=[(list(im.get("names") or []), int(im.get("sizeBytes") or 0)) for im in (status.get("images") or [])],
        annotations={k: str(v) for k, v in (md.get("annotations") or {}).items()},
    )


def _container(c) -> Container:
    res = c.get("resources") or {}
    return Container({k: str(v) for k, v in (res.get("requests") or {}).items()},
                     [ContainerPort(int(p.get("hostPort") or 0), p.get("protocol") or "TCP", p.get("hostIP") or "")
                      for p in (c.get("ports") or [])], c.get("image") or "")


def pod_from_dict(d: dict) -> Pod:
    md, spec = d.get("metadata", {}), d.get("spec", {}) or {}
    affinity = spec.get("affinity") or {}
    aff = affinity.get("nodeAffinity") or {}
    pa = affinity.get("podAffinity") or {}
    paa = affinity.get("podAntiAffinity") or {}
    req = aff.get("requiredDuringSchedulingIgnoredDuringExecution")
    pref = aff.get("preferredDuringSchedulingIgnoredDuringExecution") or []
    return Pod(
        name=md.get("name", ""),
        namespace=md.get("namespace", "default"),
        labels=dict(md.get("labels") or {}),
        containers=[_container(c) for c in (spec.get("containers") or [])],
        init_containers=[_container(c) for c in (spec.get("initContainers") or [])],
        overhead={k: str(v) for k, v in (spec.get("overhead") or {}).items()},
        node_selector=dict(spec.get("nodeSelector") or {}),
        required_terms=None if req is None else [_term(t) for t in (req.get("nodeSelectorTerms") or [])],
        preferred_terms=[PreferredTerm(int(p.get("weight", 0)), _term(p.get("preference") or {})) for p in pref],
        tolerations=[Toleration(t.get("key", ""), t.get("operator", ""), t.get("value", ""), t.get("effect", ""))
                     for t in (spec.get("tolerations") or [])],
        node_name=spec.get("nodeName", "") or "",
        has_volumes=any(any(k in v for k in _VOLUME_SOURCES if k != "persistentVolumeClaim")
                        for v in (spec.get("volumes") or [])),
        pvc_claims=[(v.get("persistentVolumeClaim") or {}).get("claimName", "")
                    for v in (spec.get("volumes") or []) if "persistentVolumeClaim" in v],
        priority=int(spec.get("priority") or 0),
        topology_spread=[_spread(c) for c in (spec.get("topologySpreadConstraints") or [])],
        pod_affinity_required=[_pod_term(t) for t in (pa.get("requiredDuringSchedulingIgnoredDuringExecution") or [])],
        pod_affinity_preferred=[_weighted(t) for t in (pa.get("preferredDuringSchedulingIgnoredDuringExecution") or [])],
        pod_anti_affinity_required=[_pod_term(t) for t in
                                    (paa.get("requiredDuringSchedulingIgnoredDuringExecution") or [])],
        pod_anti_affinity_preferred=[_weighted(t) for t in
                                     (paa.get("preferredDuringSchedulingIgnoredDuringExecution") or [])],
        annotations={k: str(v) for k, v in (md.get("annotations") or {}).items()},
        owner=next(((o.get("apiVersion", ""), o.get("kind", ""), o.get("name", ""))
                    for o in (md.get("ownerReferences") or []) if o.get("controller")), None),
    )


@dataclass
class Service:
    """v1.Service as helper.GetPodServices reads it: a nil selector matches no pod."""
    name: str
    namespace: str = "default"
    selector: Optional[Dict[str, str]] = None


@dataclass
class Controller:
    """A ReplicationController (selector: a label map, nil = none) or a
    ReplicaSet / StatefulSet (selector: a LabelSelector, nil = Nothing), as
    helper.DefaultSelector reads them; kind is the object's Kind."""
    kind: str
    name: str
    namespace: str = "default"
    selector: object = None


def service_from_dict(d: dict) -> Service:
    md, spec = d.get("metadata", {}) or {}, d.get("spec", {}) or {}
    sel = spec.get("selector")
    return Service(md.get("name", ""), md.get("namespace", "default"), None if sel is None else dict(sel))


def controller_from_dict(kind: str, d: dict) -> Controller:
    md, spec = d.get("metadata", {}) or {}, d.get("spec", {}) or {}
    sel = spec.get("selector")
    if kind == "ReplicationController":
        sel = None if sel is None else dict(sel)
    else:
        sel = _selector(sel)
    return Controller(kind, md.get("name", ""), md.get("namespace", "default"), sel)
