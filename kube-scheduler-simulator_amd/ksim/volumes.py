"""PersistentVolumeClaims for VolumeBinding, VolumeZone and VolumeRestrictions
([upstream] k8s.io/kubernetes v1.26.2 pkg/scheduler/framework/
plugins/volumebinding (volume_binding.go PreFilter / Filter / Reserve, binder.go
FindPodVolumes / AssumePodVolumes), pkg/controller/volume/persistentvolume/util
FindMatchingVolume, volumezone (volume_zone.go getPVbyPod / Filter) and
volumerestrictions (ReadWriteOncePod)).  The simulator imports PVs, PVCs and
StorageClasses with the cluster (/root/reference/simulator/export/export.go:
47-49,59-61) and runs the PV controller, which binds Immediate claims
(the reference's documents carry "pv.kubernetes.io/bound-by-controller").

Every per-node verdict is a set of groups of NodeSelectorTerms (ksim_engine.h
"Volume groups"): the node passes a filter iff every group has a matching term.

  VolumeBinding, bound claim   one group per PV with spec.nodeAffinity: its
                 terms.  CheckNodeAffinity builds a node with labels only, so a
                 matchFields metadata.name requirement compares with "".
  VolumeBinding, unbound WaitForFirstConsumer claim   one group per claim: the
                 node-affinity terms of every PV FindMatchingVolume could pick
                 for it (class, access modes, volume mode, capacity, selector,
                 not claimed by another claim), plus the class's
                 allowedTopologies when it can be provisioned dynamically; no
                 group when some candidate has no node affinity or provisioning
                 is unrestricted.  Claims of one pod that compete for a PV
                 (FindPodVolumes' chosenPVs) get one exact group: the names of
                 the nodes where the whole matching succeeds.
  VolumeZone     one group per bound PV label whose key is a topology label and
                 whose value parses (LabelZonesToSet): {key In zones} or {no
                 topology label on the node}; unbound WaitForFirstConsumer
                 claims are skipped.
  A claim whose provisioning already started (annotation
  volume.kubernetes.io/selected-node) admits that node only, if its class can
  provision there.
The bound-PV groups come first; the unbound-claim groups carry
abi.VB_UNBOUND_GROUP in their group index, so the engine's failure detail says
which reasons the node gets (ErrReasonNodeConflict, ErrReasonBindConflict, or
both, in FindPodVolumes' order).

PreFilter rejections (VolumeBinding PreFilter, UnschedulableAndUnresolvable: a
missing claim, an unbound Immediate claim -- a claim whose class does not
exist is Immediate, IsDelayBindingMode treats NotFound as not delayed):
``prefilter_rejection`` gives the message the hosts record as VolumeBinding's
PreFilter status (no Filter runs, nextStartNodeIndex unchanged); the engine
gets one group no node matches, which leaves nextStartNodeIndex where it was
(every node is processed) and the pod unschedulable.

The verdicts depend on which PVs earlier pods took, so a pod with unbound
WaitForFirstConsumer claims is encoded at its turn (``stateful``;
ksim.ingest.schedule_queue) and ``assume`` records its bindings
(AssumePodVolumes) once the cycle chose a node.  Dynamic provisioning: the
simulator's PV controller runs without provisioning plugins
(/root/reference/simulator/controller/pvcontroller.go, VolumeConfig{}) and no
external provisioner runs, so a pod whose claims need provisioning is assumed
on the node, its claims get the selected-node annotation, and it waits in
PreBind (``waiting``; it never binds: its bindTimeoutSeconds run out after the
simulation).  ``provisioning=True`` models a working provisioner instead (the
PVC is bound to a new PV of the claim's size, without node affinity).

Still unsupported (VolumeUnsupported: the pod is reported and not scheduled,
never mis-scheduled): PVs counted against node volume limits (EBS / GCE PD /
Azure disk / Cinder by their in-tree limit plugins; CSI volumes by
NodeVolumeLimits when a node publishes attachable-volumes-* limits);
ReadWriteOncePod claims (the ReadWriteOncePod feature gate is alpha and off in
v1.26: the API server refuses the access mode and VolumeRestrictions skips
the check; the reference sets no feature gates).
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Sequence, Set, Tuple

from . import abi
from .model import (NodeSelectorTerm, PersistentVolume, PersistentVolumeClaim, Pod, Requirement, StorageClass,
                    selector_matches)

# volume_zone.go topologyLabels
TOPOLOGY_LABELS = ("failure-domain.beta.kubernetes.io/zone", "failure-domain.beta.kubernetes.io/region",
                   "topology.kubernetes.io/zone", "topology.kubernetes.io/region")
LIMITED_SOURCES = ("awsElasticBlockStore", "gcePersistentDisk", "azureDisk", "cinder")
NO_PROVISIONER = "kubernetes.io/no-provisioner"                     # volume.NotSupportedProvisioner
MSG_VOLUME_BINDING = "node(s) had volume node affinity conflict"    # volumebinding ErrReasonNodeConflict
MSG_BIND_CONFLICT = "node(s) didn't find available persistent volumes to bind"   # ErrReasonBindConflict
MSG_VOLUME_ZONE = "node(s) had no available volume zone"            # volumezone ErrReasonConflict
MSG_UNBOUND_IMMEDIATE = "pod has unbound immediate PersistentVolumeClaims"

_NEVER = NodeSelectorTerm([], [Requirement("", "__false__", [])])   # a term no node matches
_ALWAYS = NodeSelectorTerm([], [Requirement("", "__true__", [])])


class VolumeUnsupported(ValueError):
    pass


def label_zones_to_set(value: str) -> Optional[List[str]]:
    """volumehelpers.LabelZonesToSet; None when the value does not parse."""
    out = []
    for z in value.split("__"):
        z = z.strip()
        if not z:
            return None
        if z not in out:
            out.append(z)
    return out


def _req_ok(r: Requirement, labels: Dict[str, str]) -> bool:
    has = r.key in labels
    if r.operator == "In":
        return bool(r.values) and has and labels[r.key] in r.values
    if r.operator == "NotIn":
        return bool(r.values) and (not has or labels[r.key] not in r.values)
    if r.operator == "Exists":
        return not r.values and has
    if r.operator == "DoesNotExist":
        return not r.values and not has
    if r.operator in ("Gt", "Lt"):
        if len(r.values) != 1 or not has:
            return False
        try:
            a, b = int(labels[r.key]), int(r.values[0])
        except ValueError:
            return False
        return a > b if r.operator == "Gt" else a < b
    return False


def pv_node_affinity_ok(pv: PersistentVolume, labels: Dict[str, str]) -> bool:
    """volumeutil.CheckNodeAffinity on a node carrying labels only."""
    if pv.node_affinity is None:
        return True
    for t in pv.node_affinity:
        if not t.match_expressions and not t.match_fields:
            continue
        if not all(_req_ok(r, labels) for r in t.match_expressions):
            continue
        ok = True
        for r in t.match_fields:   # the node's name is ""
            well = r.key == "metadata.name" and r.operator in ("In", "NotIn") and len(r.values) == 1
            if not well or (r.values[0] == "") != (r.operator == "In"):
                ok = False
        if ok:
            return True
    return False


def binding_message(detail: int) -> str:
    """VolumeBinding Filter's Status.Message(): its reasons joined (FindPodVolumes order)."""
    out = []
    if detail & abi.VB_NODE_CONFLICT or not detail:
        out.append(MSG_VOLUME_BINDING)
    if detail & abi.VB_BIND_CONFLICT:
        out.append(MSG_BIND_CONFLICT)
    return ", ".join(out)


def can_provision(sc: Optional[StorageClass]) -> bool:
    """checkVolumeProvisions: a class with no provisioner ("" or
    kubernetes.io/no-provisioner) cannot provision."""
    return sc is not None and sc.provisioner not in ("", NO_PROVISIONER)


def topology_ok(sc: StorageClass, labels: Dict[str, str]) -> bool:
    """v1helper.MatchTopologySelectorTerms over allowedTopologies."""
    if not sc.allowed_topologies:
        return True
    for term in sc.allowed_topologies:
        if not term:
            continue                                   # an empty term selects nothing
        if all(vals and k in labels and labels[k] in vals for k, vals in term):
            return True
    return False


class VolumeIndex:
    """The snapshot's PVs, PVCs and StorageClasses (ResourcesForImport pvs /
    pvcs / storageClasses) and the bindings the run has made so far."""

    def __init__(self, pvs: Iterable[PersistentVolume] = (), pvcs: Iterable[PersistentVolumeClaim] = (),
                 csi_limits: bool = False, classes: Iterable[StorageClass] = (), provisioning: bool = False):
        self.pvs: Dict[str, PersistentVolume] = {pv.name: pv for pv in pvs}
        self.pvcs: Dict[Tuple[str, str], PersistentVolumeClaim] = {(c.namespace, c.name): c for c in pvcs}
        self.classes: Dict[str, StorageClass] = {c.name: c for c in classes}
        self.csi_limits = csi_limits          # some node publishes attachable-volumes-* allocatable
        self.users: Dict[Tuple[str, str], int] = {}   # claim -> pods on nodes using it (RWOP)
        self.provisioned = 0
        self.nodes: Optional[list] = None     # the cluster's nodes (the exact group of competing claims)
        self.provisioning = provisioning      # a provisioner acts on selected-node claims (none in the simulator)
        self.waiting: Dict[Tuple[str, str], str] = {}   # pods waiting in PreBind for provisioning -> node

    @staticmethod
    def from_nodes(nodes, pvs=(), pvcs=(), classes=(), provisioning: bool = False) -> "VolumeIndex":
        lim = any(k.startswith("attachable-volumes-") for n in nodes for k in n.allocatable)
        v = VolumeIndex(pvs, pvcs, lim, classes, provisioning)
        v.nodes = list(nodes)
        return v

    # ---- the PV controller (Immediate claims) ---------------------------------
    def _class_of(self, pvc: PersistentVolumeClaim) -> str:
        return pvc.storage_class or ""

    def delay_binding(self, pvc: PersistentVolumeClaim) -> bool:
        """IsDelayBindingMode: class "", a class that does not exist (NotFound is
        not an error there) or Immediate: False."""
        sc = self.classes.get(self._class_of(pvc))
        return sc is not None and sc.volume_binding_mode == "WaitForFirstConsumer"

    def candidates(self, pvc: PersistentVolumeClaim, exclude: Set[str] = frozenset()) -> List[PersistentVolume]:
        """The PVs FindMatchingVolume may pick for pvc, node affinity not
        checked: a PV pre-bound to the claim (spec.claimRef) alone -- it is
        returned at once, or nothing if the node does not suit it -- else the
        available PVs of the claim's class with its access modes, volume mode,
        selector and at least its size, smallest first (ties by name: upstream
        walks an unordered cache)."""
        key = (pvc.namespace, pvc.name)
        out = []
        for pv in sorted(self.pvs.values(), key=lambda v: v.name):
            if pv.name in exclude or (pv.claim_ref is not None and pv.claim_ref != key):
                continue                              # bound (or pre-bound) to another claim
            if pv.capacity < pvc.request or pv.volume_mode != pvc.volume_mode or pv.deleting:
                continue
            if pv.claim_ref == key:
                return [pv]                           # IsVolumeBoundToClaim: taken as it is
            if pvc.selector is not None and not selector_matches(pvc.selector, pv.labels):
                continue
            if pv.storage_class != self._class_of(pvc) or not set(pvc.access_modes) <= set(pv.access_modes):
                continue
            out.append(pv)
        out.sort(key=lambda pv: (pv.capacity, pv.name))
        return out

    def _pick(self, pvc: PersistentVolumeClaim, labels: Dict[str, str], exclude: Set[str]):
        """FindMatchingVolume on a node: the smallest candidate whose node
        affinity the node satisfies; a pre-bound PV that it does not: None."""
        for pv in self.candidates(pvc, exclude):
            if pv_node_affinity_ok(pv, labels):
                return pv
            if pv.claim_ref == (pvc.namespace, pvc.name):
                return None
        return None

    def bind(self, pvc: PersistentVolumeClaim, pv: PersistentVolume) -> None:
        pv.claim_ref = (pvc.namespace, pvc.name)
        pvc.volume_name = pv.name

    def run_pv_controller(self) -> int:
        """The PV controller's sync of every unbound Immediate claim (class ""
        or volumeBindingMode Immediate, or a class that does not exist): bind it
        to the smallest matching available PV (findBestMatchForClaim, no node);
        claims pre-bound by a PV's claimRef first.  Claims with no match stay
        unbound.  Returns the number of bindings."""
        n = 0
        for pvc in self.pvcs.values():            # a claim naming its PV: the PV is bound to it
            pv = self.pvs.get(pvc.volume_name) if pvc.volume_name else None
            if pv is not None and pv.claim_ref is None:
                pv.claim_ref = (pvc.namespace, pvc.name)
        for pvc in self.pvcs.values():
            if pvc.volume_name or self.delay_binding(pvc):
                continue
            # the controller's volume index holds only PVs with the claim's access modes
            c = [pv for pv in self.candidates(pvc) if set(pvc.access_modes) <= set(pv.access_modes)]
            if c:
                self.bind(pvc, c[0])
                n += 1
        return n

    def add_users(self, pods: Iterable[Pod]) -> None:
        """Pods on nodes (bound pods, and every pod the run binds): the claims they use."""
        for p in pods:
            for claim in p.pvc_claims:
                k = (p.namespace, claim)
                self.users[k] = self.users.get(k, 0) + 1

    # ---- per pod ---------------------------------------------------------------
    def _claims(self, pod: Pod):
        """(bound PVs, unbound delay-binding claims) of the pod, or a PreFilter
        rejection message (str)."""
        bound, delay = [], []
        for claim in pod.pvc_claims:
            pvc = self.pvcs.get((pod.namespace, claim))
            if pvc is None:
                return f'persistentvolumeclaim "{claim}" not found'
            if "ReadWriteOncePod" in pvc.access_modes:
                raise VolumeUnsupported("ReadWriteOncePod: feature gate off in v1.26")
            if pvc.volume_name:
                pv = self.pvs.get(pvc.volume_name)
                if pv is None:
                    raise VolumeUnsupported(f"persistentvolume {pvc.volume_name!r} not found")
                if pv.source in LIMITED_SOURCES or (pv.source == "csi" and self.csi_limits):
                    raise VolumeUnsupported(f"persistentvolume {pv.name!r}: {pv.source} volumes count against "
                                            f"node limits")
                bound.append(pv)
                continue
            if not self.delay_binding(pvc):
                return MSG_UNBOUND_IMMEDIATE
            delay.append(pvc)
        return bound, delay

    def prefilter_rejection(self, pod: Pod) -> Optional[str]:
        """VolumeBinding PreFilter's UnschedulableAndUnresolvable message, or None."""
        if not pod.pvc_claims:
            return None
        got = self._claims(pod)
        return got if isinstance(got, str) else None

    def stateful(self, pod: Pod) -> bool:
        """The pod's verdicts depend on the bindings earlier pods make."""
        for claim in pod.pvc_claims:
            pvc = self.pvcs.get((pod.namespace, claim))
            if pvc is not None and not pvc.volume_name and self.delay_binding(pvc):
                return True
        return False

    def _delay_sorted(self, delay: List[PersistentVolumeClaim]) -> List[PersistentVolumeClaim]:
        return sorted(delay, key=lambda c: c.request)     # byPVCSize (stable here)

    def match_on_node(self, pod: Pod, labels: Dict[str, str], name: Optional[str] = None):
        """FindPodVolumes for the unbound delay-binding claims on one node
        (``name``: the node's name, for claims with a selected node):
        ([(pvc, pv)] static bindings, [pvc] to provision) or None (the node
        fails: no PV and no provisioning)."""
        got = self._claims(pod)
        if isinstance(got, str):
            return None
        _, delay = got
        chosen: Set[str] = set()
        static, provision = [], []
        for pvc in delay:                                 # AnnSelectedNode: that node only, to provision
            if pvc.selected_node:
                if name is not None and pvc.selected_node != name:
                    return None
                provision.append(pvc)
        for pvc in self._delay_sorted([c for c in delay if not c.selected_node]):
            pv = self._pick(pvc, labels, chosen)
            if pv is not None:
                chosen.add(pv.name)
                static.append((pvc, pv))
            else:
                provision.append(pvc)
        for pvc in provision:                             # checkVolumeProvisions
            sc = self.classes.get(self._class_of(pvc))
            if not can_provision(sc) or not topology_ok(sc, labels):
                return None
        return static, provision

    def groups(self, pod: Pod, nodes: Optional[Sequence] = None) -> Tuple[List[List[NodeSelectorTerm]],
                                                                           List[List[NodeSelectorTerm]], int]:
        """(VolumeBinding groups, VolumeZone groups, how many of the VolumeBinding
        groups are bound-PV groups -- the rest are unbound-claim groups) of the
        pod under the current bindings.  ``nodes`` (objects with name /
        labels): needed only for the exact group of competing claims."""
        got = self._claims(pod)
        if isinstance(got, str):
            return [[_NEVER]], [], 1                      # a PreFilter rejection: no node passes
        bound, delay = got
        vb: List[List[NodeSelectorTerm]] = []
        vz: List[List[NodeSelectorTerm]] = []
        absent = NodeSelectorTerm([Requirement(k, "DoesNotExist", []) for k in TOPOLOGY_LABELS], [])
        for pv in bound:
            if pv.node_affinity is not None:   # no terms: MatchNodeSelectorTerms matches nothing
                vb.append([_labels_only_term(t) for t in pv.node_affinity] or [_NEVER])
            for k, v in pv.labels.items():
                if k not in TOPOLOGY_LABELS:
                    continue
                zones = label_zones_to_set(v)
                if zones is None:
                    continue                            # getPVbyPod skips a label it cannot parse
                vz.append([NodeSelectorTerm([Requirement(k, "In", zones)], []), absent])
        n_bound = len(vb)
        for pvc in [c for c in delay if c.selected_node]:  # provisioning started on one node
            sc = self.classes.get(self._class_of(pvc))
            known = nodes if nodes is not None else self.nodes
            ok = can_provision(sc) and (known is None or any(
                n.name == pvc.selected_node and topology_ok(sc, n.labels) for n in known))
            vb.append([NodeSelectorTerm([], [Requirement("metadata.name", "In", [pvc.selected_node])])] if ok
                      else [_NEVER])
        delay = [c for c in delay if not c.selected_node]
        if delay:
            cands = [self.candidates(pvc) for pvc in delay]
            names = [{pv.name for pv in c} for c in cands]
            compete = any(names[a] & names[b] for a in range(len(names)) for b in range(a))
            if compete:
                nodes = nodes if nodes is not None else self.nodes
                if nodes is None:
                    raise VolumeUnsupported("claims competing for one PV need the node list")
                ok = [n.name for n in nodes if self.match_on_node(pod, n.labels, n.name) is not None]
                vb.append([NodeSelectorTerm([], [Requirement("metadata.name", "In", [nm])]) for nm in ok] or [_NEVER])
            else:
                for pvc, cs in zip(delay, cands):
                    group: List[NodeSelectorTerm] = []
                    always = False
                    for pv in cs:
                        if pv.node_affinity is None:
                            always = True
                            break
                        group.extend(_labels_only_term(t) for t in pv.node_affinity)
                    sc = self.classes[self._class_of(pvc)]
                    if not always and can_provision(sc):
                        if not sc.allowed_topologies:
                            always = True
                        else:
                            for term in sc.allowed_topologies:
                                if term:
                                    group.append(NodeSelectorTerm([Requirement(k, "In", list(v)) for k, v in term], []))
                    if not always:
                        vb.append(group or [_NEVER])
        return vb, vz, n_bound

    def assume(self, pod: Pod, labels: Dict[str, str], name: Optional[str] = None) -> bool:
        """AssumePodVolumes on the chosen node ``name`` (then PreBind): static
        matches bind their PV.  Claims to provision get the selected-node
        annotation and the pod waits in PreBind (``waiting``; returns False:
        not bound) -- or, with ``provisioning``, a new PV of their size.  The
        pod's claims count as in use."""
        m = self.match_on_node(pod, labels, name)
        bound = True
        if m is not None:
            static, provision = m
            for pvc, pv in static:
                self.bind(pvc, pv)
            for pvc in provision:
                if not self.provisioning:
                    pvc.selected_node = name or pvc.selected_node
                    self.waiting[(pod.namespace, pod.name)] = name or ""
                    bound = False
                    continue
                self.provisioned += 1
                pv_name = f"pvc-provisioned-{self.provisioned}"
                # the provisioner's topology is unknown here: the new PV carries no node affinity
                pv = PersistentVolume(name=pv_name, capacity=pvc.request, storage_class=self._class_of(pvc),
                                      access_modes=list(pvc.access_modes), volume_mode=pvc.volume_mode)
                self.pvs[pv_name] = pv
                self.bind(pvc, pv)
        self.add_users([pod])
        return bound


def _labels_only_term(t: NodeSelectorTerm) -> NodeSelectorTerm:
    """A PV node-affinity term as CheckNodeAffinity evaluates it: the node has
    labels only, so metadata.name is "" (a parse error fails the term)."""
    fields = []
    for r in t.match_fields:
        ok_form = r.key == "metadata.name" and r.operator in ("In", "NotIn") and len(r.values) == 1
        if ok_form and (r.values[0] == "") == (r.operator == "In"):
            fields.append(Requirement("", "__true__", []))
        else:
            fields.append(Requirement("", "__false__", []))
    return NodeSelectorTerm(list(t.match_expressions), fields)
