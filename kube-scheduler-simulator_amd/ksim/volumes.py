"""Bound PersistentVolumeClaims for VolumeBinding and VolumeZone (SURVEY §8(f) 1,
[upstream] k8s.io/kubernetes v1.26.2 pkg/scheduler/framework/plugins/
volumebinding (binder.go checkBoundClaims -> volumeutil.CheckNodeAffinity) and
volumezone (volume_zone.go getPVbyPod / Filter)).

A claim bound to a PV makes both filters depend on node labels only, so the
host turns them into groups of NodeSelectorTerms (ksim_engine.h "Volume
groups"): the node passes a filter iff every group has a matching term.

  VolumeBinding  one group per PV with spec.nodeAffinity.required: its terms.
                 CheckNodeAffinity builds a node with labels only, so a
                 matchFields metadata.name requirement compares with "".
  VolumeZone     one group per PV label whose key is a topology label and whose
                 value parses (LabelZonesToSet: "__"-separated, no empty
                 zone): {key In zones} or {no topology label on the node}.

Supported: claims that exist and are bound to an existing PV whose source no
volume-limit plugin counts (EBS / GCE PD / Azure disk / Cinder are counted by
their in-tree limit plugins; CSI volumes by NodeVolumeLimits when a node
publishes attachable-volumes-* limits) and that is not ReadWriteOncePod
(VolumeRestrictions).  Anything else raises VolumeUnsupported: the pod is
reported and not scheduled (KSIM_POD_HAS_VOLUMES), never mis-scheduled.
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Tuple

from .model import NodeSelectorTerm, PersistentVolume, PersistentVolumeClaim, Pod, Requirement

# volume_zone.go topologyLabels
TOPOLOGY_LABELS = ("failure-domain.beta.kubernetes.io/zone", "failure-domain.beta.kubernetes.io/region",
                   "topology.kubernetes.io/zone", "topology.kubernetes.io/region")
LIMITED_SOURCES = ("awsElasticBlockStore", "gcePersistentDisk", "azureDisk", "cinder")
MSG_VOLUME_BINDING = "node(s) had volume node affinity conflict"    # volumebinding ErrReasonNodeConflict
MSG_VOLUME_ZONE = "node(s) had no available volume zone"            # volumezone ErrReasonConflict


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


class VolumeIndex:
    """The snapshot's PVs and PVCs (ResourcesForImport pvs / pvcs)."""

    def __init__(self, pvs: Iterable[PersistentVolume] = (), pvcs: Iterable[PersistentVolumeClaim] = (),
                 csi_limits: bool = False):
        self.pvs: Dict[str, PersistentVolume] = {pv.name: pv for pv in pvs}
        self.pvcs: Dict[Tuple[str, str], PersistentVolumeClaim] = {(c.namespace, c.name): c for c in pvcs}
        self.csi_limits = csi_limits          # some node publishes attachable-volumes-* allocatable

    @staticmethod
    def from_nodes(nodes, pvs=(), pvcs=()) -> "VolumeIndex":
        lim = any(k.startswith("attachable-volumes-") for n in nodes for k in n.allocatable)
        return VolumeIndex(pvs, pvcs, lim)

    def bound_pvs(self, pod: Pod) -> List[PersistentVolume]:
        out = []
        for claim in pod.pvc_claims:
            pvc = self.pvcs.get((pod.namespace, claim))
            if pvc is None:
                raise VolumeUnsupported(f"persistentvolumeclaim {claim!r} not found")
            if not pvc.volume_name:
                raise VolumeUnsupported(f"persistentvolumeclaim {claim!r} is not bound")
            if "ReadWriteOncePod" in pvc.access_modes:
                raise VolumeUnsupported(f"persistentvolumeclaim {claim!r} is ReadWriteOncePod")
            pv = self.pvs.get(pvc.volume_name)
            if pv is None:
                raise VolumeUnsupported(f"persistentvolume {pvc.volume_name!r} not found")
            if pv.source in LIMITED_SOURCES or (pv.source == "csi" and self.csi_limits):
                raise VolumeUnsupported(f"persistentvolume {pv.name!r}: {pv.source} volumes count against node limits")
            out.append(pv)
        return out

    def groups(self, pod: Pod) -> Tuple[List[List[NodeSelectorTerm]], List[List[NodeSelectorTerm]]]:
        """(VolumeBinding groups, VolumeZone groups) of the pod's bound claims."""
        vb: List[List[NodeSelectorTerm]] = []
        vz: List[List[NodeSelectorTerm]] = []
        absent = NodeSelectorTerm([Requirement(k, "DoesNotExist", []) for k in TOPOLOGY_LABELS], [])
        for pv in self.bound_pvs(pod):
            if pv.node_affinity is not None:   # no terms: MatchNodeSelectorTerms matches nothing
                vb.append([_labels_only_term(t) for t in pv.node_affinity] or [NodeSelectorTerm([], [])])
            for k, v in pv.labels.items():
                if k not in TOPOLOGY_LABELS:
                    continue
                zones = label_zones_to_set(v)
                if zones is None:
                    continue                            # getPVbyPod skips a label it cannot parse
                vz.append([NodeSelectorTerm([Requirement(k, "In", zones)], []), absent])
        return vb, vz


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
