"""Object-level restatement of the scheduling cycle in pure Python (ORACLE).

TEST INFRASTRUCTURE ONLY (like ksim_oracle.c): used by tests/ to pin the C
oracle AND the host encoder (ksim/encode.py, ksim/topology.py) on small
clusters.  It works on the Node / Pod objects with string labels and Go-style
maps, following the structure of the upstream k8s.io/kubernetes v1.26.2
plugins (pinned at simulator/go.mod:53; absent from /root/reference, restated
per SURVEY.md Appendix A and the notes in DESIGN.md), so it shares no code
with the encoder or the C restatement except the Quantity / toleration /
selector helpers of ksim.model and the nodeTree order of ksim.encode.

Pure-Python loops: small cases only (tens of nodes, hundreds of pods).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Tuple

from ksim.encode import node_tree_order, pod_nonzero_requests, pod_requests, zone_key
from ksim.model import (LabelSelector, Node, PersistentVolume, Pod, PodAffinityTerm, Taint, parse_quantity,
                        selector_matches)

MAX_NODE_SCORE = 100
LABEL_HOSTNAME = "kubernetes.io/hostname"
M64 = (1 << 64) - 1
KEY_NODE_MASK = (1 << 18) - 1

# filter failure messages (framework.Status.Message())
PTS_MISSING = "node(s) didn't match pod topology spread constraints (missing required label)"
PTS_SKEW = "node(s) didn't match pod topology spread constraints"
IPA_AFF = "node(s) didn't match pod affinity rules"
IPA_ANTI = "node(s) didn't match pod anti-affinity rules"
IPA_EXIST = "node(s) didn't satisfy existing pods anti-affinity rules"


def splitmix64(x: int) -> int:
    z = (x + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def tb_lo(seed: int, seq: int, node: int) -> int:
    """The tie-break word of selectHost's TB(seed)."""
    h = splitmix64((seed ^ ((seq << 20) & M64) ^ node) & M64) >> 38
    return (h << 18) | (KEY_NODE_MASK - node)


def tb_key(total: int, seed: int, seq: int, node: int) -> tuple:
    """selectHost's order: the max of (total, tie-break word), total a full int64."""
    return (total, tb_lo(seed, seq, node))


def num_feasible_nodes_to_find(pct: int, n: int) -> int:
    if n < 100 or pct >= 100:
        return n
    a = pct if pct > 0 else max(5, 50 - n // 125)
    return max(n * a // 100, 100)


def go_i64(x: int) -> int:
    """Go int64 arithmetic wraps: (capacity - requested) * 100 overflows for
    capacities past 2^56 (leastRequestedScore), and the quotient is of the
    wrapped product."""
    x &= M64
    return x - (1 << 64) if x >> 63 else x


def go_div(a: int, b: int) -> int:
    """Go integer division (truncates toward zero)."""
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


# ---- affinity terms ------------------------------------------------------------
class AffinityTerm:
    """framework.AffinityTerm (newAffinityTerm + getNamespacesFromPodAffinityTerm)."""

    def __init__(self, owner: Pod, t: PodAffinityTerm, weight: int = 0):
        self.namespaces = set(t.namespaces)
        if not t.namespaces and t.namespace_selector is None:
            self.namespaces.add(owner.namespace)
        self.ns_selector: Optional[LabelSelector] = t.namespace_selector
        self.selector: Optional[LabelSelector] = t.label_selector
        self.topology_key = t.topology_key
        self.weight = weight

    def matches(self, pod: Pod, ns_labels: Optional[Dict[str, str]]) -> bool:
        """AffinityTerm.Matches: namespace listed, or the namespace selector
        (nil = Nothing, {} = Everything) matches ns_labels; then the selector."""
        ns_ok = pod.namespace in self.namespaces or selector_matches(self.ns_selector, ns_labels or {})
        return ns_ok and selector_matches(self.selector, pod.labels)


class PodInfo:
    def __init__(self, pod: Pod):
        self.pod = pod
        self.required_affinity = [AffinityTerm(pod, t) for t in pod.pod_affinity_required]
        self.required_anti = [AffinityTerm(pod, t) for t in pod.pod_anti_affinity_required]
        self.preferred_affinity = [AffinityTerm(pod, w.term, w.weight) for w in pod.pod_affinity_preferred]
        self.preferred_anti = [AffinityTerm(pod, w.term, w.weight) for w in pod.pod_anti_affinity_preferred]


class NodeInfo:
    def __init__(self, node: Node):
        self.node = node
        self.alloc = {"cpu": 0, "memory": 0, "ephemeral-storage": 0, "pods": 0}
        from ksim.model import quantity_milli_value, quantity_value
        for k, v in node.allocatable.items():
            self.alloc[k] = quantity_milli_value(v) if k == "cpu" else quantity_value(v)
        self.requested: Dict[str, int] = {}
        self.nz_cpu = 0
        self.nz_mem = 0
        self.pods: List[PodInfo] = []
        self.used_ports: Dict[str, set] = {}     # HostPortInfo: ip -> {(protocol, port)}

    def add_pod(self, pod: Pod) -> None:
        for c in pod.containers:                 # NodeInfo.updateUsedPorts (Spec.Containers)
            for p in c.ports:
                if p.host_port <= 0:
                    continue
                ip, proto = p.host_ip or "0.0.0.0", p.protocol or "TCP"
                self.used_ports.setdefault(ip, set()).add((proto, p.host_port))
        for k, v in pod_requests(pod).items():
            self.requested[k] = self.requested.get(k, 0) + v
        c, m = pod_nonzero_requests(pod)
        self.nz_cpu += c
        self.nz_mem += m
        self.pods.append(PodInfo(pod))

    def save(self):
        return (dict(self.requested), self.nz_cpu, self.nz_mem, len(self.pods),
                {k: set(v) for k, v in self.used_ports.items()})

    def restore(self, saved) -> None:
        """Undo add_pod calls made after save() (addNominatedPods works on a clone)."""
        self.requested, self.nz_cpu, self.nz_mem, n, self.used_ports = saved
        del self.pods[n:]


class ObjScheduler:
    """One simulated scheduler (sequential semantics, TB tie-break)."""

    def __init__(self, nodes: List[Node], bound: List[Pod] = (), namespaces: Optional[Dict[str, Dict]] = None,
                 pct: int = 0, weights: Optional[Dict[str, int]] = None, seed: int = 0x4B53494D,
                 hard_pod_affinity_weight: int = 1, network_bandwidth=None, nb_filter: bool = True,
                 nb_score: bool = True, pvs=(), pvcs=(), storage_classes=(), fit=None, node_affinity=None,
                 preemption=None, spread=None, services=(), controllers=(), provisioning: bool = False):
        """fit / node_affinity / preemption / spread: ksim.profile FitArgs,
        NodeAffinityArgs, PreemptionArgs, PodTopologySpreadArgs (the plugin args of
        the profile; None = the defaults).  services / controllers: the
        ksim.model Service / Controller objects helper.DefaultSelector reads."""
        order = node_tree_order([zone_key(n.labels) for n in nodes])
        self.nodes = [NodeInfo(nodes[i]) for i in order]
        # cache.addNodeImageStates, nodes in the order they were added: name -> [size, {node names}]
        self.image_states: Dict[str, list] = {}
        for n in nodes:
            for names, size in n.images:
                for name in names:
                    self.image_states.setdefault(name, [int(size), set()])[1].add(n.name)
        self.by_name = {ni.node.name: ni for ni in self.nodes}
        for p in bound:
            if p.node_name in self.by_name:
                self.by_name[p.node_name].add_pod(p)
        self.ns_labels = dict(namespaces or {})
        self.pct = pct
        self.weights = weights or {"NodeResourcesBalancedAllocation": 1, "ImageLocality": 1, "InterPodAffinity": 1,
                                   "NodeResourcesFit": 1, "NodeAffinity": 1, "PodTopologySpread": 2,
                                   "TaintToleration": 1}
        self.score_order = ["NodeResourcesBalancedAllocation", "ImageLocality", "InterPodAffinity",
                            "NodeResourcesFit", "NodeAffinity", "PodTopologySpread", "TaintToleration"]
        self.filter_order = ["NodeUnschedulable", "NodeName", "TaintToleration", "NodeAffinity", "NodePorts",
                             "NodeResourcesFit", "VolumeRestrictions", "EBSLimits", "GCEPDLimits",
                             "NodeVolumeLimits", "AzureDiskLimits", "VolumeBinding", "VolumeZone",
                             "PodTopologySpread", "InterPodAffinity"]
        # NetworkBandwidth (out-of-tree, enabled by a profile): appended after the
        # in-tree plugins, as mergePluginSet places a user-enabled plugin
        self.nb = network_bandwidth
        if self.nb is not None:
            if nb_filter:
                self.filter_order.append("NetworkBandwidth")
            if nb_score:
                self.score_order.append("NetworkBandwidth")
        self.seed = seed
        self.hard_w = hard_pod_affinity_weight
        from ksim.profile import FitArgs, NodeAffinityArgs, PreemptionArgs, is_extended_resource_name
        self.fit = fit or FitArgs()
        rw: Dict[str, int] = {}
        for r, w in self.fit.resources:            # resourcesToWeightMap
            rw.pop(r, None)
            rw[r] = w
        self.fit_weights = rw
        self.is_extended = is_extended_resource_name
        self.added = node_affinity or NodeAffinityArgs()
        self.preemption = preemption or PreemptionArgs()
        from ksim.profile import PodTopologySpreadArgs
        self.spread = spread or PodTopologySpreadArgs()
        self.services = list(services)
        self.controllers = list(controllers)
        # the snapshot's PersistentVolumes, PersistentVolumeClaims and StorageClasses
        # (VolumeBinding / VolumeZone / VolumeRestrictions); copies, bound as the run goes
        import copy
        self.pvs = {pv.name: copy.deepcopy(pv) for pv in pvs}
        self.pvcs = {(c.namespace, c.name): copy.deepcopy(c) for c in pvcs}
        self.classes = {c.name: c for c in storage_classes}
        self.claim_users: Dict[Tuple[str, str], int] = {}
        for p in bound:
            for claim in p.pvc_claims:
                self.claim_users[(p.namespace, claim)] = self.claim_users.get((p.namespace, claim), 0) + 1
        self.provisioned = 0
        self.provisioning = provisioning             # a provisioner acts (the simulator runs none)
        self._pv_controller()
        self.next_start = 0
        self.seq = 0

    # ---- NodeAffinity / taints (component-helpers, v1helper) -------------------
    @staticmethod
    def _req_match(r, labels: Dict[str, str]) -> bool:
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

    def _term_match(self, t, node: Node) -> bool:
        if not t.match_expressions and not t.match_fields:
            return False
        for r in t.match_expressions:
            if not self._req_match(r, node.labels):
                return False
        for r in t.match_fields:
            if r.key != "metadata.name" or r.operator not in ("In", "NotIn") or len(r.values) != 1:
                return False
            if (node.name in r.values) != (r.operator == "In"):
                return False
        return True

    def node_affinity_filter(self, pod: Pod, node: Node) -> Optional[str]:
        """nodeaffinity.Filter: addedNodeSelector first (errReasonEnforced), then the pod's."""
        if self.added.required is not None and not any(self._term_match(t, node) for t in self.added.required):
            return "node(s) didn't match scheduler-enforced node affinity"
        if not self.required_node_affinity(pod, node):
            return "node(s) didn't match Pod's node affinity/selector"
        return None

    def required_node_affinity(self, pod: Pod, node: Node) -> bool:
        for k, v in pod.node_selector.items():
            if node.labels.get(k) != v:
                return False
        if pod.required_terms is not None:
            return any(self._term_match(t, node) for t in pod.required_terms)
        return True

    # ---- VolumeBinding / VolumeZone for bound claims (v1.26) ---------------------
    TOPOLOGY_LABELS = ("failure-domain.beta.kubernetes.io/zone", "failure-domain.beta.kubernetes.io/region",
                       "topology.kubernetes.io/zone", "topology.kubernetes.io/region")

    def _bound_pvs(self, pod: Pod):
        out = []
        for c in pod.pvc_claims:
            pvc = self.pvcs[(pod.namespace, c)]
            if pvc.volume_name:
                out.append(self.pvs[pvc.volume_name])
        return out

    # ---- unbound claims: the PV controller and the volume binder (v1.26) -----------
    def _find_matching_volume(self, pvc, labels: Optional[Dict[str, str]], excluded, delay: bool):
        """pv/util FindMatchingVolume over the PVs in name order (upstream: the
        cache's order); labels None: the PV controller's call (node nil)."""
        key = (pvc.namespace, pvc.name)
        best = None
        for name in sorted(self.pvs):
            pv = self.pvs[name]
            if name in excluded:
                continue
            if pv.claim_ref is not None and pv.claim_ref != key:
                continue
            if pv.capacity < pvc.request or pv.volume_mode != pvc.volume_mode or pv.deleting:
                continue
            if labels is None and not set(pvc.access_modes) <= set(pv.access_modes):
                continue                              # the controller's index by access modes
            aff = labels is None or self._pv_affinity(pv, labels)
            if pv.claim_ref == key:
                return pv if aff else None
            if labels is None and delay:
                continue
            if pvc.selector is not None and not selector_matches(pvc.selector, pv.labels):
                continue
            if pv.storage_class != (pvc.storage_class or "") or not aff:
                continue
            if labels is not None and not set(pvc.access_modes) <= set(pv.access_modes):
                continue
            if best is None or pv.capacity < best.capacity:
                best = pv
        return best

    def _pv_affinity(self, pv, labels: Dict[str, str]) -> bool:
        if pv.node_affinity is None:
            return True
        labels_only = Node(name="", labels=labels)
        return any(self._term_match(t, labels_only) for t in pv.node_affinity)

    def _delay(self, pvc) -> bool:
        """IsDelayBindingMode: a class that does not exist is NotFound, not an
        error, so such a claim is Immediate."""
        sc = self.classes.get(pvc.storage_class or "")
        return sc is not None and sc.volume_binding_mode == "WaitForFirstConsumer"

    def _pv_controller(self) -> None:
        for pvc in self.pvcs.values():               # syncClaim of a claim naming its PV
            pv = self.pvs.get(pvc.volume_name) if pvc.volume_name else None
            if pv is not None and pv.claim_ref is None:
                pv.claim_ref = (pvc.namespace, pvc.name)
        for pvc in self.pvcs.values():
            if pvc.volume_name or self._delay(pvc):
                continue
            pv = self._find_matching_volume(pvc, None, set(), False)
            if pv is not None:
                pv.claim_ref, pvc.volume_name = (pvc.namespace, pvc.name), pv.name

    def volume_prefilter(self, pod: Pod) -> Optional[str]:
        """VolumeBinding PreFilter (VolumeRestrictions' ReadWriteOncePod check is
        behind a feature gate that is off in v1.26)."""
        immediate = False
        for claim in pod.pvc_claims:
            pvc = self.pvcs.get((pod.namespace, claim))
            if pvc is None:
                return f'persistentvolumeclaim "{claim}" not found'
            if not pvc.volume_name:
                immediate = immediate or not self._delay(pvc)
        return "pod has unbound immediate PersistentVolumeClaims" if immediate else None

    def find_pod_volumes(self, pod: Pod, node: Node):
        """binder.go FindPodVolumes for the unbound WaitForFirstConsumer claims:
        (static [(pvc, pv)], to provision [pvc]) or None (ErrReasonBindConflict)."""
        delay = [self.pvcs[(pod.namespace, c)] for c in pod.pvc_claims if not self.pvcs[(pod.namespace, c)].volume_name]
        chosen, static, provision = set(), [], []
        for pvc in delay:                              # AnnSelectedNode: provisioning started there
            if pvc.selected_node:
                if pvc.selected_node != node.name:
                    return None
                provision.append(pvc)
        delay = sorted((c for c in delay if not c.selected_node), key=lambda c: c.request)
        for pvc in delay:
            pv = self._find_matching_volume(pvc, node.labels, chosen, True)
            if pv is None:
                provision.append(pvc)
            else:
                chosen.add(pv.name)
                static.append((pvc, pv))
        for pvc in provision:                          # checkVolumeProvisions
            sc = self.classes[pvc.storage_class or ""]
            if sc.provisioner in ("", "kubernetes.io/no-provisioner"):
                return None
            if sc.allowed_topologies and not any(
                    term and all(vals and node.labels.get(k) in vals for k, vals in term)
                    for term in sc.allowed_topologies):
                return None
        return static, provision

    def assume_volumes(self, pod: Pod, node: Node) -> None:
        got = self.find_pod_volumes(pod, node)
        if got is not None:
            static, provision = got
            for pvc, pv in static:
                pv.claim_ref, pvc.volume_name = (pvc.namespace, pvc.name), pv.name
            for pvc in provision:
                if not self.provisioning:              # no provisioner: the claim waits on its node
                    pvc.selected_node = node.name
                    continue
                self.provisioned += 1
                pv = PersistentVolume(name=f"pvc-provisioned-{self.provisioned}", capacity=pvc.request,
                                      storage_class=pvc.storage_class or "", access_modes=list(pvc.access_modes),
                                      volume_mode=pvc.volume_mode, claim_ref=(pvc.namespace, pvc.name))
                self.pvs[pv.name] = pv
                pvc.volume_name = pv.name
        for claim in pod.pvc_claims:
            self.claim_users[(pod.namespace, claim)] = self.claim_users.get((pod.namespace, claim), 0) + 1

    def volume_binding_ok(self, pod: Pod, node: Node) -> bool:
        """binder.go checkBoundClaims: volumeutil.CheckNodeAffinity(pv, node.Labels)
        for every bound claim; the node it builds carries labels only."""
        labels_only = Node(name="", labels=node.labels)
        for pv in self._bound_pvs(pod):
            if pv.node_affinity is None:
                continue
            if not any(self._term_match(t, labels_only) for t in pv.node_affinity):
                return False
        return True

    def volume_zone_ok(self, pod: Pod, node: Node) -> bool:
        """volume_zone.go getPVbyPod + Filter."""
        tops = []
        for pv in self._bound_pvs(pod):
            for k, v in pv.labels.items():
                if k not in self.TOPOLOGY_LABELS:
                    continue
                zones = [z.strip() for z in v.split("__")]
                if any(not z for z in zones):
                    continue                      # LabelZonesToSet error: the label is ignored
                tops.append((k, set(zones)))
        if not any(k in node.labels for k in self.TOPOLOGY_LABELS):
            return True                           # the node has no zone constraints
        return all(k in node.labels and node.labels[k] in zs for k, zs in tops)

    @staticmethod
    def untolerated_taint(pod: Pod, node: Node, effects=("NoSchedule", "NoExecute")):
        for t in node.taints:
            if t.effect in effects and not any(tol.tolerates(t) for tol in pod.tolerations):
                return t
        return None

    # ---- PodTopologySpread (filtering.go / scoring.go) ---------------------------
    def _default_selector(self, pod: Pod) -> Optional[LabelSelector]:
        """helper.DefaultSelector: the Services selecting the pod (merged label
        maps), then its controller's selector (an RC's map merged in, a
        ReplicaSet's / StatefulSet's requirements added); None when Empty()."""
        merged: Dict[str, str] = {}
        for svc in self.services:
            if svc.namespace != pod.namespace or svc.selector is None:
                continue
            if LabelSelector(dict(svc.selector)).matches(pod.labels):
                merged.update(svc.selector)
        reqs = []
        if pod.owner is not None:
            api, kind, name = pod.owner
            gvk = {("v1", "ReplicationController"), ("apps/v1", "ReplicaSet"), ("apps/v1", "StatefulSet")}
            if (api, kind) in gvk:
                for ctl in self.controllers:
                    if ctl.kind == kind and ctl.namespace == pod.namespace and ctl.name == name:
                        if kind == "ReplicationController":
                            merged.update(ctl.selector or {})
                        elif ctl.selector is not None:
                            from ksim.model import Requirement
                            reqs += [Requirement(k, "In", [v]) for k, v in ctl.selector.match_labels.items()]
                            reqs += list(ctl.selector.match_expressions)
                        break
        if not merged and not reqs:
            return None
        return LabelSelector(merged, reqs)

    def _pod_constraints(self, pod: Pod):
        """(constraints, system-defaulted): the pod's own, else buildDefaultConstraints."""
        if pod.topology_spread:
            return list(pod.topology_spread), False
        import dataclasses
        sel = self._default_selector(pod)
        cons = self.spread.constraints()
        if sel is None or not cons:
            return [], False
        return [dataclasses.replace(c, label_selector=sel) for c in cons], self.spread.defaulting_type == "System"

    def _constraints(self, pod: Pod, when: str):
        return [c for c in self._pod_constraints(pod)[0] if c.when_unsatisfiable == when]

    @staticmethod
    def _count_match(ni: NodeInfo, sel: Optional[LabelSelector], ns: str) -> int:
        if sel is None or sel.empty():          # Nothing / selector.Empty() -> 0
            return 0
        return sum(1 for pi in ni.pods if pi.pod.namespace == ns and sel.matches(pi.pod.labels))

    def _inclusion(self, c, pod: Pod, node: Node) -> bool:
        if (c.node_affinity_policy or "Honor") == "Honor" and not self.required_node_affinity(pod, node):
            return False
        if (c.node_taints_policy or "Ignore") == "Honor" and self.untolerated_taint(pod, node) is not None:
            return False
        return True

    def pts_prefilter(self, pod: Pod):
        cons = self._constraints(pod, "DoNotSchedule")
        pair_num: Dict[Tuple[str, str], int] = {}
        for ni in self.nodes:
            node = ni.node
            if not all(c.topology_key in node.labels for c in cons):
                continue
            tp: Dict[Tuple[str, str], int] = {}
            for c in cons:
                if not self._inclusion(c, pod, node):
                    continue
                tp[(c.topology_key, node.labels[c.topology_key])] = self._count_match(ni, c.label_selector,
                                                                                      pod.namespace)
            for k, v in tp.items():
                pair_num[k] = pair_num.get(k, 0) + v
        crit = {c.topology_key: 2 ** 31 - 1 for c in cons}
        for (k, v), num in pair_num.items():
            crit[k] = min(crit[k], num)
        return cons, pair_num, crit

    def pts_filter(self, pod: Pod, state, node: Node) -> Optional[str]:
        cons, pair_num, crit = state
        for c in cons:
            if c.topology_key not in node.labels:
                return PTS_MISSING
            self_match = 1 if selector_matches(c.label_selector, pod.labels) else 0
            match = pair_num.get((c.topology_key, node.labels[c.topology_key]), 0)
            if match + self_match - crit[c.topology_key] > c.max_skew:
                return PTS_SKEW
        return None

    def pts_prescore(self, pod: Pod, filtered: List[NodeInfo]):
        cons = self._constraints(pod, "ScheduleAnyway")
        # requireAllTopologies = len(pod.Spec.TopologySpreadConstraints) > 0 || !systemDefaulted
        require_all = bool(pod.topology_spread) or self.spread.defaulting_type != "System"
        ignored = set()
        pair_counts: Dict[Tuple[str, str], int] = {}
        weights = []
        if not cons:
            return cons, ignored, pair_counts, weights
        topo_size = [0] * len(cons)
        for ni in filtered:
            node = ni.node
            if require_all and not all(c.topology_key in node.labels for c in cons):
                ignored.add(node.name)
                continue
            for i, c in enumerate(cons):
                if c.topology_key == LABEL_HOSTNAME:
                    continue
                pair = (c.topology_key, node.labels.get(c.topology_key, ""))
                if pair not in pair_counts:
                    pair_counts[pair] = 0
                    topo_size[i] += 1
        for i, c in enumerate(cons):
            sz = topo_size[i]
            if c.topology_key == LABEL_HOSTNAME:
                sz = len(filtered) - len(ignored)
            weights.append(math.log(float(sz + 2)))
        for ni in self.nodes:
            node = ni.node
            if require_all and not all(c.topology_key in node.labels for c in cons):
                continue
            for c in cons:
                if not self._inclusion(c, pod, node):
                    continue
                pair = (c.topology_key, node.labels.get(c.topology_key, ""))
                if pair not in pair_counts:
                    continue
                pair_counts[pair] += self._count_match(ni, c.label_selector, pod.namespace)
        return cons, ignored, pair_counts, weights

    def pts_score(self, pod: Pod, state, ni: NodeInfo) -> int:
        cons, ignored, pair_counts, weights = state
        if ni.node.name in ignored:
            return 0
        score = 0.0
        for i, c in enumerate(cons):
            if c.topology_key in ni.node.labels:
                if c.topology_key == LABEL_HOSTNAME:
                    cnt = self._count_match(ni, c.label_selector, pod.namespace)
                else:
                    cnt = pair_counts[(c.topology_key, ni.node.labels[c.topology_key])]
                score += float(cnt) * weights[i] + float(c.max_skew - 1)
        return int(math.floor(score + 0.5)) if score >= 0 else -int(math.floor(-score + 0.5))

    @staticmethod
    def pts_normalize(state, names: List[str], scores: List[int]) -> List[int]:
        _, ignored, _, _ = state
        mn, mx = 2 ** 63 - 1, 0
        for n, s in zip(names, scores):
            if n in ignored:
                continue
            mn, mx = min(mn, s), max(mx, s)
        out = []
        for n, s in zip(names, scores):
            if n in ignored:
                out.append(0)
            elif mx == 0:
                out.append(MAX_NODE_SCORE)
            else:
                out.append(go_div(MAX_NODE_SCORE * (mx + mn - s), mx))
        return out

    # ---- InterPodAffinity (filtering.go / scoring.go) ----------------------------
    def _nslabels(self, ns: str) -> Dict[str, str]:
        return self.ns_labels.get(ns, {})

    def _merge_ns(self, t: AffinityTerm) -> AffinityTerm:
        """mergeAffinityTermNamespacesIfNotEmpty (incoming pod's terms)."""
        if t.ns_selector is None or t.ns_selector.empty():
            return t
        import copy
        t = copy.copy(t)
        t.namespaces = set(t.namespaces) | {n for n, lab in self.ns_labels.items() if t.ns_selector.matches(lab)}
        t.ns_selector = None                     # labels.Nothing()
        return t

    def ipa_prefilter(self, pod: Pod):
        info = PodInfo(pod)
        req_aff = [self._merge_ns(t) for t in info.required_affinity]
        req_anti = [self._merge_ns(t) for t in info.required_anti]
        ns_labels = self._nslabels(pod.namespace)
        existing: Dict[Tuple[str, str], int] = {}
        for ni in self.nodes:
            for epi in ni.pods:
                for t in epi.required_anti:
                    if t.matches(pod, ns_labels) and t.topology_key in ni.node.labels:
                        pair = (t.topology_key, ni.node.labels[t.topology_key])
                        existing[pair] = existing.get(pair, 0) + 1
        aff: Dict[Tuple[str, str], int] = {}
        anti: Dict[Tuple[str, str], int] = {}
        for ni in self.nodes:
            for epi in ni.pods:
                if req_aff and all(t.matches(epi.pod, None) for t in req_aff):
                    for t in req_aff:
                        if t.topology_key in ni.node.labels:
                            pair = (t.topology_key, ni.node.labels[t.topology_key])
                            aff[pair] = aff.get(pair, 0) + 1
                for t in req_anti:
                    if t.matches(epi.pod, None) and t.topology_key in ni.node.labels:
                        pair = (t.topology_key, ni.node.labels[t.topology_key])
                        anti[pair] = anti.get(pair, 0) + 1
        self_match = bool(req_aff) and all(t.matches(pod, None) for t in req_aff)
        return req_aff, req_anti, existing, aff, anti, self_match

    @staticmethod
    def ipa_filter(state, node: Node) -> Optional[str]:
        req_aff, req_anti, existing, aff, anti, self_match = state
        pods_exist = True
        for t in req_aff:
            if t.topology_key in node.labels:
                if aff.get((t.topology_key, node.labels[t.topology_key]), 0) <= 0:
                    pods_exist = False
            else:
                return IPA_AFF
        if not pods_exist and not (len(aff) == 0 and self_match):
            return IPA_AFF
        if anti:
            for t in req_anti:
                if t.topology_key in node.labels and anti.get((t.topology_key, node.labels[t.topology_key]), 0) > 0:
                    return IPA_ANTI
        if existing:
            for k, v in node.labels.items():
                if existing.get((k, v), 0) > 0:
                    return IPA_EXIST
        return None

    def ipa_prescore(self, pod: Pod) -> Dict[str, Dict[str, int]]:
        info = PodInfo(pod)
        pref_aff = [self._merge_ns(t) for t in info.preferred_affinity]
        pref_anti = [self._merge_ns(t) for t in info.preferred_anti]
        ns_labels = self._nslabels(pod.namespace)
        topo: Dict[str, Dict[str, int]] = {}

        def process(t: AffinityTerm, weight: int, target: Pod, nsl, node: Node, mult: int):
            if t.matches(target, nsl) and t.topology_key in node.labels:
                d = topo.setdefault(t.topology_key, {})
                v = node.labels[t.topology_key]
                d[v] = d.get(v, 0) + weight * mult

        for ni in self.nodes:
            node = ni.node
            for epi in ni.pods:
                if not node.labels:
                    continue
                for t in pref_aff:
                    process(t, t.weight, epi.pod, None, node, 1)
                for t in pref_anti:
                    process(t, t.weight, epi.pod, None, node, -1)
                if self.hard_w > 0:
                    for t in epi.required_affinity:
                        process(t, self.hard_w, pod, ns_labels, node, 1)
                for t in epi.preferred_affinity:
                    process(t, t.weight, pod, ns_labels, node, 1)
                for t in epi.preferred_anti:
                    process(t, t.weight, pod, ns_labels, node, -1)
        return topo

    @staticmethod
    def ipa_score(topo, node: Node) -> int:
        s = 0
        for k, vals in topo.items():
            if k in node.labels:
                s += vals.get(node.labels[k], 0)
        return s

    @staticmethod
    def ipa_normalize(topo, scores: List[int]) -> List[int]:
        if not topo:
            return list(scores)
        mn, mx = min(scores), max(scores)
        d = mx - mn
        return [int(float(MAX_NODE_SCORE) * (float(s - mn) / float(d))) if d > 0 else 0 for s in scores]

    # ---- NetworkBandwidth (simulator/scheduler/plugin/networkbandwidth/plugin.go) ------
    # Exact quantities (Fractions); the node's allocated amount is summed from the
    # pods on it each time, as getNodeAllocatedAmount does.
    @staticmethod
    def _q(s):
        try:
            return parse_quantity(s)
        except ValueError:
            return None

    def _nb_allocated(self, ni: NodeInfo):
        a = self.nb
        total = 0
        for key in (a.ingress_request_annotation, a.egress_request_annotation):   # :107-120
            for pi in ni.pods:
                if key in pi.pod.annotations:
                    q = self._q(pi.pod.annotations[key])
                    if q is not None:
                        total += q
        return total

    def nb_filter(self, pod: Pod, ni: NodeInfo):
        """(status, message): status None (Success), "unschedulable", "skip" or "error"."""
        a, node = self.nb, ni.node
        if a.node_limit_annotation not in node.annotations:
            return "skip", f"Node {node.name} does not have {a.node_limit_annotation} annotation present"
        limit = self._q(node.annotations[a.node_limit_annotation])
        if limit is None:
            return "error", f"Node {node.name} has an incorrect quantity in {a.node_limit_annotation} annotation present"
        allocated = self._nb_allocated(ni)
        req = 0
        for key, fallback in ((a.ingress_request_annotation, "kubernetes.io/ingress-bandwidth"),
                              (a.egress_request_annotation, "kubernetes.io/egress-bandwidth")):
            s = pod.annotations.get(key)
            if s is None:
                s = pod.annotations.get(fallback)
            if s is not None:
                q = self._q(s)
                if q is None:
                    return "error", f"Could not parse quantity from pod {pod.name} {key} annotations"
                req += q
        if req == 0:
            return "skip", (f"Pod {pod.name} does not have network bandwidth request annotations set. "
                            f"(Missing {a.ingress_request_annotation} or {a.egress_request_annotation})")
        if allocated + req > limit:
            return "unschedulable", f"Node {node.name} does not have enough network bandwidth capacity to schedule pod"
        return None, None

    def nb_score(self, ni: NodeInfo) -> Optional[int]:
        """Score's value, or None when it returns Skip / Error."""
        a, node = self.nb, ni.node
        if a.node_limit_annotation not in node.annotations:
            return None
        limit = self._q(node.annotations[a.node_limit_annotation])
        if limit is None:
            return None
        d = limit - self._nb_allocated(ni)
        return math.ceil(d) if d >= 0 else -math.ceil(-d)     # Quantity.Value(): away from zero

    @staticmethod
    def nb_normalize(scores: List[int]) -> List[int]:
        mn, mx = min(scores), max(scores)
        d = mx - mn
        return [int(float(MAX_NODE_SCORE) * (float(s - mn) / float(d))) if d > 0 else 0 for s in scores]

    # ---- resources -------------------------------------------------------------------
    def fit_filter(self, pod: Pod, ni: NodeInfo, scalar_order=None) -> Optional[str]:
        """fitsRequest; scalar reasons follow ``scalar_order`` (Go appends them in
        map order; the C restatement in column order)."""
        req = pod_requests(pod)
        reasons = []
        if len(ni.pods) + 1 > ni.alloc.get("pods", 0):
            reasons.append("Too many pods")
        native = ("cpu", "memory", "ephemeral-storage")
        if any(v for v in req.values()) or any(k not in native for k in req):
            for r in native:
                if req.get(r, 0) > ni.alloc.get(r, 0) - ni.requested.get(r, 0):
                    reasons.append(f"Insufficient {r}")
            scal = [k for k in req if k not in native]
            if scalar_order is not None:
                scal.sort(key=lambda k: scalar_order.index(k) if k in scalar_order else len(scalar_order))
            for r in scal:
                q = req[r]
                if q == 0:
                    continue
                if self.is_extended(r) and (r in self.fit.ignored_resources or
                                            r.split("/")[0] in self.fit.ignored_resource_groups):
                    continue                       # ignoredResources / ignoredResourceGroups
                if q > ni.alloc.get(r, 0) - ni.requested.get(r, 0):
                    reasons.append(f"Insufficient {r}")
        return ", ".join(reasons) if reasons else None

    def _alloc_req(self, pod: Pod, ni: NodeInfo, r: str, use_requested: bool):
        """calculateResourceAllocatableRequest (+ calculatePodResourceRequest)."""
        req = pod_requests(pod)
        if r in ("cpu", "memory") and not use_requested:
            ncpu, nmem = pod_nonzero_requests(pod)
            pr = ncpu if r == "cpu" else nmem
            have = ni.nz_cpu if r == "cpu" else ni.nz_mem
            return ni.alloc.get(r, 0), have + pr
        pr = req.get(r, 0)
        if r in ("cpu", "memory", "ephemeral-storage"):
            return ni.alloc.get(r, 0), ni.requested.get(r, 0) + pr
        if pr == 0:                                # an extended resource the pod does not request
            return 0, 0
        if r in ni.alloc:
            return ni.alloc[r], ni.requested.get(r, 0) + pr
        return 0, 0

    def _broken_linear(self, p: int) -> int:
        shape = [(u, sc * 10) for u, sc in self.fit.shape]
        for i, (u, sc) in enumerate(shape):
            if p <= u:
                if i == 0:
                    return sc
                pu, ps = shape[i - 1]
                return ps + go_div((sc - ps) * (p - pu), u - pu)
        return shape[-1][1]

    def least_allocated(self, pod: Pod, ni: NodeInfo) -> int:
        """NodeResourcesFit.Score under the profile's scoring strategy (the name
        keeps the default's)."""
        score = wsum = 0
        strat = self.fit.strategy
        for r, w in self.fit_weights.items():
            alloc, req = self._alloc_req(pod, ni, r, False)
            if alloc == 0:
                continue
            if strat == "MostAllocated":
                s = go_div(go_i64(min(req, alloc) * MAX_NODE_SCORE), alloc)
            elif strat == "RequestedToCapacityRatio":
                s = self._broken_linear(100 if req > alloc else go_div(go_i64(req * 100), alloc))
                if s <= 0:
                    continue
            else:
                s = 0 if req > alloc else go_div(go_i64((alloc - req) * MAX_NODE_SCORE), alloc)
            score += s * w
            wsum += w
        if not wsum:
            return 0
        if strat == "RequestedToCapacityRatio":
            x = float(score) / float(wsum)
            return int(math.floor(x + 0.5)) if x >= 0 else -int(math.floor(-x + 0.5))   # math.Round
        return go_div(score, wsum)

    @staticmethod
    def balanced(pod: Pod, ni: NodeInfo) -> int:
        req = pod_requests(pod)
        fr = []
        for r in ("cpu", "memory"):
            a = ni.alloc[r]
            if a == 0:
                continue
            f = float(ni.requested.get(r, 0) + req.get(r, 0)) / float(a)
            fr.append(1.0 if f > 1 else f)
        std = abs((fr[0] - fr[1]) / 2) if len(fr) == 2 else 0.0
        return int((1 - std) * MAX_NODE_SCORE)

    @staticmethod
    def default_normalize(scores: List[int], reverse: bool) -> List[int]:
        m = max([0] + scores)
        if m == 0:
            return [MAX_NODE_SCORE] * len(scores) if reverse else list(scores)
        out = [go_div(MAX_NODE_SCORE * s, m) for s in scores]
        return [MAX_NODE_SCORE - s for s in out] if reverse else out

    # ---- DefaultPreemption (preemption.go / default_preemption.go) -------------------
    def preempt(self, pod: Pod, priority: int, start_time: Dict[str, int], order: Dict[str, int],
                nominated=None):
        """PostFilter for an unschedulable pod, deterministic (offset 0, candidates
        in nodeTree order).  start_time / order: per bound pod name (order breaks
        MoreImportantPod ties).  ``nominated``: the PodNominator as in cycle();
        SelectVictimsOnNode's filter runs RunFilterPluginsWithNominatedPods, so
        the nominated pods of priority >= the pod's stay on the node (pass 1;
        pass 2 without them passes whenever pass 1 does for Fit).  Returns
        (nominated node name or None, victim names)."""
        pts, ipa = self.pts_prefilter(pod), self.ipa_prefilter(pod)
        potential = [ni for ni in self.nodes
                     if self.filter_with_nominated(pod, ni, pts, ipa, nominated)[0] == "NodeResourcesFit"]
        pa = self.preemption
        want = min(max(len(potential) * pa.min_candidate_nodes_percentage // 100, pa.min_candidate_nodes_absolute),
                   len(potential))
        want_req = pod_requests(pod)
        nothing = not any(want_req.values())

        def fits(ni, req, npods):
            if npods + 1 > ni.alloc.get("pods", 0):
                return False
            if nothing:
                return True
            return all(want_req.get(r, 0) <= ni.alloc.get(r, 0) - req.get(r, 0)
                       for r in set(want_req) | {"cpu", "memory", "ephemeral-storage"} if want_req.get(r, 0))

        def select_victims(ni):
            lower = [pi.pod for pi in ni.pods if pi.pod.priority < priority]
            lower.sort(key=lambda q: (-q.priority, start_time[q.name], order[q.name]))   # MoreImportantPod
            req = dict(ni.requested)
            n = len(ni.pods) - len(lower)
            for q in self._nominated_for(pod, ni, nominated):
                for k, v in pod_requests(q).items():
                    req[k] = req.get(k, 0) + v
                n += 1
            for q in lower:
                for k, v in pod_requests(q).items():
                    req[k] = req.get(k, 0) - v
            if not fits(ni, req, n):
                return None
            victims = []
            for q in lower:                        # reprievePod
                qr = pod_requests(q)
                for k, v in qr.items():
                    req[k] = req.get(k, 0) + v
                n += 1
                if not fits(ni, req, n):
                    for k, v in qr.items():
                        req[k] -= v
                    n -= 1
                    victims.append(q)
            return victims

        cands = []
        for ni in potential:
            if len(cands) >= want:
                break
            v = select_victims(ni)
            if v is not None:
                cands.append((ni, v))
        if not cands:
            return None, []

        def criteria(c):                           # pickOneNodeForPreemption (no PDBs)
            v = c[1]
            high = v[0].priority if v else -(2 ** 31)
            total = sum(q.priority + 2 ** 31 for q in v)
            early = min((start_time[q.name] for q in v if q.priority == high), default=2 ** 63)
            return (high, total, len(v), -early)
        best = min(range(len(cands)), key=lambda i: (criteria(cands[i]), i))
        return cands[best][0].node.name, [q.name for q in cands[best][1]]

    # ---- ImageLocality (imagelocality.Score) ----------------------------------------
    def image_locality(self, pod: Pod, node: Node) -> int:
        mb = 1024 * 1024
        min_t, max_t = 23 * mb, 1000 * mb * len(pod.containers)
        total_nodes = len(self.nodes)
        have = {nm for names, _ in node.images for nm in names}
        s = 0
        for c in pod.containers:                  # sumImageScores
            name = c.image
            if name.rfind(":") <= name.rfind("/"):
                name += ":latest"                 # normalizedImageName
            if name in have:
                size, on = self.image_states[name]
                spread = float(len(on)) / float(total_nodes)
                s += int(float(size) * spread)    # scaledImageScore
        if s < min_t:                             # calculatePriority
            s = min_t
        elif s > max_t:
            s = max_t
        return go_div(MAX_NODE_SCORE * (s - min_t), max_t - min_t)

    # ---- NodePorts (nodeports.fitsPorts, HostPortInfo.CheckConflict) -----------------
    @staticmethod
    def fits_ports(pod: Pod, ni: NodeInfo) -> bool:
        for c in pod.containers:                 # getContainerPorts
            for p in c.ports:
                if p.host_port <= 0:
                    continue
                ip, pp = p.host_ip or "0.0.0.0", (p.protocol or "TCP", p.host_port)
                if ip == "0.0.0.0":
                    if any(pp in m for m in ni.used_ports.values()):
                        return False
                elif any(pp in ni.used_ports.get(k, ()) for k in ("0.0.0.0", ip)):
                    return False
        return True

    # ---- the cycle ---------------------------------------------------------------------
    def filter_node(self, pod: Pod, ni: NodeInfo, pts, ipa) -> Tuple[Optional[str], Optional[str]]:
        """(failing plugin, message); the plugin is "NetworkBandwidth!" when its
        status was Skip / Error (RunFilterPlugins: framework.Error)."""
        node = ni.node
        for pl in self.filter_order:
            msg = None
            if pl == "NetworkBandwidth":
                st, msg = self.nb_filter(pod, ni)
                if st in ("skip", "error"):
                    return pl + "!", msg
                if st:
                    return pl, msg
                continue
            if pl == "NodeUnschedulable":
                if node.unschedulable and not any(
                        t.tolerates(Taint("node.kubernetes.io/unschedulable", "", "NoSchedule"))
                        for t in pod.tolerations):
                    msg = "node(s) were unschedulable"
            elif pl == "NodeName":
                if pod.node_name and pod.node_name != node.name:
                    msg = "node(s) didn't match the requested node name"
            elif pl == "TaintToleration":
                t = self.untolerated_taint(pod, node)
                if t is not None:
                    msg = f"node(s) had untolerated taint {{{t.key}: {t.value}}}"
            elif pl == "NodeAffinity":
                msg = self.node_affinity_filter(pod, node)
            elif pl == "NodePorts":
                if not self.fits_ports(pod, ni):
                    msg = "node(s) didn't have free ports for the requested pod ports"
            elif pl == "NodeResourcesFit":
                msg = self.fit_filter(pod, ni, getattr(self, "scalar_order", None))
            elif pl == "PodTopologySpread":
                msg = self.pts_filter(pod, pts, node)
            elif pl == "InterPodAffinity":
                msg = self.ipa_filter(ipa, node)
            elif pl == "VolumeBinding" and pod.pvc_claims:   # FindPodVolumes' reasons, in its order
                reasons = []
                if not self.volume_binding_ok(pod, node):
                    reasons.append("node(s) had volume node affinity conflict")
                if self.find_pod_volumes(pod, node) is None:
                    reasons.append("node(s) didn't find available persistent volumes to bind")
                msg = ", ".join(reasons) or None
            elif pl == "VolumeZone":
                if pod.pvc_claims and not self.volume_zone_ok(pod, node):
                    msg = "node(s) had no available volume zone"
            if msg:
                return pl, msg
        return None, None

    @staticmethod
    def _nominated_for(pod: Pod, ni: NodeInfo, nominated) -> List[Pod]:
        """addNominatedPods' pods: the node's nominated pods of priority >= the
        pod's, the pod itself excluded (framework/runtime/framework.go v1.26)."""
        if not nominated:
            return []
        return [q for q in nominated.get(ni.node.name, ()) if q.priority >= pod.priority and q.name != pod.name]

    def filter_with_nominated(self, pod: Pod, ni: NodeInfo, pts, ipa, nominated):
        """RunFilterPluginsWithNominatedPods: with nominated pods, pass 1 runs on
        a clone carrying them (PreFilterExtensions.AddPod: the PTS / IPA counts
        recomputed over the clone); only if it passes, pass 2 on the node as is."""
        add = self._nominated_for(pod, ni, nominated)
        if add:
            saved = ni.save()
            for q in add:
                ni.add_pod(q)
            pl, msg = self.filter_node(pod, ni, self.pts_prefilter(pod), self.ipa_prefilter(pod))
            ni.restore(saved)
            if pl is not None:
                return pl, msg
        return self.filter_node(pod, ni, pts, ipa)

    @staticmethod
    def node_affinity_prefilter(pod: Pod) -> Optional[set]:
        """nodeaffinity.PreFilter's PreFilterResult.NodeNames (v1.26): None for
        all nodes; an empty set when the terms conflict."""
        if not pod.required_terms:
            return None
        out = None
        for t in pod.required_terms:
            term = None
            for r in t.match_fields:
                if r.key == "metadata.name" and r.operator == "In":
                    term = set(r.values) if term is None else term & set(r.values)
            if term is None:
                return None                   # this term admits every node (terms are ORed)
            out = set(term) if out is None else out | term
        return out

    def cycle(self, pod: Pod, extender=None, nominated=None, nominated_node: Optional[str] = None) -> dict:
        """``extender(kept node names) -> (filtered-out names, {name: combined weighted score})``
        models the scheduler's extenders (findNodesThatPassExtenders, prioritizeNodes).
        ``nominated``: the PodNominator, {node name: [pods nominated there]};
        ``nominated_node``: the pod's own status.nominatedNodeName."""
        seq = self.seq
        self.seq += 1
        vmsg = self.volume_prefilter(pod) if pod.pvc_claims else None
        if vmsg is not None:                               # UnschedulableAndUnresolvable at PreFilter
            return {"filter": {}, "n_feasible": 0, "raw": {}, "norm": {}, "total": {}, "error": None,
                    "chosen": None, "prefilter": vmsg}
        pts = self.pts_prefilter(pod)
        ipa = self.ipa_prefilter(pod)
        filt: Dict[str, Tuple[Optional[str], Optional[str]]] = {}
        # findNodesThatFitPod: PreFilterResult.NodeNames restricts the scan to
        # those nodes (upstream in Go map order; here nodeTree order, the
        # deterministic stand-in)
        names_pf = self.node_affinity_prefilter(pod)
        scan = self.nodes
        if names_pf is not None:
            if any(n not in self.by_name for n in names_pf):      # NodeInfos().Get fails
                return {"filter": filt, "n_feasible": 0, "raw": {}, "norm": {}, "total": {},
                        "error": "prefilter", "chosen": None}
            if not names_pf:                                      # "pod affinity terms conflict"
                return {"filter": filt, "n_feasible": 0, "raw": {}, "norm": {}, "total": {},
                        "error": None, "chosen": None}
            scan = [ni for ni in self.nodes if ni.node.name in names_pf]
        failed = set()
        if nominated_node is not None and nominated_node in self.by_name:
            # evaluateNominatedNode (schedule_one.go v1.26): the nominated node
            # first, whatever the PreFilterResult; if it passes it is the only
            # feasible node (no scoring, nextStartNodeIndex untouched); if it
            # fails its status stays in the diagnosis and counts as processed
            ni = self.by_name[nominated_node]
            pl, msg = self.filter_with_nominated(pod, ni, pts, ipa, nominated)
            filt[nominated_node] = (pl[:-1] if pl and pl.endswith("!") else pl, msg)
            if pl is None:
                ni.add_pod(pod)
                if pod.pvc_claims:
                    self.assume_volumes(pod, ni.node)
                return {"filter": filt, "n_feasible": 1, "raw": {}, "norm": {}, "total": {}, "error": None,
                        "chosen": nominated_node, "nominated_pass": True}
            if not pl.endswith("!"):
                failed.add(nominated_node)
        N = len(scan)
        K = num_feasible_nodes_to_find(self.pct, N)
        feasible: List[NodeInfo] = []
        error = None
        for i in range(N):
            ni = scan[(self.next_start + i) % N]
            pl, msg = self.filter_with_nominated(pod, ni, pts, ipa, nominated)
            if pl is not None and pl.endswith("!"):        # checkNode: the error ends the scan
                filt[ni.node.name] = (pl[:-1], msg)
                error = "filter"
                break
            filt[ni.node.name] = (pl, msg)
            if pl is None:
                if len(feasible) == K:
                    break
                feasible.append(ni)
            else:
                failed.add(ni.node.name)
        # processedNodes = feasible + len(diagnosis.NodeToStatusMap)
        self.next_start = (self.next_start + len(feasible) + len(failed)) % N
        ext_scores: Dict[str, int] = {}
        if extender is not None:
            out, ext_scores = extender([ni.node.name for ni in feasible])
            for name in out:
                filt[name] = ("extender", "filtered out by an extender")
            feasible = [ni for ni in feasible if ni.node.name not in out]
        res = {"filter": filt, "n_feasible": len(feasible), "raw": {}, "norm": {}, "total": {}, "error": error}
        if error is None and len(feasible) > 1 and "NetworkBandwidth" in self.score_order and \
                any(self.nb_score(ni) is None for ni in feasible):
            error = res["error"] = "score"                 # RunScorePlugins fails
        if error or not feasible:
            res["chosen"] = None
            return res
        if len(feasible) == 1:
            chosen = feasible[0]
        else:
            names = [ni.node.name for ni in feasible]
            pstate = self.pts_prescore(pod, feasible)
            topo = self.ipa_prescore(pod)
            totals = [0] * len(feasible)
            for pl in self.score_order:
                if pl == "NodeResourcesBalancedAllocation":
                    raw = [self.balanced(pod, ni) for ni in feasible]
                    norm = raw
                elif pl == "ImageLocality":
                    raw = [self.image_locality(pod, ni.node) for ni in feasible]
                    norm = raw
                elif pl == "InterPodAffinity":
                    raw = [self.ipa_score(topo, ni.node) for ni in feasible]
                    norm = self.ipa_normalize(topo, raw)
                elif pl == "NodeResourcesFit":
                    raw = [self.least_allocated(pod, ni) for ni in feasible]
                    norm = raw
                elif pl == "NodeAffinity":
                    raw = [sum(t.weight for t in list(pod.preferred_terms) + list(self.added.preferred)
                               if t.weight and self._term_match(t.term, ni.node))
                           for ni in feasible]
                    norm = self.default_normalize(raw, False)
                elif pl == "PodTopologySpread":
                    raw = [self.pts_score(pod, pstate, ni) for ni in feasible]
                    norm = self.pts_normalize(pstate, names, raw)
                elif pl == "NetworkBandwidth":
                    raw = [self.nb_score(ni) for ni in feasible]
                    norm = self.nb_normalize(raw)
                else:   # TaintToleration
                    raw = [sum(1 for t in ni.node.taints if t.effect == "PreferNoSchedule" and not any(
                        tol.tolerates(t) for tol in pod.tolerations if tol.effect in ("", "PreferNoSchedule")))
                        for ni in feasible]
                    norm = self.default_normalize(raw, True)
                w = self.weights.get(pl, 0) or 1
                res["raw"][pl] = dict(zip(names, raw))
                res["norm"][pl] = dict(zip(names, norm))
                totals = [a + b * w for a, b in zip(totals, norm)]
            if extender is not None:
                totals = [t + ext_scores.get(nm, 0) for t, nm in zip(totals, names)]
            res["total"] = dict(zip(names, totals))
            index = {ni.node.name: i for i, ni in enumerate(self.nodes)}
            best = max(range(len(feasible)), key=lambda j: tb_key(totals[j], self.seed, seq, index[names[j]]))
            chosen = feasible[best]
        chosen.add_pod(pod)
        if pod.pvc_claims:
            self.assume_volumes(pod, chosen.node)
        res["chosen"] = chosen.node.name
        return res
