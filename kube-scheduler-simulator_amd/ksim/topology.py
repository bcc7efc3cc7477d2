"""Host compiler for PodTopologySpread and InterPodAffinity.

Upstream evaluates label selectors and affinity terms against every existing
pod in PreFilter / PreScore ([upstream] podtopologyspread/filtering.go
calPreFilterState, scoring.go PreScore; interpodaffinity/filtering.go
getExistingAntiAffinityCounts / getIncomingAffinityAntiAffinityCounts,
scoring.go processExistingPod).  All of that string work depends only on the
pods' namespaces and labels, never on where pods are bound, so the host does
it once and the device keeps integer COUNT CLASSES:

  cnt[c][node] = sum over pods bound to node of mult(pod, c)

* selector class  — a pod matcher (namespace predicate + label selector);
                    mult = 1 if the pod matches.  Used by the incoming pod's
                    spread constraints and (anti)affinity terms.
* carried class   — (kind, matcher, topology key) of a term some pod CARRIES
                    (required anti-affinity, required affinity, preferred
                    affinity / anti-affinity); mult = number of such terms
                    (required) or the sum of their weights (preferred).  Used
                    when the incoming pod matches the carried term.

Every plugin quantity is then a domain sum of one class over the nodes sharing
the node's value of a topology key, which the engine computes on the device:
  PTS  TpPairToMatchNum[(k, v)]          = sum over eligible nodes with k=v of cnt[sel]
  IPA  existingAntiAffinityCounts[(k,v)] = sum over nodes with k=v of cnt[carried anti]
       affinityCounts / antiAffinityCounts, topologyScore[k][v] likewise.
A pod's "uses" (ksim_topo_use) list which class / key / role it needs; its
"adds" (ksim_class_add) are what its bind contributes to cnt (NodeInfo.AddPod).
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import abi
from .model import Controller, LabelSelector, Pod, PodAffinityTerm, Requirement, Service, TopologySpreadConstraint

LABEL_HOSTNAME = "kubernetes.io/hostname"

# carried-term kinds
CARRY_REQ_ANTI = "req_anti"
CARRY_REQ_AFF = "req_aff"
CARRY_PREF_AFF = "pref_aff"
CARRY_PREF_ANTI = "pref_anti"


class TopologyError(ValueError):
    pass


@dataclass(frozen=True)
class Matcher:
    """framework.AffinityTerm.Matches / countPodsMatchSelector as a predicate
    over (namespace, labels).  ``selector`` is LabelSelector.key() or None
    (nil selector -> labels.Nothing())."""
    namespaces: frozenset
    all_namespaces: bool
    selector: Optional[tuple]


def _validate_selector(sel: Optional[LabelSelector]) -> None:
    """LabelSelectorAsSelector errors make upstream PreFilter fail the cycle;
    the engine rejects such pods instead of diverging silently."""
    if sel is None:
        return
    for r in sel.match_expressions:
        if r.operator in ("In", "NotIn") and not r.values:
            raise TopologyError(f"selector requirement {r.key} {r.operator} needs values")
        if r.operator in ("Exists", "DoesNotExist") and r.values:
            raise TopologyError(f"selector requirement {r.key} {r.operator} must not have values")
        if r.operator not in ("In", "NotIn", "Exists", "DoesNotExist"):
            raise TopologyError(f"selector operator {r.operator} not supported")


class TopologyIndex:
    """Count classes of one cluster (kept on EncodedCluster.topo)."""

    def __init__(self, n_nodes: int, namespaces: Optional[Dict[str, Dict[str, str]]] = None):
        self.n = n_nodes
        self.ns_labels: Dict[str, Dict[str, str]] = dict(namespaces or {})
        self.selectors: Dict[tuple, LabelSelector] = {}
        self.keys: List[tuple] = []                 # class id -> identity
        self.ids: Dict[tuple, int] = {}
        self.counts: List[np.ndarray] = []          # class id -> int32[N]
        # bound pods grouped by (namespace, labels) signature: sig -> node positions
        self.bound_sigs: Dict[tuple, List[int]] = {}
        self.sig_pods: Dict[tuple, Pod] = {}
        self._match_cache: Dict[Tuple[tuple, Matcher], bool] = {}
        self.sel_ids: List[int] = []                # selector classes (subset of ids)
        self.carry_ids: List[int] = []              # carried classes
        self.port_ids: List[int] = []               # host-port classes (NodePorts)
        self.image_ids: List[int] = []              # image-signature classes (ImageLocality)
        self.images: Dict[str, Tuple[int, np.ndarray]] = {}   # image name -> (size, node mask)
        self.bound_ports: List[Tuple[int, tuple]] = []   # (node position, (ip, protocol, port)) of bound pods
        self._carry_uses: Dict[tuple, List[tuple]] = {}   # signature -> carried uses (valid for a class count)
        # Device matching (ksim.termmatch): with a ``matcher`` the
        # selector classes are matched against the bound pods in one
        # ksim_match_terms call per ``resolve``; while ``deferred`` no class is
        # matched on the host.
        self.matcher = None
        self.deferred = False
        self._sig_sel: Dict[tuple, List[int]] = {}        # signature -> selector classes it matches
        self._sig_sel_n = -1                              # len(sel_ids) when _sig_sel was filled

    # ---- matchers ------------------------------------------------------------
    def _sel_key(self, sel: Optional[LabelSelector]) -> Optional[tuple]:
        if sel is None:
            return None
        _validate_selector(sel)
        k = sel.key()
        self.selectors.setdefault(k, sel)
        return k

    def note_namespace(self, ns: str) -> None:
        self.ns_labels.setdefault(ns, {})

    def term_matcher(self, owner: Pod, t: PodAffinityTerm) -> Matcher:
        """newAffinityTerm + getNamespacesFromPodAffinityTerm, with a non-empty
        namespaceSelector resolved over the known namespaces
        (mergeAffinityTermNamespacesIfNotEmpty); an empty one ({}) matches every
        namespace, a nil one none."""
        names = set(t.namespaces)
        all_ns = False
        if not t.namespaces and t.namespace_selector is None:
            names.add(owner.namespace)
        if t.namespace_selector is not None:
            _validate_selector(t.namespace_selector)
            if t.namespace_selector.empty():
                all_ns = True
            else:
                names.update(ns for ns, lab in self.ns_labels.items() if t.namespace_selector.matches(lab))
        return Matcher(frozenset(names), all_ns, self._sel_key(t.label_selector))

    def matches(self, m: Matcher, ns: str, labels: Dict[str, str]) -> bool:
        if not (m.all_namespaces or ns in m.namespaces):
            return False
        return m.selector is not None and self.selectors[m.selector].matches(labels)

    def _pod_matches(self, m, pod: Pod) -> bool:
        sig = (pod.namespace, tuple(sorted(pod.labels.items())))
        return self._sig_matches(m, sig, pod)

    def _sig_matches(self, m, sig, pod: Pod) -> bool:
        ck = (sig, m)
        v = self._match_cache.get(ck)
        if v is None:
            if isinstance(m, tuple) and m and m[0] == "all":
                v = all(self.matches(x, pod.namespace, pod.labels) for x in m[1])
            else:
                v = self.matches(m, pod.namespace, pod.labels)
            self._match_cache[ck] = v
        return v

    # ---- classes -------------------------------------------------------------
    def _new_class(self, key: tuple, counts: np.ndarray) -> int:
        cid = len(self.keys)
        if cid >= abi.MAX_CLASSES:
            raise TopologyError("too many count classes")
        self.keys.append(key)
        self.ids[key] = cid
        self.counts.append(counts)
        {"sel": self.sel_ids, "carry": self.carry_ids, "port": self.port_ids,
         "image": self.image_ids}[key[0]].append(cid)
        return cid

    # ---- NodePorts: HostPortInfo as count classes -------------------------------
    # A class ("port", ip, protocol, port) counts the pods on a node using that
    # exact triple; ("port", "*", protocol, port) those using it on any ip.
    # HostPortInfo.CheckConflict(ip, protocol, port): ip 0.0.0.0 conflicts
    # with the (protocol, port) pair on any ip, another ip with itself and 0.0.0.0.
    def port_class(self, ip: str, protocol: str, port: int) -> int:
        key = ("port", ip, protocol, port)
        cid = self.ids.get(key)
        if cid is not None:
            return cid
        cnt = np.zeros(self.n, np.int32)
        for pos, (bip, bproto, bport) in self.bound_ports:
            if bproto == protocol and bport == port and (ip == "*" or ip == bip):
                cnt[pos] += 1
        return self._new_class(key, cnt)

    def port_check_classes(self, pod: Pod) -> List[int]:
        """Classes whose presence on a node fails NodePorts for ``pod`` (fitsPorts)."""
        out: List[int] = []
        for ip, proto, port in pod_host_ports(pod):
            keys = [("*", proto, port)] if ip == DEFAULT_BIND_ALL_HOST_IP else \
                [(DEFAULT_BIND_ALL_HOST_IP, proto, port), (ip, proto, port)]
            for k in keys:
                c = self.port_class(*k)
                if c not in out:
                    out.append(c)
        return out

    # ---- ImageLocality: static per-node scores per image signature ----------------
    def set_images(self, nodes_in_add_order, pos_of: Dict[str, int]) -> None:
        """cache.addNodeImageStates over the nodes in the order they were added:
        an image name's size is the one of the first node listing it, its
        NumNodes the nodes listing it (ImageStateSummary)."""
        for n in nodes_in_add_order:
            for names, size in n.images:
                for name in names:
                    st = self.images.get(name)
                    if st is None:
                        st = (int(size), np.zeros(self.n, bool))
                        self.images[name] = st
                    st[1][pos_of[n.name]] = True

    def image_class(self, pod: Pod) -> Optional[int]:
        """Class whose count on a node is imagelocality.Score(pod, node):
        calculatePriority(sumImageScores(node, containers, N), len(containers))."""
        names = tuple(normalized_image_name(c.image) for c in pod.containers)
        if not any(nm in self.images for nm in names):
            return None                                  # 0 on every node: no use needed
        return self._image_class(names)

    def _image_class(self, names: tuple) -> int:
        key = ("image", names)
        cid = self.ids.get(key)
        if cid is not None:
            return cid
        total = np.zeros(self.n, np.int64)
        for nm in names:
            st = self.images.get(nm)
            if st is None:
                continue
            size, mask = st
            spread = float(int(mask.sum())) / float(self.n)       # float64(NumNodes) / float64(totalNumNodes)
            total += np.where(mask, int(float(size) * spread), 0)   # int64(float64(Size) * spread)
        max_t = IMAGE_MAX_CONTAINER_THRESHOLD * len(names)
        s = np.minimum(np.maximum(total, IMAGE_MIN_THRESHOLD), max_t)
        score = (100 * (s - IMAGE_MIN_THRESHOLD)) // (max_t - IMAGE_MIN_THRESHOLD)
        return self._new_class(key, score.astype(np.int32))

    def preregister(self, src: "TopologyIndex") -> None:
        """Register the classes of ``src``, in order, before any bound pod is
        added (a re-encoded snapshot keeps the class ids of the one it
        replaces, ksim.ingest.NodeCache); the bound pods then count into them."""
        for k, v in src.selectors.items():
            self.selectors.setdefault(k, v)
        for key in src.keys:
            if key[0] == "carry":
                self.carried_class(key[1], key[2], key[3])
            elif key[0] == "sel":
                self.selector_class(key[1])
            elif key[0] == "port":
                self.port_class(*key[1:])
            else:
                self._image_class(key[1])

    def port_adds(self, pod: Pod) -> Dict[int, int]:
        """NodeInfo.AddPod -> UsedPorts.Add of each host port, on the registered classes."""
        out: Dict[int, int] = {}
        for ip, proto, port in pod_host_ports(pod):
            for k in (("port", "*", proto, port), ("port", ip, proto, port)):
                c = self.ids.get(k)
                if c is not None:
                    out[c] = out.get(c, 0) + 1
        return out

    def selector_class(self, m) -> int:
        """Class of pods matching ``m`` (a Matcher, or ("all", (Matcher, ...))
        for podMatchesAllAffinityTerms).  Counts come from the bound pods."""
        key = ("sel", m)
        cid = self.ids.get(key)
        if cid is not None:
            return cid
        cnt = np.zeros(self.n, np.int32)
        if not self.deferred:                          # deferred: counted by resolve()
            for sig, positions in self.bound_sigs.items():
                if self._sig_matches(m, sig, self.sig_pods[sig]):
                    np.add.at(cnt, np.asarray(positions, np.int64), 1)
        return self._new_class(key, cnt)

    def carried_class(self, kind: str, m: Matcher, topology_key: str) -> int:
        key = ("carry", kind, m, topology_key)
        cid = self.ids.get(key)
        if cid is None:
            cid = self._new_class(key, np.zeros(self.n, np.int32))
        return cid

    def carried_terms(self, pod: Pod) -> List[Tuple[int, int]]:
        """(class, multiplicity) of the terms ``pod`` carries once bound."""
        out: Dict[int, int] = {}
        for t in pod.pod_anti_affinity_required:
            c = self.carried_class(CARRY_REQ_ANTI, self.term_matcher(pod, t), t.topology_key)
            out[c] = out.get(c, 0) + 1
        for t in pod.pod_affinity_required:
            c = self.carried_class(CARRY_REQ_AFF, self.term_matcher(pod, t), t.topology_key)
            out[c] = out.get(c, 0) + 1
        for w in pod.pod_affinity_preferred:
            c = self.carried_class(CARRY_PREF_AFF, self.term_matcher(pod, w.term), w.term.topology_key)
            out[c] = out.get(c, 0) + w.weight
        for w in pod.pod_anti_affinity_preferred:
            c = self.carried_class(CARRY_PREF_ANTI, self.term_matcher(pod, w.term), w.term.topology_key)
            out[c] = out.get(c, 0) + w.weight
        return sorted(out.items())

    def add_bound(self, pod: Pod, pos: int, carried: Optional[List[Tuple[int, int]]] = None) -> None:
        """An existing pod bound at node position ``pos`` (NodeInfo.AddPod).
        ``carried``: its carried_terms, when the caller has them already."""
        self.note_namespace(pod.namespace)
        for c, mult in (self.carried_terms(pod) if carried is None else carried):
            self.counts[c][pos] += mult
        if not self.deferred:
            for cid in self.sel_ids:
                if self._pod_matches(self.keys[cid][1], pod):
                    self.counts[cid][pos] += 1
        for c, k in self.port_adds(pod).items():
            self.counts[c][pos] += k
        self.bound_ports.extend((pos, t) for t in pod_host_ports(pod))
        sig = (pod.namespace, tuple(sorted(pod.labels.items())))
        self.bound_sigs.setdefault(sig, []).append(pos)
        self.sig_pods.setdefault(sig, pod)

    def adds(self, pod: Pod) -> List[Tuple[int, int]]:
        """(class, count) this pod contributes when bound: its carried terms
        plus every selector class it matches."""
        out = dict(self.carried_terms(pod))
        sig = (pod.namespace, tuple(sorted(pod.labels.items())))
        sel = self._sig_sel.get(sig) if self._sig_sel_n == len(self.sel_ids) else None
        if sel is None:
            sel = [cid for cid in self.sel_ids if self._sig_matches(self.keys[cid][1], sig, pod)]
        for cid in sel:
            out[cid] = out.get(cid, 0) + 1
        for cid, k in self.port_adds(pod).items():
            out[cid] = out.get(cid, 0) + k
        return sorted(out.items())

    def carried_uses(self, cluster, pod: Pod) -> List[tuple]:
        """Uses of the carried classes whose term matches ``pod`` (cached per
        (namespace, labels) signature and class count)."""
        ck = (pod.namespace, tuple(sorted(pod.labels.items())), len(self.carry_ids))
        hit = self._carry_uses.get(ck)
        if hit is not None:
            return hit
        out = []
        sig = ck[:2]
        for cid in self.carry_ids:
            _, kind, m, tk = self.keys[cid]
            if not self._sig_matches(m, sig, pod):
                continue
            col = _col(cluster, tk)
            if kind == CARRY_REQ_ANTI:
                out.append(_use(abi.USE_IPA_EXISTING_ANTI, cid, col))
            elif kind == CARRY_REQ_AFF:
                out.append(_use(abi.USE_IPA_SCORE_HARD, cid, col, 1))
            elif kind == CARRY_PREF_AFF:
                out.append(_use(abi.USE_IPA_SCORE, cid, col, 1))
            else:
                out.append(_use(abi.USE_IPA_SCORE, cid, col, -1))
        self._carry_uses[ck] = out
        return out

    def resolve(self, pods: Sequence[Pod] = ()) -> None:
        """Match every selector and carried class against the bound pods'
        signatures and those of ``pods`` on the device (``self.matcher``,
        ksim_match_terms), set the selector classes' counts over the bound
        pods, and end the deferred state."""
        self.deferred = False
        if self.matcher is None:
            return
        from .termmatch import MatchProblem
        sigs = list(self.bound_sigs)
        index = {sig: i for i, sig in enumerate(sigs)}
        for p in pods:
            sig = (p.namespace, tuple(sorted(p.labels.items())))
            if sig not in index:
                index[sig] = len(sigs)
                sigs.append(sig)
        ms = [self.keys[c][1] for c in self.sel_ids] + [self.keys[c][2] for c in self.carry_ids]
        mp = MatchProblem(self, ms, sigs)
        lens = [len(v) for v in self.bound_sigs.values()]
        pod_sig = np.repeat(np.arange(len(lens), dtype=np.int32), lens)
        pod_node = np.fromiter((x for v in self.bound_sigs.values() for x in v), np.int32, int(sum(lens)))
        mp.set_counts(pod_sig, pod_node, self.n, range(len(self.sel_ids)))
        hit, counts = self.matcher.match(mp)
        for j, cid in enumerate(self.sel_ids):
            self.counts[cid] = counts[j].copy()
        ns = len(self.sel_ids)
        self._sig_sel = {sig: [self.sel_ids[j] for j in np.flatnonzero(hit[i, :ns])] for i, sig in enumerate(sigs)}
        self._sig_sel_n = ns
        for j, cid in enumerate(self.carry_ids):
            m = self.keys[cid][2]
            col = hit[:, ns + j]
            for i, sig in enumerate(sigs):
                self._match_cache[(sig, m)] = bool(col[i])

    def class_count_array(self) -> np.ndarray:
        if not self.counts:
            return np.zeros((0, self.n), np.int32)
        return np.stack(self.counts).astype(np.int32)


# ---- PodTopologySpread default constraints ---------------------------------------
class SpreadDefaults:
    """podtopologyspread.buildDefaultConstraints with helper.DefaultSelector
    (v1.26): a pod with no topologySpreadConstraints of its own takes the
    profile's default constraints (PodTopologySpreadArgs: System = hostname
    maxSkew 3 and zone maxSkew 5, both ScheduleAnyway; List = the args'
    defaultConstraints), with the selector merged from the Services that
    select it and its controlling ReplicationController / ReplicaSet /
    StatefulSet; none when that selector is empty.  The simulator runs the
    Deployment and ReplicaSet controllers
    (/root/reference/simulator/controller/controller.go:79-80), so every
    Deployment pod is ReplicaSet-owned."""

    def __init__(self, args, services: Sequence[Service] = (), controllers: Sequence[Controller] = ()):
        self.args = args
        self.system = args.defaulting_type == "System"
        self.defaults = args.constraints()
        self.services: Dict[str, List[Service]] = {}
        for s in services:
            self.services.setdefault(s.namespace, []).append(s)
        self.controllers = {(c.kind, c.namespace, c.name): c for c in controllers}

    def default_selector(self, pod: Pod) -> Optional[LabelSelector]:
        """helper.DefaultSelector; None when the selector is Empty()."""
        label_set: Dict[str, str] = {}
        for svc in self.services.get(pod.namespace, []):          # GetPodServices
            if svc.selector is None:                               # nil selectors match nothing
                continue
            if all(pod.labels.get(k) == v for k, v in svc.selector.items()):
                label_set.update(svc.selector)                     # labels.Merge
        extra: List[Requirement] = []
        if pod.owner is not None:
            api, kind, name = pod.owner
            if (api, kind) == ("v1", "ReplicationController"):
                rc = self.controllers.get(("ReplicationController", pod.namespace, name))
                if rc is not None and rc.selector:
                    label_set.update(rc.selector)
            elif (api, kind) in (("apps/v1", "ReplicaSet"), ("apps/v1", "StatefulSet")):
                obj = self.controllers.get((kind, pod.namespace, name))
                sel = obj.selector if obj is not None else None
                if sel is not None:                                # nil: labels.Nothing(), no requirements
                    _validate_selector(sel)
                    extra += [Requirement(k, "In", [v]) for k, v in sorted(sel.match_labels.items())]
                    extra += list(sel.match_expressions)
        if not label_set and not extra:
            return None
        return LabelSelector(dict(label_set), extra)

    def constraints(self, pod: Pod) -> Tuple[List[TopologySpreadConstraint], bool]:
        """(the pod's spread constraints, whether they are system defaults)."""
        if pod.topology_spread:
            return list(pod.topology_spread), False
        if not self.defaults:
            return [], False
        sel = self.default_selector(pod)
        if sel is None:
            return [], False
        return [dataclasses.replace(c, label_selector=sel) for c in self.defaults], self.system


def pod_spread(spread: Optional[SpreadDefaults], pod: Pod) -> Tuple[List[TopologySpreadConstraint], bool]:
    return spread.constraints(pod) if spread is not None else (list(pod.topology_spread), False)


# ---- per-pod compilation -------------------------------------------------------
DEFAULT_BIND_ALL_HOST_IP = "0.0.0.0"
_MB = 1024 * 1024
IMAGE_MIN_THRESHOLD = 23 * _MB                 # imagelocality minThreshold
IMAGE_MAX_CONTAINER_THRESHOLD = 1000 * _MB     # imagelocality maxContainerThreshold


def normalized_image_name(name: str) -> str:
    """imagelocality normalizedImageName: a name without a tag gets ":latest"."""
    if name.rfind(":") <= name.rfind("/"):
        name = name + ":latest"
    return name


def pod_host_ports(pod: Pod) -> List[tuple]:
    """(ip, protocol, port) of the pod's containers' host ports, sanitized as
    HostPortInfo does (empty ip -> 0.0.0.0, empty protocol -> TCP); port <= 0
    is no host port.  Init containers' ports are not host ports of the pod."""
    out = []
    for c in pod.containers:
        for p in c.ports:
            if p.host_port > 0:
                out.append((p.host_ip or DEFAULT_BIND_ALL_HOST_IP, p.protocol or "TCP", int(p.host_port)))
    return out


def _col(cluster, key: str) -> int:
    c = cluster.label_col(key)
    return abi.COL_NONE if c < 0 else c


def register_pod_classes(topo: TopologyIndex, pod: Pod, spread: Optional[SpreadDefaults] = None) -> None:
    """Pass 1: every class the pod will use or carry exists before any pod's
    adds are computed (so a later queue pod's selector counts earlier ones)."""
    topo.note_namespace(pod.namespace)
    topo.carried_terms(pod)
    for c in pod_spread(spread, pod)[0]:
        _validate_selector(c.label_selector)
        if c.label_selector is not None and not c.label_selector.empty():
            topo.selector_class(Matcher(frozenset([pod.namespace]), False, topo._sel_key(c.label_selector)))
    if pod.pod_affinity_required:
        topo.selector_class(("all", tuple(topo.term_matcher(pod, t) for t in pod.pod_affinity_required)))
    for t in pod.pod_anti_affinity_required:
        topo.selector_class(topo.term_matcher(pod, t))
    for w in pod.pod_affinity_preferred + pod.pod_anti_affinity_preferred:
        topo.selector_class(topo.term_matcher(pod, w.term))
    topo.port_check_classes(pod)
    topo.image_class(pod)


def _use(kind, cls, col, arg=0, flags=0):
    return (cls, arg, col, kind, flags)


def pod_uses(topo: TopologyIndex, cluster, pod: Pod, spread: Optional[SpreadDefaults] = None) -> Tuple[List[tuple], int]:
    """Pass 2: the pod's uses (ksim_topo_use rows) and topo flags."""
    uses: List[tuple] = []
    flags = 0
    # --- PodTopologySpread: filterTopologySpreadConstraints (hard, then soft) ---
    seen = {"DoNotSchedule": set(), "ScheduleAnyway": set()}
    cons, sysdef = pod_spread(spread, pod)
    if sysdef and cons:
        flags |= abi.POD_PTS_SYSTEM_DEFAULT
    for c in cons:
        if c.when_unsatisfiable not in seen:
            raise TopologyError(f"whenUnsatisfiable {c.when_unsatisfiable} not supported")
        if c.topology_key in seen[c.when_unsatisfiable]:
            raise TopologyError("duplicate topologyKey/whenUnsatisfiable (rejected by API validation)")
        seen[c.when_unsatisfiable].add(c.topology_key)
        if c.max_skew < 1:
            raise TopologyError("maxSkew must be >= 1")
        sel = c.label_selector
        cls = -1
        if sel is not None and not sel.empty():       # countPodsMatchSelector: Empty() counts 0
            cls = topo.selector_class(Matcher(frozenset([pod.namespace]), False, topo._sel_key(sel)))
        f = 0
        if sel is not None and sel.matches(pod.labels):   # c.Selector.Matches(podLabelSet)
            f |= abi.USEF_SELF_MATCH
        if (c.node_affinity_policy or "Honor") == "Honor":
            f |= abi.USEF_HONOR_AFFINITY
        if (c.node_taints_policy or "Ignore") == "Honor":
            f |= abi.USEF_HONOR_TAINTS
        if c.topology_key == LABEL_HOSTNAME:
            f |= abi.USEF_HOSTNAME
        kind = abi.USE_PTS_HARD if c.when_unsatisfiable == "DoNotSchedule" else abi.USE_PTS_SOFT
        uses.append(_use(kind, cls, _col(cluster, c.topology_key), c.max_skew, f))
    # --- InterPodAffinity filter: incoming required affinity (all terms) ---
    if pod.pod_affinity_required:
        ms = tuple(topo.term_matcher(pod, t) for t in pod.pod_affinity_required)
        cls = topo.selector_class(("all", ms))
        for t in pod.pod_affinity_required:
            uses.append(_use(abi.USE_IPA_AFFINITY, cls, _col(cluster, t.topology_key)))
        if all(topo.matches(m, pod.namespace, pod.labels) for m in ms):
            flags |= abi.POD_IPA_SELF_AFFINITY
    for t in pod.pod_anti_affinity_required:
        cls = topo.selector_class(topo.term_matcher(pod, t))
        uses.append(_use(abi.USE_IPA_ANTI, cls, _col(cluster, t.topology_key)))
    # --- carried terms of other pods that match this pod ---
    uses.extend(topo.carried_uses(cluster, pod))
    # --- incoming preferred (anti)affinity terms (score) ---
    for w in pod.pod_affinity_preferred:
        uses.append(_use(abi.USE_IPA_SCORE, topo.selector_class(topo.term_matcher(pod, w.term)),
                         _col(cluster, w.term.topology_key), w.weight))
    for w in pod.pod_anti_affinity_preferred:
        uses.append(_use(abi.USE_IPA_SCORE, topo.selector_class(topo.term_matcher(pod, w.term)),
                         _col(cluster, w.term.topology_key), -w.weight))
    # --- ImageLocality: the pod's image-signature score class ---
    ic = topo.image_class(pod)
    if ic is not None:
        uses.append(_use(abi.USE_IMAGE, ic, abi.COL_NONE))
    # --- NodePorts: a conflicting host port on the node fails the filter ---
    for cls in topo.port_check_classes(pod):
        uses.append(_use(abi.USE_NODE_PORT, cls, abi.COL_NONE))
    if len(uses) > abi.MAX_USES:
        raise TopologyError(f"pod {pod.name}: {len(uses)} topology uses > {abi.MAX_USES}")
    return uses, flags


def topo_log_table(n_nodes: int) -> np.ndarray:
    """topologyNormalizingWeight(size) = math.Log(float64(size + 2)) for
    size = 0..n_nodes, computed on the host (the simulator's Go host would
    use math.Log) so the device never evaluates log."""
    import math
    return np.array([math.log(float(s + 2)) for s in range(n_nodes + 1)], np.float64)
