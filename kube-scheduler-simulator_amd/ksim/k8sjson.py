"""Model objects back to Kubernetes v1 JSON (the inverse of model.node_from_dict
/ pod_from_dict).

Used to write fixtures for the Go harness (oracle/go): the same nodes and pods
the engine and the oracles schedule, as the v1.Node / v1.Pod documents the
reference's scheduler reads (golden vectors item 4).
"""
from typing import Dict, List, Optional

from .model import (Container, LabelSelector, Node, NodeSelectorTerm, Pod, PodAffinityTerm, Requirement,
                    TopologySpreadConstraint, WeightedPodAffinityTerm)


def _req(r: Requirement) -> dict:
    d = {"key": r.key, "operator": r.operator}
    if r.values:
        d["values"] = list(r.values)
    return d


def _term(t: NodeSelectorTerm) -> dict:
    d = {}
    if t.match_expressions:
        d["matchExpressions"] = [_req(r) for r in t.match_expressions]
    if t.match_fields:
        d["matchFields"] = [_req(r) for r in t.match_fields]
    return d


def _selector(s: Optional[LabelSelector]) -> Optional[dict]:
    if s is None:
        return None
    d = {}
    if s.match_labels:
        d["matchLabels"] = dict(s.match_labels)
    if s.match_expressions:
        d["matchExpressions"] = [_req(r) for r in s.match_expressions]
    return d


def _pod_term(t: PodAffinityTerm) -> dict:
    d = {"topologyKey": t.topology_key}
    if t.label_selector is not None:
        d["labelSelector"] = _selector(t.label_selector)
    if t.namespaces:
        d["namespaces"] = list(t.namespaces)
    if t.namespace_selector is not None:
        d["namespaceSelector"] = _selector(t.namespace_selector)
    return d


def _weighted(w: WeightedPodAffinityTerm) -> dict:
    return {"weight": w.weight, "podAffinityTerm": _pod_term(w.term)}


def _spread(c: TopologySpreadConstraint) -> dict:
    d = {"maxSkew": c.max_skew, "topologyKey": c.topology_key, "whenUnsatisfiable": c.when_unsatisfiable}
    if c.label_selector is not None:
        d["labelSelector"] = _selector(c.label_selector)
    if c.min_domains is not None:
        d["minDomains"] = c.min_domains
    if c.node_affinity_policy is not None:
        d["nodeAffinityPolicy"] = c.node_affinity_policy
    if c.node_taints_policy is not None:
        d["nodeTaintsPolicy"] = c.node_taints_policy
    return d


def _container(c: Container, name: str) -> dict:
    d = {"name": name}
    if c.image:                   # ImageLocality reads it; an empty image stays absent
        d["image"] = c.image
    if c.requests:
        d["resources"] = {"requests": dict(c.requests)}
    ports = []
    for p in c.ports:
        q = {"containerPort": p.host_port or 80, "protocol": p.protocol}
        if p.host_port:
            q["hostPort"] = p.host_port
        if p.host_ip:
            q["hostIP"] = p.host_ip
        ports.append(q)
    if ports:
        d["ports"] = ports
    return d


def node_to_dict(n: Node) -> dict:
    md = {"name": n.name}
    if n.labels:
        md["labels"] = dict(n.labels)
    if n.annotations:
        md["annotations"] = dict(n.annotations)
    spec = {}
    if n.taints:
        spec["taints"] = [{"key": t.key, "value": t.value, "effect": t.effect} if t.value else
                          {"key": t.key, "effect": t.effect} for t in n.taints]
    if n.unschedulable:
        spec["unschedulable"] = True
    status = {"allocatable": dict(n.allocatable), "capacity": dict(n.allocatable)}
    if n.images:
        status["images"] = [{"names": list(names), "sizeBytes": int(size)} for names, size in n.images]
    return {"apiVersion": "v1", "kind": "Node", "metadata": md, "spec": spec, "status": status}


def pod_to_dict(p: Pod) -> dict:
    if p.has_volumes:
        raise ValueError(f"pod {p.name}: volumes are not modelled")
    md = {"name": p.name, "namespace": p.namespace}
    if p.labels:
        md["labels"] = dict(p.labels)
    if p.annotations:
        md["annotations"] = dict(p.annotations)
    if p.owner is not None:
        api, kind, name = p.owner
        md["ownerReferences"] = [{"apiVersion": api, "kind": kind, "name": name, "uid": f"uid-{kind}-{name}",
                                  "controller": True}]
    spec: Dict[str, object] = {"containers": [_container(c, f"c{i}") for i, c in enumerate(p.containers)]}
    if p.pvc_claims:
        spec["volumes"] = [{"name": f"v{i}", "persistentVolumeClaim": {"claimName": c}}
                           for i, c in enumerate(p.pvc_claims)]
    if p.init_containers:
        spec["initContainers"] = [_container(c, f"i{i}") for i, c in enumerate(p.init_containers)]
    if p.overhead:
        spec["overhead"] = dict(p.overhead)
    if p.node_selector:
        spec["nodeSelector"] = dict(p.node_selector)
    if p.node_name:
        spec["nodeName"] = p.node_name
    if p.priority:
        spec["priority"] = p.priority
    if p.tolerations:
        spec["tolerations"] = [{k: v for k, v in (("key", t.key), ("operator", t.operator), ("value", t.value),
                                                  ("effect", t.effect)) if v} for t in p.tolerations]
    if p.topology_spread:
        spec["topologySpreadConstraints"] = [_spread(c) for c in p.topology_spread]
    aff: Dict[str, dict] = {}
    na = {}
    if p.required_terms is not None:
        na["requiredDuringSchedulingIgnoredDuringExecution"] = {"nodeSelectorTerms": [_term(t) for t in
                                                                                      p.required_terms]}
    if p.preferred_terms:
        na["preferredDuringSchedulingIgnoredDuringExecution"] = [{"weight": t.weight, "preference": _term(t.term)}
                                                                 for t in p.preferred_terms]
    if na:
        aff["nodeAffinity"] = na
    for key, req, pref in (("podAffinity", p.pod_affinity_required, p.pod_affinity_preferred),
                           ("podAntiAffinity", p.pod_anti_affinity_required, p.pod_anti_affinity_preferred)):
        d = {}
        if req:
            d["requiredDuringSchedulingIgnoredDuringExecution"] = [_pod_term(t) for t in req]
        if pref:
            d["preferredDuringSchedulingIgnoredDuringExecution"] = [_weighted(w) for w in pref]
        if d:
            aff[key] = d
    if aff:
        spec["affinity"] = aff
    return {"apiVersion": "v1", "kind": "Pod", "metadata": md, "spec": spec}


def nodes_to_list(nodes: List[Node]) -> List[dict]:
    return [node_to_dict(n) for n in nodes]


def pods_to_list(pods: List[Pod]) -> List[dict]:
    return [pod_to_dict(p) for p in pods]
