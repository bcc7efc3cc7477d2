"""Reading a Go-harness fixture (tests/golden/go, tools/make_go_fixtures.py):
the objects, the profile's plugin args, the workloads and volumes, and the
per-cycle PodNominator inputs, for the restatements that replay it
(oracle/objref.py, the C oracle, the engine)."""
from ksim import ingest, profile
from ksim.model import (controller_from_dict, node_from_dict, pod_from_dict, pv_from_dict, pvc_from_dict,
                        service_from_dict)
from ksim.topology import SpreadDefaults
from ksim.volumes import VolumeIndex
from oracle.objref import ObjScheduler


def objects(doc):
    return ([node_from_dict(d) for d in doc["nodes"]], [pod_from_dict(d) for d in doc["boundPods"]],
            [pod_from_dict(d) for d in doc["pods"]])


def scheduler_profile(doc) -> profile.SchedulerProfile:
    """The profile of the fixture (its plugin args over the defaults) with its knobs."""
    sp = ingest.profile_from_config(doc["profile"]) if doc.get("profile") else profile.SchedulerProfile()
    sp.percentage_of_nodes_to_score = doc["percentageOfNodesToScore"]
    sp.tiebreak_seed = doc["tiebreakSeed"]
    sp.hard_pod_affinity_weight = doc["hardPodAffinityWeight"]
    return sp


def workloads(doc):
    services = [service_from_dict(d) for d in doc.get("services") or []]
    controllers = [controller_from_dict(kind, d) for key, kind in
                   (("replicationControllers", "ReplicationController"), ("replicaSets", "ReplicaSet"),
                    ("statefulSets", "StatefulSet")) for d in doc.get(key) or []]
    return services, controllers


def volumes(doc, nodes):
    pvs = [pv_from_dict(d) for d in doc.get("pvs") or []]
    pvcs = [pvc_from_dict(d) for d in doc.get("pvcs") or []]
    return pvs, pvcs, (VolumeIndex.from_nodes(nodes, pvs, pvcs) if (pvs or pvcs) else None)


def objref(doc, nodes, bound) -> ObjScheduler:
    sp = scheduler_profile(doc)
    services, controllers = workloads(doc)
    pvs, pvcs, _ = volumes(doc, nodes)
    return ObjScheduler(nodes, bound, namespaces=doc["namespaces"], pct=sp.percentage_of_nodes_to_score,
                        seed=sp.tiebreak_seed, hard_pod_affinity_weight=sp.hard_pod_affinity_weight,
                        fit=sp.fit, node_affinity=sp.node_affinity, spread=sp.spread, services=services,
                        controllers=controllers, pvs=pvs, pvcs=pvcs)


def nominated_pods(doc):
    return {d["metadata"]["name"]: pod_from_dict(d) for d in doc.get("nominatedPods") or []}


def cycle_kwargs(doc, i, nominated):
    """objref cycle() keywords of cycle i: the PodNominator and the pod's own
    nominated node."""
    inputs = doc.get("cycleInputs")
    if not inputs:
        return {}
    c = inputs[i]
    return {"nominated": {node: [nominated[n] for n in names] for node, names in c["nominator"].items()},
            "nominated_node": c.get("nominatedNodeName")}


def plain(doc) -> bool:
    """Cycles the C oracle's and the engine's single-cycle calls replay as is
    (no PodNominator, no PostFilter)."""
    return not doc.get("cycleInputs") and not doc.get("preemption")


def encode(doc, encode_cluster, encode_pods):
    """(cluster, encoded pods, SchedulerProfile, compiled profile) with the
    fixture's args, workloads and volumes."""
    nodes, bound, pods = objects(doc)
    sp = scheduler_profile(doc)
    services, controllers = workloads(doc)
    _, _, vol = volumes(doc, nodes)
    scalar = sorted({k for p in pods for c in p.containers + p.init_containers for k in c.requests
                     if k not in ("cpu", "memory", "ephemeral-storage", "pods")})
    cluster, _ = encode_cluster(nodes, bound, namespaces=doc["namespaces"], extra_scalar=scalar)
    enc = encode_pods(cluster, pods, volumes=vol, added_affinity=sp.node_affinity,
                      spread=SpreadDefaults(sp.spread, services, controllers))
    return cluster, enc, sp, profile.compile_profile(sp, cluster.scalar_names)
