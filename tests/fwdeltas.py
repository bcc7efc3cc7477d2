"""Framework cycles interleaved with informer events (TEST INFRASTRUCTURE).

Drives ksim.fwsnapshot.SnapshotSync -- the Python mirror of the Go adapter's
incremental snapshot (integration/go/engine/encoder.go) -- under the racing
framework mirror (tests/fwmirror.py), with external events between cycles:
bound pods added and deleted (including pods the framework placed), pod label
updates, nodes added, updated (allocatable, labels, a zone move) and removed
with their pods.  Every event reaches every run alike.  A ``FullSync`` run is
the reference: it re-encodes its whole record every cycle and re-sends it
with set_cluster (the round-5 Go host's behaviour), so an incremental run that
agrees with it cycle by cycle applied every delta right.
"""
from __future__ import annotations

import copy
import random
from typing import List

import numpy as np

from fwmirror import Framework, annotations
from ksim import gen, profile
from ksim.fwplugins import EnginePlugins
from ksim.fwsnapshot import SnapshotSync
from ksim.model import Node
from ksim.resultstore import Store


class FullSync(SnapshotSync):
    """The reference: every cycle start re-encodes the record (nodes in add
    order, every bound pod) and sends it whole."""

    def snapshot(self) -> None:
        ev, self.events = self.events, []
        nodes = [(k, x) for k, x in ev if k in ("node", "node-")]
        if nodes:
            self._record_nodes(nodes)
        for k, x in ev:
            if k in ("pod", "pod-"):
                self._record_pod(k, x)
        for key, p in list(self.waiting.items()):
            if p.node_name in self.nodes:
                del self.waiting[key]
                self.bound[key] = (p, p.node_name)
        self._full()


class Run:
    def __init__(self, name, backend, sync, fw, store):
        self.name, self.b, self.sync, self.fw, self.store = name, backend, sync, fw, store


def make_runs(specs, nodes, bound, sp, seed):
    """specs: [(name, backend, full)] -> Runs over the same objects and seed."""
    w = profile.default_score_weights()
    runs = []
    for name, backend, full in specs:
        sync = (FullSync if full else SnapshotSync)(backend, nodes, bound)
        store = Store(w)
        fw = Framework(EnginePlugins(backend, None, sp, sync=sync), sp, store, seed=seed)
        runs.append(Run(name, backend, sync, fw, store))
    return runs


def objects(n_nodes=90, pods_per_node=3, n_incoming=160):
    nodes, bound, incoming = gen.config3_objects(n_nodes=n_nodes, pods_per_node=pods_per_node,
                                                 n_incoming=n_incoming)
    return nodes, bound, incoming


def drive(runs: List[Run], nodes, bound, incoming, seed=11, every=2, on_step=None):
    """Schedule ``incoming`` through every run with events between cycles;
    asserts the runs agree on every placement, feasible list and annotation.
    Returns the number of events."""
    rng = random.Random(seed)
    world_nodes = {n.name: n for n in nodes}
    world_pods = {(p.namespace, p.name): p for p in bound}
    extra = 0
    events = 0

    def emit(method, *args):
        for r in runs:
            getattr(r.sync, method)(*args)

    for i, pod in enumerate(incoming):
        if i % every == 0:
            for _ in range(rng.randint(1, 3)):
                kind = rng.choice(["add_pod", "add_pod", "del_pod", "del_pod", "relabel", "add_node", "upd_node",
                                   "zone_node", "rm_node"])
                if kind == "add_pod" and world_nodes:
                    proto = world_pods[rng.choice(sorted(world_pods))] if world_pods else bound[0]
                    p = copy.copy(proto)
                    p.name = f"ext-{extra:05d}"
                    extra += 1
                    p.node_name = rng.choice(sorted(world_nodes))
                    p.labels = dict(proto.labels)
                    world_pods[(p.namespace, p.name)] = p
                    emit("add_pod", p)
                elif kind == "del_pod" and world_pods:
                    key = rng.choice(sorted(world_pods))
                    emit("delete_pod", world_pods.pop(key))
                elif kind == "relabel" and world_pods:
                    key = rng.choice(sorted(world_pods))
                    old = world_pods[key]
                    new = copy.copy(old)
                    new.labels = dict(old.labels, app=f"a{rng.randrange(64)}")
                    world_pods[key] = new
                    emit("update_pod", old, new)
                elif kind == "add_node":
                    z = rng.randrange(3)
                    name = f"extra-{extra:05d}"
                    extra += 1
                    n = Node(name=name, labels={"kubernetes.io/hostname": name, "topology.kubernetes.io/zone": f"z{z}"},
                             allocatable={"cpu": str(rng.choice([16, 32])), "memory": "64Gi", "pods": "110"})
                    world_nodes[name] = n
                    emit("add_node", n)
                elif kind in ("upd_node", "zone_node") and world_nodes:
                    old = world_nodes[rng.choice(sorted(world_nodes))]
                    n = copy.copy(old)
                    if kind == "upd_node":
                        n.allocatable = dict(old.allocatable, cpu=str(rng.choice([8, 16, 48])))
                        n.labels = dict(old.labels, rack=f"r{rng.randrange(4)}")
                    else:
                        z = int(old.labels.get("topology.kubernetes.io/zone", "z0")[1:])
                        n.labels = dict(old.labels, **{"topology.kubernetes.io/zone": f"z{(z + 1) % 3}"})
                    world_nodes[n.name] = n
                    emit("update_node", n)
                elif kind == "rm_node" and len(world_nodes) > 20 and rng.random() < 0.5:
                    name = rng.choice(sorted(world_nodes))
                    del world_nodes[name]
                    for key in [k for k, p in world_pods.items() if p.node_name == name]:
                        del world_pods[key]            # the pod GC removes them; the snapshot already did
                    emit("remove_node", name)
                else:
                    continue
                events += 1
        recs = []
        for r in runs:
            ps = r.fw.pl.begin(pod)
            rec = r.fw.schedule_one(ps, 0, 0, None)
            recs.append((rec, ps))
        base, bps = recs[0]
        names0 = runs[0].fw.names
        for r, (rec, ps) in zip(runs[1:], recs[1:]):
            names = r.fw.names
            assert list(names) == list(names0), (i, r.name, "node order")
            assert rec["chosen"] == base["chosen"], (i, r.name, rec["chosen"], base["chosen"])
            assert rec.get("feasible") == base.get("feasible"), (i, r.name)
            assert rec.get("totals") == base.get("totals"), (i, r.name)
            assert annotations(r.store, ps, 0) == annotations(runs[0].store, bps, 0), (i, r.name)
        if base["chosen"] >= 0:
            placed = copy.copy(pod)
            placed.node_name = names0[base["chosen"]]
            world_pods[(pod.namespace, pod.name)] = placed
        if on_step is not None:
            on_step(i)
    return events


def same_node_state(runs: List[Run]) -> None:
    """Node aggregates by node name, every run against the first."""
    def by_name(r):
        st = r.b.node_state()
        return {k: dict(zip(r.sync.cluster.node_names, np.asarray(v).tolist())) for k, v in st.items()}
    ref = by_name(runs[0])
    for r in runs[1:]:
        got = by_name(r)
        for k in ref:
            assert got[k] == ref[k], (r.name, k)
