"""The drop-in's incremental snapshot: informer events -> engine deltas.

The Python mirror of integration/go/engine/encoder.go NativeEncoder (the
informer handlers, Snapshot, Assume / Forget).  The reference's scheduler runs
off informers (simulator/scheduler/scheduler.go:160-167): node and pod events
reach the scheduler cache, the framework's Reserve assumes the cycle's pod in
it, and each cycle starts from UpdateSnapshot, which copies only what changed.
The engine's device-resident snapshot follows the same events through the
encoder's delta calls (include/ksim_engine.h "snapshot deltas", ABI 11):

  node added / updated / removed   ksim_encoder_update_nodes, then
                                   ksim_update_node_rows when the delta moved no node
                                   and added no vocabulary (ksim_encoder_changed_rows),
                                   else ksim_upsert_nodes (the engine replays its binds
                                   on kept nodes); one per cycle start;
  bound pod added                  ksim_encode_pods of the pod, the table re-sent
                                   when the compile grew it, ksim_assume,
                                   ksim_encoder_bind;
  bound pod deleted                ksim_encode_pods, re-send rule, ksim_forget,
                                   ksim_encoder_unbind;
  Reserve / Unreserve              the cycle's pod, as a bound pod added / deleted.

Events queue between cycles and are applied at the next cycle start
(``cycle``), node events first.  A pod event for a node the snapshot does not
hold yet waits for the node.  The whole snapshot is encoded once, at
construction (``stats["full_encodes"]``), and again only when a delta cannot
be encoded (a vocabulary or class limit): the host's own record of the nodes
and bound pods is re-encoded then and sent with ksim_set_cluster.
"""
from __future__ import annotations

import copy
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .encode import EncodeError
from .model import Node, Pod
from .nativeenc import NativeEncoder


def _bound_copy(pod: Pod, node: str) -> Pod:
    if pod.node_name == node:
        return pod
    p = copy.copy(pod)
    p.node_name = node
    return p


class SnapshotSync:
    """The engine's snapshot kept in step with the cluster by events.

    ``backend``: set_cluster(cluster), upsert_nodes(cluster, old_pos),
    assume(pods, index, node), forget(pods, index, node) (ksim.engine.Engine,
    or the oracle's framework binding in the tests).  ``pod_args``: the
    profile's compile options (added_affinity, spread), as encode_pods takes."""

    def __init__(self, backend, nodes: Sequence[Node], bound: Sequence[Pod] = (),
                 namespaces: Optional[Dict[str, Dict[str, str]]] = None, nb_args=None, extra_scalar=(),
                 pod_args: Optional[dict] = None):
        self.b = backend
        self.namespaces = dict(namespaces or {})
        self.nb_args = nb_args
        self.extra_scalar = list(extra_scalar)
        self.pod_args = dict(pod_args or {})
        self.nodes: Dict[str, Node] = {}          # informer add order
        for n in nodes:
            self.nodes[n.name] = n
        self.bound: Dict[Tuple[str, str], Tuple[Pod, str]] = {}   # (namespace, name) -> (pod, node)
        for p in bound:
            if p.node_name in self.nodes:
                self.bound[(p.namespace, p.name)] = (p, p.node_name)
        self.waiting: Dict[Tuple[str, str], Pod] = {}             # bound to a node not yet added
        self.events: List[tuple] = []
        self.stats = {"full_encodes": 0, "node_deltas": 0, "node_rows_in_place": 0, "pod_adds": 0,
                      "pod_deletes": 0, "resends": 0, "reserves": 0, "unreserves": 0}
        self._encodes = 0
        self._cycle: Optional[Pod] = None
        self._cycle_set = None
        self._assumed: Optional[Tuple[Pod, int]] = None
        self._full()

    # ---- the snapshot ----------------------------------------------------------
    def _full(self) -> None:
        self.enc = NativeEncoder()
        bound = [_bound_copy(p, node) for p, node in self.bound.values()]
        cluster, _ = self.enc.encode_cluster(list(self.nodes.values()), bound, namespaces=self.namespaces,
                                             nb_args=self.nb_args, extra_scalar=self.extra_scalar)
        self.b.set_cluster(cluster)
        self._use(cluster)
        self.stats["full_encodes"] += 1

    def _use(self, cluster) -> None:
        self.cluster = cluster
        self.pos = {n: i for i, n in enumerate(cluster.node_names)}
        self._layout = (cluster.n_label_cols, int(cluster.class_count.shape[0]))
        self._cycle_set = None

    def _resend(self) -> None:
        """The compile added label columns or count classes: the table again,
        every node kept (their rows replay the device's binds)."""
        c = self.cluster
        layout = (c.n_label_cols, int(c.class_count.shape[0]))
        if layout != self._layout:
            self.b.upsert_nodes(c, np.arange(c.n_nodes, dtype=np.int32))
            self._layout = layout
            self.stats["resends"] += 1

    def _encode(self, pod: Pod):
        self._encodes += 1                         # the encoder's pod set (ksim_encoder_bind's reference) changes
        return self.enc.encode_pods(self.cluster, [pod], **self.pod_args)

    # ---- informer events ----------------------------------------------------------
    def add_node(self, node: Node) -> None:
        self.events.append(("node", node))

    def update_node(self, node: Node) -> None:
        self.events.append(("node", node))

    def remove_node(self, name: str) -> None:
        self.events.append(("node-", name))

    def add_pod(self, pod: Pod) -> None:
        """An informer Add (or an Update that bound the pod); unbound pods are the queue's."""
        if pod.node_name:
            self.events.append(("pod", pod))

    def update_pod(self, old: Pod, new: Pod) -> None:
        if old.node_name and new.node_name == old.node_name and new is old:
            return
        if old.node_name:
            self.events.append(("pod-", old))
        if new.node_name:
            self.events.append(("pod", new))

    def delete_pod(self, pod: Pod) -> None:
        self.events.append(("pod-", pod))

    # ---- applying them (the next cycle start) -----------------------------------------
    def snapshot(self) -> None:
        ev, self.events = self.events, []
        pods = [(k, x) for k, x in ev if k in ("pod", "pod-")]
        done = 0
        try:
            nodes = [(k, x) for k, x in ev if k in ("node", "node-")]
            if nodes:
                self._apply_nodes(nodes)
            for k, x in pods:
                if k == "pod":
                    self._pod_added(x)
                else:
                    self._pod_deleted(x)
                done += 1
            for key, p in list(self.waiting.items()):
                if p.node_name in self.pos:
                    del self.waiting[key]
                    self._pod_added(p)
        except EncodeError:
            # a limit the delta cannot meet: the rest of the events into the
            # host's record, and the record encoded whole
            for k, x in pods[done:]:
                self._record_pod(k, x)
            self._full()

    def _record_nodes(self, ev) -> Tuple[List[Node], List[str]]:
        """The node events into the host's record (informer add order, the
        bound pods of removed nodes dropped); returns (added or updated nodes,
        removed names) for the encoder."""
        from .encode import zone_key
        upserts: Dict[str, Node] = {}
        removed: List[str] = []
        for k, x in ev:
            if k == "node":
                upserts[x.name] = x
            else:
                upserts.pop(x, None)
                if x in self.nodes and x not in removed:
                    removed.append(x)
        for name in removed:
            del self.nodes[name]
            for key in [key for key, (_, node) in self.bound.items() if node == name]:
                del self.bound[key]                # the node's pods leave the snapshot with it
        for name, n in upserts.items():
            if name in self.nodes and zone_key(self.nodes[name].labels) != zone_key(n.labels):
                del self.nodes[name]               # nodeTree.updateNode: re-added at the end
            self.nodes[name] = n
        return list(upserts.values()), removed

    def _record_pod(self, k: str, x: Pod) -> None:
        key = (x.namespace, x.name)
        if k == "pod-":
            self.bound.pop(key, None)
            self.waiting.pop(key, None)
        elif x.node_name in self.nodes:
            self.bound[key] = (x, x.node_name)
        else:
            self.waiting[key] = x

    def _apply_nodes(self, ev) -> None:
        upserts, removed = self._record_nodes(ev)
        cluster, old_pos, rows = self.enc.update_nodes(upserts, removed)
        if rows is not None:                       # in place: the rows' static columns only
            self.b.update_node_rows(cluster, rows)
            self.stats["node_rows_in_place"] += 1
        else:
            self.b.upsert_nodes(cluster, old_pos)
        self._use(cluster)
        self.stats["node_deltas"] += 1

    def _pod_added(self, pod: Pod) -> None:
        key = (pod.namespace, pod.name)
        have = self.bound.get(key)
        if have is not None:
            if have[1] == pod.node_name:
                return                             # the engine's own Reserve, seen again by the informer
            self._pod_deleted(have[0])
        if pod.node_name not in self.pos:
            self.waiting[key] = pod
            return
        node = self.pos[pod.node_name]
        ps = self._encode(pod)
        self._resend()
        self.b.assume(ps, 0, node)
        self.enc.bind(0, node)
        self.bound[key] = (pod, pod.node_name)
        self.stats["pod_adds"] += 1

    def _pod_deleted(self, pod: Pod, stat: str = "pod_deletes") -> None:
        key = (pod.namespace, pod.name)
        self.waiting.pop(key, None)
        have = self.bound.get(key)
        if have is None:
            return
        ps = self._encode(have[0])                 # the pod as it was bound: the adds it made
        self._resend()
        node = self.enc.unbind(key[0], key[1])
        self.b.forget(ps, 0, node)
        del self.bound[key]
        self.stats[stat] += 1

    # ---- the cycle ----------------------------------------------------------------------
    def cycle(self, pod: Pod):
        """Cycle start (NativeEncoder.Snapshot + Pod + Resync): queued events
        applied, the pod compiled against the snapshot; returns its pod set."""
        self.snapshot()
        ps = self._encode(pod)
        self._resend()
        self._cycle, self._cycle_set = pod, (ps, self._encodes)
        return ps

    def assume(self, node: int) -> None:
        """KsimAssume.Reserve: the cycle's pod on the framework's node."""
        pod = self._cycle
        ps = None
        if self._cycle_set is not None and self._cycle_set[1] == self._encodes:
            ps = self._cycle_set[0]
        if ps is None:                             # the encoder compiled something else since
            ps = self._encode(pod)
            self._resend()
        self.b.assume(ps, 0, node)
        self.enc.bind(0, node)
        self.bound[(pod.namespace, pod.name)] = (pod, self.cluster.node_names[node])
        self._assumed = (pod, node)
        self._cycle_set = None
        self.stats["reserves"] += 1

    def forget(self) -> None:
        """KsimAssume.Unreserve: forget only what Reserve assumed."""
        if self._assumed is None:
            return
        pod, _ = self._assumed
        self._assumed = None
        self._pod_deleted(pod, "unreserves")

    def bound_pods(self) -> List[Pod]:
        """The snapshot's bound pods (spec.nodeName set), in bind order."""
        return [_bound_copy(p, node) for p, node in self.bound.values()]
