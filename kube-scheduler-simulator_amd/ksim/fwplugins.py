"""Engine-backed framework plugins: the Python mirror of the Go adapter in
integration/go/engine/plugins.go.

In the reference every in-tree plugin is built by the factory closure at
simulator/scheduler/plugin/plugins.go:75-87 and wrapped by NewWrappedPlugin
(:86).  The engine replaces the ORIGINAL plugin ``p`` of that closure; the
wrapper (wrappedplugin.go) and the result store stay as they are.  The
framework, not the engine, then decides:

  * which nodes Filter runs on: 16 racing Parallelizer workers stop after
    numFeasibleNodesToFind feasible nodes (simulator/scheduler/scheduler.go:
    149,153 pin parallelism 16 and percentageOfNodesToScore 0);
  * the feasible list PreScore / Score / NormalizeScore see;
  * the node Reserve records (selectHost's reservoir over math/rand).

So the plugins answer under those choices (ksim_engine.h "framework-driven
compat mode"):

  PreFilter       the first wrapped PreFilter of a cycle calls ksim_fw_prefilter:
                  Filter of every node of the pod's scan set on the device
                  (wrappedplugin.go:459-486);
  Filter(node)    a read of that pass: plugin k of the profile's Filter order
                  fails on the node iff the pass stopped at k (RunFilterPlugins
                  calls k only after 0..k-1 passed)  (:491-516);
  PreScore(list)  the first wrapped PreScore calls ksim_fw_score(list)  (:427-454);
  Score(node)     raw[slot][node]  (:388-413);
  NormalizeScore  ksim_fw_normalize over the NodeScoreList it is handed  (:356-375);
  Reserve(node)   ksim_assume on the framework's node; Unreserve ksim_forget
                  (:583-584, 617);
  PostFilter      DefaultPreemption's dry run, ksim_preempt: the nominated node
                  (:518-538, Store.AddPostFilterResult store.go:437-452).

Nominated pods (RunFilterPluginsWithNominatedPods, framework.go v1.26): the
framework hands Filter a NodeInfo / CycleState clone carrying the node's
nominated pods of priority >= the pod's (PreFilterExtensions.AddPod); the
plugins answer that first pass from ksim_fw_filter_nominated, one call per
cycle over every such node, and the dry run from ksim_preempt_nominated.

One cycle is in flight at a time (upstream scheduleOne is serial); the wrapped
plugins of a profile share one ``EnginePlugins``.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import abi
from .profile import SchedulerProfile
from .wrapped import ERR_NODE_AFFINITY_CONFLICT, filter_message

# framework.Code
SUCCESS, ERROR, UNSCHEDULABLE, UNSCHEDULABLE_AND_UNRESOLVABLE, SKIP = 0, 1, 2, 3, 6

# filter plugins whose failures are UnschedulableAndUnresolvable in v1.26
_UNRESOLVABLE = {"NodeUnschedulable", "NodeName", "TaintToleration", "NodeAffinity", "VolumeBinding",
                 "VolumeZone"}


class Status:
    """framework.Status: a code and a message (nil status = SUCCESS)."""
    __slots__ = ("code", "message", "failed_plugin")

    def __init__(self, code: int = SUCCESS, message: str = "", failed_plugin: str = ""):
        self.code, self.message, self.failed_plugin = code, message, failed_plugin

    def is_success(self) -> bool:
        return self.code == SUCCESS

    def __repr__(self):
        return f"Status({self.code}, {self.message!r})"


def filter_code(plugin: str, detail: int) -> int:
    """The framework.Code of a failing Filter (upstream v1.26 plugin returns)."""
    if plugin == "NetworkBandwidth":
        return UNSCHEDULABLE if detail == abi.NB_INSUFFICIENT else ERROR
    if plugin == "PodTopologySpread":
        return UNSCHEDULABLE_AND_UNRESOLVABLE if detail == abi.PTS_MISSING_LABEL else UNSCHEDULABLE
    if plugin == "InterPodAffinity":
        return UNSCHEDULABLE_AND_UNRESOLVABLE if detail == abi.IPA_AFFINITY else UNSCHEDULABLE
    return UNSCHEDULABLE_AND_UNRESOLVABLE if plugin in _UNRESOLVABLE else UNSCHEDULABLE


class EnginePlugins:
    """The engine-backed plugin set of one profile.  ``backend`` is a
    ksim.engine.Engine (the product); tests pass the oracle's framework-mode
    binding (same method names) to get the reference answers under the same
    framework choices."""

    def __init__(self, backend, cluster, prof: SchedulerProfile, sync=None):
        self.b = backend
        self.sync = sync
        self._cluster = cluster if sync is None else None
        self.prof = prof
        self.forder = prof.filter_order()
        self.snames = [p.name for p in prof.score_plugins()]
        self._pos = {n: i for i, n in enumerate(cluster.node_names)} if sync is None else None
        self._pods = None
        self._idx = -1
        self._filter: Optional[Dict] = None
        self._score: Optional[Dict] = None

    @property
    def cluster(self):
        """The snapshot the answers refer to (the SnapshotSync's current one)."""
        return self._cluster if self.sync is None else self.sync.cluster

    @property
    def pos(self) -> Dict[str, int]:
        return self._pos if self.sync is None else self.sync.pos

    def begin(self, pod):
        """Cycle start with an incremental snapshot (plugins.go ensureFilter:
        Encoder.Snapshot, Pod, Resync): the queued informer events applied,
        the pod compiled; returns its one-pod set for ``pre_filter``."""
        return self.sync.cycle(pod)

    # ---- PreFilter / Filter ---------------------------------------------------
    def pre_filter(self, pods, index: int, nominated: Optional[Dict[int, List[int]]] = None
                   ) -> Tuple[Status, Optional[List[str]]]:
        """The engine's PreFilter pass; returns NodeAffinity's status and
        PreFilterResult.NodeNames (None = all nodes).  ``nominated``: {node:
        [indices of ``pods``]}, the nominated pods addNominatedPods would add
        for this pod (priority >= its own, itself excluded)."""
        self._pods, self._idx = pods, index
        self._score = None
        self._groups = [(n, list(v)) for n, v in (nominated or {}).items() if v]
        self._nom: Dict[int, Tuple[int, int]] = {}
        names = pods.prefilter_names[index] if pods.prefilter_names else None
        rej = pods.rejection(index)
        if rej is not None:                       # the original VolumeBinding's PreFilter answers
            self._filter = None
            return Status(UNSCHEDULABLE_AND_UNRESOLVABLE, rej[1], rej[0]), names
        if names is not None and len(names) == 0:
            self._filter = None
            return Status(UNSCHEDULABLE_AND_UNRESOLVABLE, ERR_NODE_AFFINITY_CONFLICT, "NodeAffinity"), []
        self._filter = self.b.fw_prefilter(pods, index)
        if self._filter["status"] == abi.STATUS_ERROR:
            return Status(ERROR, "node in PreFilterResult not found", "NodeAffinity"), names
        if self._groups:
            fp, fd = self.b.fw_filter_nominated(pods, self._groups)
            self._nom = {n: (int(fp[k]), int(fd[k])) for k, (n, _) in enumerate(self._groups)}
        return Status(), names

    def has_nominated(self, node: int) -> bool:
        """addNominatedPods added pods for ``node`` (the first pass runs)."""
        return node in self._nom

    def filter(self, plugin: str, node: int, nominated: bool = False) -> Status:
        """wrappedPlugin.Filter's original-plugin call for ``plugin`` on ``node``
        (``nominated``: on the clone carrying the node's nominated pods)."""
        k = self.forder.index(plugin)
        if nominated:
            r, d = self._nom[node]
        else:
            r = int(self._filter["fail_plugin"][node])
            d = int(self._filter["fail_detail"][node])
        if r == abi.NOT_EVALUATED:
            raise RuntimeError(f"Filter on node {node} outside the pod's scan set")
        if r == abi.PASSED or r != k:
            if r != abi.PASSED and r < k:
                raise RuntimeError(f"{plugin} called on node {node} after {self.forder[r]} failed")
            return Status()
        ns, name = self._pods.names[self._idx]
        msg = filter_message(self.cluster, plugin, d, self.cluster.node_names[node], name)
        return Status(filter_code(plugin, d), msg, plugin)

    def run_filter_plugins(self, node: int, nominated: bool = False) -> Tuple[Status, List[Tuple[str, Status]]]:
        """framework.RunFilterPlugins: the plugins in order up to the first
        non-success; returns the cycle status and each (plugin, status) run."""
        ran = []
        for pl in self.forder:
            st = self.filter(pl, node, nominated)
            ran.append((pl, st))
            if not st.is_success():
                return st, ran
        return Status(), ran

    # ---- PreScore / Score / NormalizeScore ------------------------------------
    def pre_score(self, nodes: Sequence[int]) -> Status:
        self._score = self.b.fw_score(np.asarray(nodes, np.int32))
        if self._score["status"] == abi.STATUS_ERROR:
            return Status(ERROR, "NetworkBandwidth Score failed")
        return Status()

    def score(self, plugin: str, node: int) -> int:
        return int(self._score["raw"][self.snames.index(plugin)][node])

    def normalize_score(self, plugin: str, nodes: Sequence[int], scores: Sequence[int]) -> List[int]:
        """NormalizeScore over exactly the NodeScoreList handed in."""
        return [int(x) for x in self.b.fw_normalize(self.snames.index(plugin), nodes, scores)]

    # ---- Reserve / Unreserve / PostFilter -------------------------------------
    def reserve(self, node: int) -> Status:
        """KsimAssume.Reserve: assume the cycle's pod on the framework's node;
        the pod set and index are kept for Unreserve (the Go adapter keeps an
        owned copy of the encoding: Unreserve may run after the next cycle)."""
        self._assumed = (self._pods, self._idx, node)
        if self.sync is not None:
            self.sync.assume(node)                # the device, and the snapshot's membership
        else:
            self.b.assume(self._pods, self._idx, node)
        return Status()

    def unreserve(self, node: int) -> None:
        """KsimAssume.Unreserve: forget only what Reserve assumed (a Reserve
        plugin failing before KsimAssume ran leaves nothing to undo)."""
        a = getattr(self, "_assumed", None)
        if a is None:
            return
        self._assumed = None
        if self.sync is not None:
            self.sync.forget()
        else:
            self.b.forget(a[0], a[1], a[2])

    def post_filter(self, priority: int, bound=None, nominated_node: int = -1, nominated_status=None,
                    terminating_lower=None) -> Tuple[Status, int, List[int], bool]:
        """DefaultPreemption.PostFilter (default_preemption.go v1.26):
        PodEligibleToPreemptOthers, then the dry run over this cycle's
        nominated groups.  Returns (status, nominated node or -1, victim
        indices of the bound-pod table, override): override False is a nil
        result (ModeNoop, the pod keeps its nomination), True with node -1 is
        NominatedNodeName "" (ModeOverride clears it).  ``terminating_lower(node,
        priority)``: a Terminating pod of lower priority is on the node."""
        if nominated_node >= 0 and (nominated_status is None or
                                    nominated_status.code != UNSCHEDULABLE_AND_UNRESOLVABLE):
            if terminating_lower is not None and terminating_lower(nominated_node, priority):
                return (Status(UNSCHEDULABLE, "preemption: not eligible due to a terminating pod on the "
                                              "nominated node."), -1, [], False)
        if bound is None:
            node, victims = self.b.preempt(self._pods, self._idx, priority, groups=self._groups)[:2]
        else:
            node, victims = self.b.preempt(self._pods, self._idx, priority, bound, groups=self._groups)[:2]
        if node < 0:
            return Status(UNSCHEDULABLE, "preemption: no candidate node"), -1, [], True
        return Status(), int(node), list(victims), True
