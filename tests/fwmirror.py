"""A mirror of upstream's scheduling framework driving the wrapped plugins
(TEST INFRASTRUCTURE: it plays [upstream] k8s.io/kubernetes v1.26.2
pkg/scheduler, which the Go host keeps; not product code).

What it reproduces of schedule_one.go / framework/runtime / parallelize:

  findNodesThatPassFilters   Parallelizer(16).Until over the scan set from
                             nextStartNodeIndex, chunked as chunkSizeFor(n, 16),
                             workers racing: every worker takes chunks in order,
                             checks ctx.Done() before each piece, and a piece
                             may be in flight while another worker cancels, so
                             several feasible nodes past the K-th can be
                             evaluated (recorded, then dropped);
                             nextStartNodeIndex += feasible + failed;
  PreFilterResult            its node set in Go map order (shuffled);
  prioritizeNodes            PreScore / Score / NormalizeScore over the feasible
                             list in completion order, weights (0 -> 1);
  selectHost                 reservoir sampling, rand.Intn(cnt) == 0 replaces,
                             over a seeded random.Random (or TB, the engine's
                             deterministic rule, for the parallelism-1 check);
  Reserve / Unreserve        the framework's node;
  PostFilter                 DefaultPreemption over NodeToStatusMap.
  PodNominator               nominated pods (queue.AddNominatedPod after a
                             PostFilter nomination; deleted when the pod is
                             assumed, cleared by ModeOverride "" and by
                             prepareCandidate for lower-priority pods nominated
                             on the chosen node); RunFilterPluginsWithNominated
                             Pods' two passes (each recorded, the second's
                             calls overwriting the first's in the store);
                             evaluateNominatedNode before the scan;
                             PodEligibleToPreemptOthers (a terminating
                             lower-priority pod on the nominated node blocks).
  victims                    deleted with the default grace period: with no
                             kubelet in the simulator they stay Terminating,
                             bound and counted (``terminating``).

The wrapper recording (simulator/scheduler/plugin/wrappedplugin.go) goes into
a ksim.resultstore.Store as the Go wrapper does, per plugin call.  The random
interleaving is drawn from ``seed`` only and from the plugins' answers, so two
runs with plugin sets that answer alike make identical choices.
"""
from __future__ import annotations

import math
import random
from typing import Dict, List, Optional, Set

from ksim import abi
from ksim.fwplugins import ERROR, EnginePlugins, Status
from ksim.profile import SchedulerProfile, num_feasible_nodes_to_find, original_name
from ksim.resultstore import PASSED_FILTER_MESSAGE, SUCCESS_MESSAGE, Store
from ksim.wrapped import HAS_NORMALIZE


def chunk_size_for(n: int, parallelism: int) -> int:
    """parallelize.chunkSizeFor (v1.26)."""
    s = int(math.sqrt(n))
    r = n // parallelism + 1
    if s > r:
        s = r
    return max(s, 1)


class Framework:
    def __init__(self, plugins: EnginePlugins, prof: SchedulerProfile, store: Store, seed: int = 0,
                 parallelism: int = 16, tie: str = "reservoir", tb_seed: int = 0):
        self.pl = plugins
        self.prof = prof
        self.store = store
        self.rng = random.Random(seed)
        self.parallelism = parallelism
        self.tie = tie
        self.tb_seed = tb_seed
        self.next_start = 0
        self.pod_seq = 0
        self.weights = {p.name: (p.weight or 1) for p in prof.score_plugins()}
        self.log: List[dict] = []
        self.nominator: Dict[int, int] = {}      # pod index -> nominated node (insertion order)
        self.nom_prio: Dict[int, int] = {}
        self.terminating: Set[int] = set()       # bound-table indices deleted by preemption

    @property
    def names(self):
        """The snapshot's node names (they move with node deltas)."""
        return self.pl.cluster.node_names

    # ---- PodNominator ---------------------------------------------------------
    def nominate(self, index: int, node: int, priority: int) -> None:
        self.nominator.pop(index, None)
        self.nominator[index] = node
        self.nom_prio[index] = priority

    def _nominated_view(self, index: int, priority: int) -> Dict[int, List[int]]:
        """addNominatedPods' choice per node: priority >= the pod's, itself excluded."""
        out: Dict[int, List[int]] = {}
        for j, node in self.nominator.items():
            if j != index and self.nom_prio[j] >= priority:
                out.setdefault(node, []).append(j)
        return out

    def _filter_node(self, node: int, ns: str, name: str) -> Status:
        """RunFilterPluginsWithNominatedPods, each pass's plugin calls recorded."""
        def record(ran):
            for pl, s in ran:                     # wrappedPlugin.Filter records each call
                self.store.add_filter_result(ns, name, self.names[node], pl,
                                             PASSED_FILTER_MESSAGE if s.is_success() else s.message)
        if self.pl.has_nominated(node):
            st, ran = self.pl.run_filter_plugins(node, nominated=True)
            record(ran)
            if not st.is_success():
                return st
        st, ran = self.pl.run_filter_plugins(node)
        record(ran)
        return st

    # ---- findNodesThatPassFilters (racing Parallelizer) ------------------------
    def _race(self, nodes: List[int], k: int, ns: str, name: str, status_map: Optional[dict] = None):
        n = len(nodes)
        feasible: List[int] = []
        status_map = {} if status_map is None else status_map
        evaluated: List[int] = []
        state = {"length": 0, "cancel": False, "error": None}
        chunk = chunk_size_for(n, self.parallelism)
        chunks = list(range((n + chunk - 1) // chunk))
        workers = [{"chunk": None, "p": None, "end": None, "flight": None, "done": False}
                   for _ in range(min(self.parallelism, len(chunks)))]
        slots = [None] * k

        def check_node(i: int):
            node = nodes[(self.next_start + i) % n]
            evaluated.append(node)
            st = self._filter_node(node, ns, name)
            if st.code == ERROR:
                if state["error"] is None:
                    state["error"] = st
                state["cancel"] = True
                return
            if st.is_success():
                state["length"] += 1
                if state["length"] > k:
                    state["cancel"] = True
                    state["length"] -= 1
                else:
                    slots[state["length"] - 1] = node
            else:
                status_map[node] = st

        while True:
            live = [w for w in workers if not w["done"]]
            if not live:
                break
            w = self.rng.choice(live)
            if w["flight"] is not None:           # finish the piece that passed the ctx check
                p, w["flight"] = w["flight"], None
                check_node(p)
                continue
            if w["p"] is None or w["p"] >= w["end"]:
                if not chunks:
                    w["done"] = True
                    continue
                c = chunks.pop(0)
                w["p"], w["end"] = c * chunk, min(n, (c + 1) * chunk)
            if state["cancel"]:                   # select { case <-stop: return }
                w["done"] = True
                continue
            w["flight"] = w["p"]
            w["p"] += 1
        feasible = slots[:state["length"]]
        return feasible, status_map, evaluated, state["error"]

    # ---- selectHost -----------------------------------------------------------
    def _select(self, lst: List[int], totals: List[int], seq: int) -> int:
        if self.tie == "tb":
            from oracle.objref import tb_key
            best = max(range(len(lst)), key=lambda j: tb_key(totals[j], self.tb_seed, seq, lst[j]))
            return lst[best]
        best, sel, cnt = totals[0], lst[0], 1
        for node, t in zip(lst[1:], totals[1:]):
            if t > best:
                best, sel, cnt = t, node, 1
            elif t == best:
                cnt += 1
                if self.rng.randrange(cnt) == 0:
                    sel = node
        return sel

    # ---- scheduleOne ----------------------------------------------------------
    def schedule_one(self, pods, index: int, priority: int = 0, bound=None) -> dict:
        ns, name = pods.names[index]
        rec = {"pod": index, "chosen": -1, "status": abi.STATUS_UNSCHEDULABLE, "nominated": -1}
        self.log.append(rec)
        st, names = self.pl.pre_filter(pods, index, self._nominated_view(index, priority))
        conflict = not st.is_success() and st.code != ERROR   # RunPreFilterPlugins stops at st.failed_plugin
        for p in self.prof.plugins["preFilter"].enabled:
            plugin = original_name(p.name)
            if conflict and plugin == st.failed_plugin:
                self.store.add_pre_filter_result(ns, name, plugin, st.message, None)
                break
            if plugin == "NodeAffinity" and names is not None:
                self.store.add_pre_filter_result(ns, name, plugin, SUCCESS_MESSAGE, list(names))
            else:
                self.store.add_pre_filter_result(ns, name, plugin, SUCCESS_MESSAGE, None)
        seq = self.pod_seq                        # the tie-break sequence of this cycle
        self.pod_seq += 1
        if st.code == ERROR:
            rec["status"], rec["chosen"] = abi.STATUS_ERROR, abi.CHOSEN_ERROR
            return rec
        if conflict:
            for p in self.prof.plugins["postFilter"].enabled:
                self.store.add_post_filter_result(ns, name, "", original_name(p.name), list(self.names))
            return rec
        pos = self.pl.pos
        if names is None:
            nodes = list(range(len(self.names)))
        else:
            nodes = sorted(pos[x] for x in names)
            if self.tie != "tb":
                self.rng.shuffle(nodes)           # Go map iteration order of PreFilterResult.NodeNames
        status_map = {}
        mine = self.nominator.get(index)
        feasible = []
        if mine is not None:
            # evaluateNominatedNode: the pod's nominated node first, whatever the
            # PreFilterResult; passing, it is the only feasible node (no scoring,
            # nextStartNodeIndex untouched); failing, its status stays in the
            # diagnosis (and counts in processedNodes)
            nst = self._filter_node(mine, ns, name)
            rec["nominated_eval"] = mine
            if nst.is_success():
                feasible = [mine]
                rec["evaluated"], rec["feasible"], rec["failed"] = [mine], [mine], []
                rec["next_start"] = self.next_start
            elif nst.code != ERROR:
                status_map[mine] = nst
        if not feasible:
            k = num_feasible_nodes_to_find(len(nodes), self.prof.percentage_of_nodes_to_score)
            feasible, status_map, evaluated, err = self._race(nodes, k, ns, name, status_map)
            rec["evaluated"] = evaluated
            processed = len(feasible) + len(status_map)
            self.next_start = (self.next_start + processed) % len(nodes)
            rec["next_start"] = self.next_start
            rec["feasible"] = list(feasible)
            rec["failed"] = list(status_map)
            if err is not None:
                rec["status"], rec["chosen"] = abi.STATUS_ERROR, abi.CHOSEN_ERROR
                return rec
        if not feasible:
            for p in self.prof.plugins["postFilter"].enabled:
                nom = -1
                if original_name(p.name) == "DefaultPreemption" and bound is not None:
                    nom = self._post_filter(index, priority, bound, status_map, rec)
                rec["nominated"] = nom
                self.store.add_post_filter_result(ns, name, self.names[nom] if nom >= 0 else "",
                                                  original_name(p.name), [self.names[x] for x in status_map])
            return rec
        if len(feasible) == 1:
            chosen = feasible[0]
        else:
            splugins = self.prof.score_plugins()
            if not splugins:
                totals = [1] * len(feasible)
            else:
                for p in self.prof.plugins["preScore"].enabled:
                    self.store.add_pre_score_result(ns, name, original_name(p.name), SUCCESS_MESSAGE)
                pst = self.pl.pre_score(feasible)
                if pst.code == ERROR:
                    rec["status"], rec["chosen"] = abi.STATUS_ERROR, abi.CHOSEN_ERROR
                    return rec
                totals = [0] * len(feasible)
                for p in splugins:
                    raws = [self.pl.score(p.name, x) for x in feasible]
                    for x, v in zip(feasible, raws):
                        self.store.add_score_result(ns, name, self.names[x], p.name, v)
                    vals = raws
                    if p.name in HAS_NORMALIZE:
                        vals = self.pl.normalize_score(p.name, feasible, raws)
                        for x, v in zip(feasible, vals):
                            self.store.add_normalized_score_result(ns, name, self.names[x], p.name, v)
                    for j, v in enumerate(vals):
                        totals[j] += v * self.weights[p.name]
            chosen = self._select(feasible, totals, seq)
            rec["totals"] = dict(zip(feasible, totals))
        # assume (the engine's reserve hook, unrecorded), then the wrapped Reserve
        # plugins; the assumed pod leaves the nominator (DeleteNominatedPodIfExists)
        self.pl.reserve(chosen)
        self.nominator.pop(index, None)
        for p in self.prof.plugins["reserve"].enabled:
            self.store.add_selected_node(ns, name, self.names[chosen])
            self.store.add_reserve_result(ns, name, original_name(p.name), SUCCESS_MESSAGE)
        for p in self.prof.plugins["preBind"].enabled:
            self.store.add_pre_bind_result(ns, name, original_name(p.name), SUCCESS_MESSAGE)
        for p in self.prof.plugins["bind"].enabled:
            self.store.add_bind_result(ns, name, original_name(p.name), SUCCESS_MESSAGE)
        rec["chosen"] = chosen
        rec["status"] = abi.STATUS_SCHEDULED
        return rec


    def _post_filter(self, index: int, priority: int, bound, status_map: dict, rec: dict) -> int:
        """DefaultPreemption.PostFilter with the queue's handling of its
        NominatingInfo; returns the node the wrapper records (-1: none)."""
        mine = self.nominator.get(index, -1)

        def terminating_lower(node, prio):        # the snapshot's DeletionTimestamp'd pods
            return any(int(bound.node[j]) == node and int(bound.priority[j]) < prio for j in self.terminating)
        pst, nom, victims, override = self.pl.post_filter(priority, bound, mine, status_map.get(mine),
                                                          terminating_lower)
        if not override:                          # nil result: ModeNoop, the nomination stays
            rec["eligible"] = False
            return -1
        rec["victims"] = victims
        if nom < 0:
            self.nominator.pop(index, None)       # ModeOverride "": the nomination is cleared
            return -1
        # prepareCandidate: the victims are deleted (Terminating from now on) and
        # lower-priority pods nominated on the node lose their nomination
        self.terminating.update(victims)
        for j in [j for j, n in self.nominator.items() if n == nom and self.nom_prio[j] < priority]:
            del self.nominator[j]
        self.nominate(index, nom, priority)
        return nom


class OracleBackend:
    """The C oracle's framework-mode calls under the engine's method names
    (ksim.fwplugins.EnginePlugins' backend protocol)."""

    def __init__(self, oracle, bound=None):
        self.o = oracle
        self.bound = bound

    # the snapshot calls (ksim.fwsnapshot.SnapshotSync's backend protocol)
    def set_cluster(self, cluster):
        from oracle.oracle import Oracle
        prof = self.o.profile
        self.o.close()
        self.o = Oracle(cluster, prof)

    def upsert_nodes(self, cluster, old_pos):
        self.o.upsert_nodes(cluster, old_pos)

    def update_node_rows(self, cluster, rows):
        """The oracle has no row update: the table again, every node kept
        (ksim_oracle_upsert_nodes, the same state)."""
        import numpy as np
        self.o.upsert_nodes(cluster, np.arange(cluster.n_nodes, dtype=np.int32))

    def node_state(self):
        return self.o.node_state()

    def fw_prefilter(self, pods, index):
        return self.o.fw_prefilter(pods, index)

    def fw_score(self, nodes):
        return self.o.fw_score(nodes)

    def fw_normalize(self, slot, nodes, scores):
        return self.o.fw_normalize(slot, nodes, scores)

    def assume(self, pods, index, node):
        self.o.assume(pods, index, node, 1)

    def forget(self, pods, index, node):
        self.o.assume(pods, index, node, -1)

    def fw_filter_nominated(self, pods, groups):
        return self.o.fw_filter_nominated(pods, groups)

    def preempt(self, pods, index, priority, bound=None, groups=None):
        return self.o.preempt(pods, index, priority, bound if bound is not None else self.bound, groups)


class EngineBackend:
    """ksim.engine.Engine with the bound-pod table argument the oracle takes."""

    def __init__(self, engine):
        self.e = engine
        self._bound = None

    def __getattr__(self, k):
        return getattr(self.e, k)

    def preempt(self, pods, index, priority, bound=None, groups=None):
        if bound is not None and bound is not self._bound:
            self.e.set_bound_pods(bound)
            self._bound = bound
        return self.e.preempt(pods, index, priority, groups)


def annotations(store: Store, pods, index: int) -> dict:
    """Every annotation AddStoredResultToPod would write for the pod."""
    ns, name = pods.names[index]
    out = {}
    store.add_stored_result_to_pod(ns, name, out)
    return out
