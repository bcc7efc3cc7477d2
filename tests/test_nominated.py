"""Nominated pods on the CPU: the framework mirror's
PodNominator (tests/fwmirror.py) over the C oracle's framework-mode answers
(ksim_oracle_fw_filter_nominated, ksim_oracle_preempt_nominated) against
oracle/objref.py's own restatement of upstream v1.26:

  RunFilterPluginsWithNominatedPods  objref.filter_with_nominated (the node
                                     cloned with the pods added, PTS / IPA
                                     PreFilter state recomputed on the clone);
  evaluateNominatedNode              objref.cycle(nominated_node=...);
  SelectVictimsOnNode's filter       objref.preempt(nominated=...);
  the queue's nominator bookkeeping  ObjQueue below, written apart from the
                                     mirror's.

One worker and the TB tie-break make the mirror's choices the deterministic
ones objref makes, so every cycle must agree: placement, nomination, victims,
nextStartNodeIndex and the failing nodes.  Parity against Go stays unpinned
(no fixture in the reference covers nominated pods)."""
import dataclasses

import numpy as np
import pytest

from ksim import gen, profile
from ksim.encode import encode_cluster, encode_pods
from ksim.fwplugins import EnginePlugins
from ksim.model import Container, Pod
from ksim.preemption import bound_table
from ksim.resultstore import Store
from oracle import objref
from oracle.objref import ObjScheduler
from oracle.oracle import Oracle

from fwmirror import Framework, OracleBackend
from test_preemption import crowded

# UnschedulableAndUnresolvable failures (fwplugins.filter_code by message)
_UNRESOLVABLE = {"NodeUnschedulable", "NodeName", "TaintToleration", "NodeAffinity", "VolumeBinding",
                 "VolumeZone"}


def _unresolvable(pl, msg) -> bool:
    if pl == "PodTopologySpread":
        return msg == objref.PTS_MISSING
    if pl == "InterPodAffinity":
        return msg == objref.IPA_AFF
    return pl in _UNRESOLVABLE


class ObjQueue:
    """The scheduling queue's PodNominator and DefaultPreemption's host side
    over objref: nominations in insertion order, cleared when the pod is
    assumed or when PostFilter finds no candidate (ModeOverride ""),
    prepareCandidate's clearing of lower-priority nominations on the chosen
    node, PodEligibleToPreemptOthers over the Terminating victims."""

    def __init__(self, ref: ObjScheduler, start, order):
        self.ref, self.start, self.order = ref, start, order
        self.nom = {}            # pod name -> node name
        self.pods = {}
        self.terminating = {}    # victim name -> priority, node

    def nominated(self):
        out = {}
        for name, node in self.nom.items():
            out.setdefault(node, []).append(self.pods[name])
        return out

    def schedule(self, pod: Pod, preempt: bool):
        self.pods[pod.name] = pod
        mine = self.nom.get(pod.name)
        r = self.ref.cycle(pod, nominated=self.nominated(), nominated_node=mine)
        if r["chosen"] is not None:
            self.nom.pop(pod.name, None)
            return r, None, None
        if not preempt or r.get("error"):
            return r, None, None
        if mine is not None:
            st = r["filter"].get(mine)
            if st is None or not _unresolvable(*st):
                if any(node == mine and prio < pod.priority for prio, node in self.terminating.values()):
                    return r, None, "ineligible"
        node, victims = self.ref.preempt(pod, pod.priority, self.start, self.order, nominated=self.nominated())
        if node is None:
            self.nom.pop(pod.name, None)
            return r, None, None
        for v in victims:
            q = next(pi.pod for pi in self.ref.by_name[node].pods if pi.pod.name == v)
            self.terminating[v] = (q.priority, node)
        for other in [o for o, n in self.nom.items() if n == node and self.pods[o].priority < pod.priority]:
            del self.nom[other]
        self.nom.pop(pod.name, None)
        self.nom[pod.name] = node
        return r, node, victims


def _compare(rec, r, nom, victims, names, bound_names, where):
    got = names[rec["chosen"]] if rec["chosen"] >= 0 else None
    assert got == r["chosen"], f"{where}: mirror {got} objref {r['chosen']}"
    gn = names[rec["nominated"]] if rec["nominated"] >= 0 else None
    assert gn == nom, f"{where}: nominated mirror {gn} objref {nom}"
    if nom is not None:
        assert [bound_names[v] for v in rec["victims"]] == victims, where
    if "failed" in rec:
        failed = {n for n, (pl, _) in r["filter"].items() if pl is not None}
        assert {names[x] for x in rec["failed"]} == failed, f"{where}: failing nodes"


@pytest.mark.parametrize("seed", [3, 7])
def test_preemption_nominations_vs_objref(seed):
    """Preemptors nominated, their victims left Terminating (no kubelet), the
    nominated pods re-queued: lower / equal-priority pods see the nominated
    pods' requests on their node (pass 1), the preemptor re-evaluates its node
    first and is refused a second preemption while its victims terminate."""
    nodes, bound, start, order = crowded(n_nodes=150, seed=seed)
    cluster, _ = encode_cluster(nodes, bound)
    table = bound_table(cluster, bound, start)
    rng = np.random.default_rng(seed + 50)
    pods = [Pod(f"p{i}", priority=int(rng.choice([0, 5, 50, 500, 5000])),
                containers=[Container({"cpu": f"{int(rng.integers(5, 300)) * 100}m",
                                       "memory": f"{int(rng.integers(2, 30))}Gi"})]) for i in range(90)]
    enc = encode_pods(cluster, pods)
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=0)
    prof = profile.compile_profile(sp)
    ora = Oracle(cluster.copy_state(), prof)
    fw = Framework(EnginePlugins(OracleBackend(ora, table), cluster, sp), sp, Store(profile.default_score_weights()),
                   parallelism=1, tie="tb", tb_seed=sp.tiebreak_seed)
    q = ObjQueue(ObjScheduler(nodes, bound, pct=0, seed=sp.tiebreak_seed), start, order)
    names = cluster.node_names
    placed = list(bound)                  # the snapshot's pods: the dry run's victims come from them
    stats = {"nominated": 0, "two_pass": 0, "nominated_eval": 0, "ineligible": 0, "scheduled_on_nom": 0}
    queue = list(range(len(pods)))
    retries = []
    step = 0
    while queue:
        i = queue.pop(0)
        rec = fw.schedule_one(enc, i, pods[i].priority, table)
        r, nom, victims = q.schedule(pods[i], preempt=True)
        where = f"step {step} pod {i}"
        _compare(rec, r, nom, victims, names, [p.name for p in placed], where)
        if r["chosen"] is not None:       # bound now, with a later start time
            placed.append(dataclasses.replace(pods[i], node_name=r["chosen"]))
            start[pods[i].name] = 100 + step
            order[pods[i].name] = len(order)
            table = bound_table(cluster, placed, start)   # rows append-only: victim indices stay
        assert fw.next_start == q.ref.next_start, where
        assert {names[n] for n in fw.nominator.values()} == set(q.nom.values()), where
        stats["nominated"] += nom is not None
        stats["ineligible"] += victims == "ineligible"
        stats["nominated_eval"] += "nominated_eval" in rec
        stats["scheduled_on_nom"] += rec.get("nominated_eval") == rec["chosen"]
        stats["two_pass"] += any(fw.pl.has_nominated(x) for x in rec.get("evaluated", []))
        if nom is not None and step < 200:
            retries.append(i)
        if len(retries) >= 3 or (not queue and retries):   # the requeued preemptors come back
            queue.extend(retries)
            retries = []
        step += 1
    a = ora.node_state()
    for pos, name in enumerate(names):
        ni = q.ref.by_name[name]
        assert a["req_cpu"][pos] == ni.requested.get("cpu", 0) and a["num_pods"][pos] == len(ni.pods), name
    assert stats["nominated"] > 5 and stats["two_pass"] > 5 and stats["nominated_eval"] > 5, stats
    assert stats["ineligible"] > 0, stats


@pytest.mark.parametrize("pct", [0, 100])
def test_seeded_nominations_with_topology_vs_objref(pct):
    """Nominations seeded on incoming pods that spread (PodTopologySpread
    DoNotSchedule over zones) and prefer apart: the first pass carries their
    AddPod updates into the PTS / IPA PreFilter state of the nominated node,
    then the seeded pods come back and try their nominated node first."""
    nodes, bound, incoming = gen.config3_objects(n_nodes=120, pods_per_node=3, n_incoming=150)
    cluster, _ = encode_cluster(nodes, bound)
    enc = encode_pods(cluster, incoming)
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=pct)
    prof = profile.compile_profile(sp)
    ora = Oracle(cluster.copy_state(), prof)
    fw = Framework(EnginePlugins(OracleBackend(ora), cluster, sp), sp, Store(profile.default_score_weights()),
                   parallelism=1, tie="tb", tb_seed=sp.tiebreak_seed)
    ref = ObjScheduler(nodes, bound, pct=pct, seed=sp.tiebreak_seed)
    q = ObjQueue(ref, {}, {})
    names = cluster.node_names
    rng = np.random.default_rng(pct + 1)
    seeded = list(range(30))
    for j in seeded:                      # a zone's worth of nominations piled on few nodes
        node = int(rng.integers(0, 12)) * 3
        fw.nominate(j, node, incoming[j].priority)
        q.pods[incoming[j].name] = incoming[j]
        q.nom[incoming[j].name] = names[node]
    two_pass = diff_first = 0
    for step, i in enumerate(list(range(30, len(incoming))) + seeded):
        rec = fw.schedule_one(enc, i, incoming[i].priority)
        r, _, _ = q.schedule(incoming[i], preempt=False)
        where = f"step {step} pod {i}"
        _compare(rec, r, None, None, names, [], where)
        assert fw.next_start == ref.next_start, where
        ev = [x for x in rec.get("evaluated", []) if fw.pl.has_nominated(x)]
        two_pass += bool(ev)
        for x in ev:                      # the first pass decided differently from the second
            diff_first += fw.pl._nom[x][0] != int(fw.pl._filter["fail_plugin"][x])
    assert two_pass > 20 and diff_first > 0, (two_pass, diff_first)
    assert not fw.nominator or all(j in seeded for j in fw.nominator)
