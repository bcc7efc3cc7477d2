"""Framework-driven compat mode on the GPU (ksim_fw_*): the engine answers the
wrapped plugins under the FRAMEWORK's own choices, as the simulator runs it
(parallelism 16, percentageOfNodesToScore 0: simulator/scheduler/
scheduler.go:149,153,231-241).  The framework mirror (tests/fwmirror.py) races
16 workers over the scan set, breaks ties by reservoir sampling and hands
Reserve its own node; the same mirror over the C oracle's answers, with the
same seed, must make the same choices and record the same annotations, and
both snapshots must end equal."""
import numpy as np
import pytest

from ksim import abi, gen, profile
from ksim.encode import encode_cluster, encode_pods
from ksim.engine import Engine
from ksim.fwplugins import EnginePlugins
from ksim.model import Container, Pod
from ksim.preemption import bound_table
from ksim.resultstore import Store
from oracle.oracle import Oracle

from fwmirror import EngineBackend, Framework, OracleBackend, annotations

pytestmark = pytest.mark.gpu


def _cases(kind):
    if kind == "config1":
        cluster, pods = gen.config1(n_nodes=300, n_pods=300)
        return cluster, pods, None, None
    if kind == "prefilter":
        nodes, pods_o = gen.prefilter_objects(n_nodes=300, n_pods=240)
        cluster, _ = encode_cluster(nodes, [])
        return cluster, encode_pods(cluster, pods_o), None, None
    if kind == "config3":
        nodes, bound, incoming = gen.config3_objects(n_nodes=400, pods_per_node=4, n_incoming=200)
        cluster, _ = encode_cluster(nodes, bound)
        return cluster, encode_pods(cluster, incoming), None, None
    if kind == "ipa":
        # InterPodAffinity only (no spread constraints): ksim_fw_score is
        # answered on the host from the filter pass's raw scores
        nodes, bound, incoming = gen.config3_objects(n_nodes=400, pods_per_node=4, n_incoming=200)
        for p in incoming:
            p.topology_spread = []
        cluster, _ = encode_cluster(nodes, bound)
        return cluster, encode_pods(cluster, incoming), None, None
    if kind == "preempt":
        # crowded config-1 nodes with bound pods of mixed priorities: many
        # cycles find no node and run DefaultPreemption's PostFilter
        rng = np.random.default_rng(11)
        nodes, _ = gen.config1_objects(n_nodes=160, n_pods=1)
        bound, start = [], {}
        for ni, n in enumerate(nodes):
            for k in range(6):
                nm = f"b{ni}-{k}"
                bound.append(Pod(nm, node_name=n.name, priority=int(rng.choice([0, 10, 100, 1000])),
                                 containers=[Container({"cpu": f"{int(rng.integers(2, 12)) * 100}m",
                                                        "memory": f"{int(rng.integers(1, 6))}Gi"})]))
                start[nm] = int(rng.integers(0, 50))
        cluster, _ = encode_cluster(nodes, bound)
        table = bound_table(cluster, bound, start)
        pods_o = [Pod(f"p{i}", priority=int(rng.choice([0, 5, 50, 500, 5000])),
                      containers=[Container({"cpu": f"{int(rng.integers(10, 300)) * 100}m",
                                             "memory": f"{int(rng.integers(2, 40))}Gi"})]) for i in range(120)]
        return cluster, encode_pods(cluster, pods_o), table, [p.priority for p in pods_o]
    if kind == "replicaset":
        # ReplicaSet / Service / StatefulSet-owned pods under the System default
        # spreading (requireAllTopologies = false) on nodes missing zone or
        # hostname labels
        from ksim.topology import SpreadDefaults
        from test_spread_defaults import WORKLOADS, mixed_nodes, workload_pods
        nodes = mixed_nodes(300, seed=4)
        bound = workload_pods(600, seed=12, bound_nodes=[n.name for n in nodes])
        cluster, _ = encode_cluster(nodes, bound)
        pods = encode_pods(cluster, workload_pods(300, seed=13),
                           spread=SpreadDefaults(profile.PodTopologySpreadArgs(), *WORKLOADS))
        assert (pods.pods["topo_flags"] & abi.POD_PTS_SYSTEM_DEFAULT).any()
        return cluster, pods, None, None
    raise ValueError(kind)


@pytest.mark.parametrize("kind", ["config1", "prefilter", "config3", "ipa", "preempt", "replicaset"])
@pytest.mark.parametrize("seed", [1, 2])
def test_framework_driven_cycles(kind, seed):
    cluster, pods, table, prio = _cases(kind)
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=0)
    prof = profile.compile_profile(sp)
    w = profile.default_score_weights()
    eng = Engine(0)
    eng.set_profile(prof)
    eng.set_cluster(cluster.copy_state())
    ora = Oracle(cluster.copy_state(), prof)
    se, so = Store(w), Store(w)
    fe = Framework(EnginePlugins(EngineBackend(eng), cluster, sp), sp, se, seed=seed)
    fo = Framework(EnginePlugins(OracleBackend(ora), cluster, sp), sp, so, seed=seed)
    raced = ties = nominated = 0
    for i in range(pods.n_pods):
        p = prio[i] if prio else 0
        re = fe.schedule_one(pods, i, p, table)
        ro = fo.schedule_one(pods, i, p, table)
        for k in ("chosen", "status", "nominated", "feasible", "failed", "evaluated", "next_start", "totals"):
            assert re.get(k) == ro.get(k), f"pod {i} {k}: engine {re.get(k)} oracle {ro.get(k)}"
        assert annotations(se, pods, i) == annotations(so, pods, i), f"pod {i} annotations"
        if "evaluated" in re:
            raced += len(re["evaluated"]) > len(re["feasible"]) + len(re["failed"])
        if "totals" in re:
            t = list(re["totals"].values())
            ties += t.count(max(t)) > 1
        nominated += re["nominated"] >= 0
    es, os_ = eng.node_state(), ora.node_state()
    for k in es:
        np.testing.assert_array_equal(es[k], os_[k], err_msg=k)
    np.testing.assert_array_equal(eng.class_count(), ora.class_count())
    if kind != "preempt":
        assert raced > 0, "no cycle evaluated a feasible node past the K-th"
    else:
        assert nominated > 0


def test_queued_reserve_lands_before_every_other_call():
    """The framework's Reserve of the cycle's pod is queued (ksim_assume binds
    from the pod's upload) and runs inside the next ksim_fw_prefilter's upload
    launch; any other call lands it first.  Cycles interleaved with state
    reads, next-start writes and a cluster reset keep the node state equal to
    the oracle's after every step."""
    cluster, pods = gen.config1(n_nodes=200, n_pods=120)
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=0)
    prof = profile.compile_profile(sp)
    w = profile.default_score_weights()
    eng = Engine(0)
    eng.set_profile(prof)
    eng.set_cluster(cluster.copy_state())
    ora = Oracle(cluster.copy_state(), prof)
    se, so = Store(w), Store(w)
    fe = Framework(EnginePlugins(EngineBackend(eng), cluster, sp), sp, se, seed=3)
    fo = Framework(EnginePlugins(OracleBackend(ora), cluster, sp), sp, so, seed=3)

    def same_state():
        es, os_ = eng.node_state(), ora.node_state()
        for k in es:
            np.testing.assert_array_equal(es[k], os_[k], err_msg=k)

    for i in range(pods.n_pods):
        re, ro = fe.schedule_one(pods, i, 0, None), fo.schedule_one(pods, i, 0, None)
        assert re.get("chosen") == ro.get("chosen"), i
        if i % 7 == 3:
            same_state()                        # a getter: the queued Reserve lands now
        if i % 11 == 5:
            eng.set_next_start(eng.next_start)
        if i == 60:
            same_state()
            eng.reset_cluster()                 # the queued Reserve first, then the reset
            ora = Oracle(cluster.copy_state(), prof)
            fo = Framework(EnginePlugins(OracleBackend(ora), cluster, sp), sp, so, seed=3)
            fe = Framework(EnginePlugins(EngineBackend(eng), cluster, sp), sp, se, seed=3)
            same_state()
    same_state()


def test_reserve_after_unscored_cycle_lands_before_every_call():
    """The round-5 r05b failure: a cycle with ONE feasible node is not scored
    (the framework skips prioritizeNodes), so its Reserve arrives while the
    cycle is still open and is queued (pend_bind) -- at r05b (eaa7358) into
    deferred_binds, which ksim_get_node_state read past: the last cycle's bind
    was missing from the state read after the run.  Each such Reserve is
    followed here by a different call -- every state getter, a compat cycle
    (ksim_eval_pod), a loaded-queue run (ksim_schedule_batch), a next-start
    write -- and the engine must equal the oracle after it."""
    nodes, bound, incoming = gen.config3_objects(n_nodes=240, pods_per_node=3, n_incoming=160)
    rng = np.random.default_rng(4)
    for k, p in enumerate(incoming):
        if k % 2 == 0:                              # pinned to one node: one feasible node, no Score
            p.node_selector = {"kubernetes.io/hostname": nodes[int(rng.integers(0, len(nodes)))].name}
    extra = gen.config3_objects(n_nodes=240, pods_per_node=0, n_incoming=60, seed=77)[2]
    for k, p in enumerate(extra):
        p.name = f"other-{k:04d}"
    cluster, _ = encode_cluster(nodes, bound)
    pods = encode_pods(cluster, incoming)
    others = encode_pods(cluster, extra)
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=0)
    prof = profile.compile_profile(sp)
    w = profile.default_score_weights()
    eng = Engine(0)
    eng.set_profile(prof)
    eng.set_cluster(cluster.copy_state())
    ora = Oracle(cluster.copy_state(), prof)
    fe = Framework(EnginePlugins(EngineBackend(eng), cluster, sp), sp, Store(w), seed=5)
    fo = Framework(EnginePlugins(OracleBackend(ora), cluster, sp), sp, Store(w), seed=5)
    unscored, j, b = 0, 0, 0
    for i in range(pods.n_pods):
        re, ro = fe.schedule_one(pods, i, 0, None), fo.schedule_one(pods, i, 0, None)
        assert re.get("chosen") == ro.get("chosen"), i
        if re.get("chosen", -1) < 0 or len(re.get("feasible", [])) != 1:
            continue
        unscored += 1                               # the Reserve is queued behind an unscored cycle
        what = unscored % 6
        if what == 0:
            es, os_ = eng.node_state(), ora.node_state()
            for k in es:
                np.testing.assert_array_equal(es[k], os_[k], err_msg=f"{i} {k}")
        elif what == 1:
            np.testing.assert_array_equal(eng.class_count(), ora.class_count(), err_msg=str(i))
        elif what == 2 and j < others.n_pods:
            e1, o1 = eng.eval_pod(others, j), ora.cycle(others, j)
            assert e1["chosen"] == o1["chosen"], (i, j)
            for k in ("fail_plugin", "raw", "total"):
                np.testing.assert_array_equal(e1[k], o1[k], err_msg=f"{i} {k}")
            j += 1
        elif what == 3 and b + 2 <= others.n_pods:
            sub = others.subset(others.n_pods - 2 - b, 2)
            ce, _ = eng.schedule_batch(sub)
            co, _ = ora.schedule(sub)
            np.testing.assert_array_equal(ce, co, err_msg=str(i))
            b += 2
        elif what == 4:
            np.testing.assert_array_equal(eng.nb_alloc(), ora.nb_alloc(), err_msg=str(i))
        else:
            assert eng.next_start == ora.next_start, i
            eng.set_next_start(eng.next_start)
    assert unscored > 40
    es, os_ = eng.node_state(), ora.node_state()      # the last Reserve lands before this read
    for k in es:
        np.testing.assert_array_equal(es[k], os_[k], err_msg=k)
    np.testing.assert_array_equal(eng.class_count(), ora.class_count())


def test_fw_api_lists_and_normalize():
    """ksim_fw_prefilter answers every node; ksim_fw_score over arbitrary
    feasible sublists (any order) and ksim_fw_normalize over lists that are
    not the scored list equal the oracle's."""
    nodes, bound, incoming = gen.config3_objects(n_nodes=300, pods_per_node=3, n_incoming=40)
    cluster, _ = encode_cluster(nodes, bound)
    pods = encode_pods(cluster, incoming)
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=0)
    prof = profile.compile_profile(sp)
    eng = Engine(0)
    eng.set_profile(prof)
    eng.set_cluster(cluster)
    ora = Oracle(cluster, prof)
    rng = np.random.default_rng(5)
    S = prof.n_score
    for i in range(pods.n_pods):
        fe, fo = eng.fw_prefilter(pods, i), ora.fw_prefilter(pods, i)
        np.testing.assert_array_equal(fe["fail_plugin"], fo["fail_plugin"])
        np.testing.assert_array_equal(fe["fail_detail"], fo["fail_detail"])
        assert fe["n_feasible"] == fo["n_feasible"] and fe["k_to_find"] == fo["k_to_find"]
        assert not (fe["fail_plugin"] == abi.NOT_EVALUATED).any()
        feas = np.nonzero(fe["fail_plugin"] == abi.PASSED)[0]
        if feas.size < 2:
            continue
        lst = rng.permutation(feas)[:int(rng.integers(2, feas.size + 1))]
        se, so = eng.fw_score(lst), ora.fw_score(lst)
        for k in ("raw", "norm", "total", "scored"):
            np.testing.assert_array_equal(se[k], so[k], err_msg=f"pod {i} {k}")
        for slot in range(S):
            sub = rng.permutation(lst)[:int(rng.integers(1, lst.size + 1))]
            vals = rng.integers(-5, 300, sub.size)
            np.testing.assert_array_equal(eng.fw_normalize(slot, sub, vals), ora.fw_normalize(slot, sub, vals),
                                          err_msg=f"pod {i} slot {slot}")
            # the scored list with its raw scores (answered from fw_score's
            # normalization), then with one score changed (the device path)
            raw = se["raw"][slot][lst]
            np.testing.assert_array_equal(eng.fw_normalize(slot, lst, raw), se["norm"][slot][lst])
            np.testing.assert_array_equal(eng.fw_normalize(slot, lst, raw), ora.fw_normalize(slot, lst, raw))
            bent = raw.copy()
            bent[-1] += 7
            np.testing.assert_array_equal(eng.fw_normalize(slot, lst, bent), ora.fw_normalize(slot, lst, bent),
                                          err_msg=f"pod {i} slot {slot} bent")
        node = int(lst[0])
        eng.assume(pods, i, node)
        ora.assume(pods, i, node)
    es, os_ = eng.node_state(), ora.node_state()
    for k in es:
        np.testing.assert_array_equal(es[k], os_[k])


def test_fw_staging_grows_with_the_cluster():
    """The pinned staging of the framework-driven calls grows past its first
    allocation (20,000 nodes: the score call's list mask alone exceeds it):
    the results' staging must survive the upload staging's reallocation, and
    every answer still equals the oracle's."""
    cluster, pods = gen.config2(n_nodes=20000, n_pods=40, seed=3)
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=0)
    prof = profile.compile_profile(sp)
    eng = Engine(0)
    eng.set_profile(prof)
    eng.set_cluster(cluster)
    ora = Oracle(cluster, prof)
    rng = np.random.default_rng(11)
    for i in range(pods.n_pods):
        fe, fo = eng.fw_prefilter(pods, i), ora.fw_prefilter(pods, i)
        np.testing.assert_array_equal(fe["fail_plugin"], fo["fail_plugin"])
        feas = np.nonzero(fe["fail_plugin"] == abi.PASSED)[0]
        lst = rng.permutation(feas)[:int(rng.integers(2, feas.size + 1))] if feas.size > 1 else feas
        if lst.size < 2:
            continue
        se, so = eng.fw_score(lst), ora.fw_score(lst)
        for k in ("raw", "norm", "total", "scored"):
            np.testing.assert_array_equal(se[k], so[k], err_msg=f"pod {i} {k}")
        for slot in range(prof.n_score):
            vals = rng.integers(-5, 300, lst.size)
            np.testing.assert_array_equal(eng.fw_normalize(slot, lst, vals), ora.fw_normalize(slot, lst, vals))
        node = int(lst[0])
        eng.assume(pods, i, node)
        ora.assume(pods, i, node)
    es, os_ = eng.node_state(), ora.node_state()
    for k in es:
        np.testing.assert_array_equal(es[k], os_[k])


def test_fw_rejects_bad_lists_and_abandons_cleanly():
    """A list with an infeasible or repeated node is refused; a framework
    cycle left without PreScore (one feasible node) does not leak its
    PreFilter domain sums into the next deterministic cycle."""
    nodes, bound, incoming = gen.config3_objects(n_nodes=200, pods_per_node=3, n_incoming=30)
    cluster, _ = encode_cluster(nodes, bound)
    pods = encode_pods(cluster, incoming)
    prof = profile.compile_profile(profile.SchedulerProfile(percentage_of_nodes_to_score=0))
    eng = Engine(0)
    eng.set_profile(prof)
    eng.set_cluster(cluster)
    ora = Oracle(cluster, prof)
    f = eng.fw_prefilter(pods, 0)
    bad = np.nonzero(f["fail_plugin"] != abi.PASSED)[0]
    good = np.nonzero(f["fail_plugin"] == abi.PASSED)[0]
    from ksim.engine import KsimError
    if bad.size:
        with pytest.raises(KsimError):
            eng.fw_score([int(good[0]), int(bad[0])])
    with pytest.raises(KsimError):
        eng.fw_score([int(good[0]), int(good[0])])
    # abandoned framework cycles, then deterministic cycles: equal to the oracle's
    for i in range(1, 10):
        eng.fw_prefilter(pods, i)
    ora.set_pod_seq(0)
    for i in range(10, pods.n_pods):
        e, o = eng.eval_pod(pods, i), ora.cycle(pods, i)
        assert e["chosen"] == o["chosen"], i
        np.testing.assert_array_equal(e["norm"], o["norm"])


def test_compat_cycle_postfilter_nominated():
    """Deterministic compat cycles with DefaultPreemption's PostFilter: the
    engine's nominated node (ksim_preempt) and the recorded annotations equal
    the oracle's."""
    from ksim.wrapped import compat_cycle
    cluster, pods, table, prio = _cases("preempt")
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=0)
    prof = profile.compile_profile(sp)
    w = profile.default_score_weights()
    eng = Engine(0)
    eng.set_profile(prof)
    eng.set_cluster(cluster.copy_state())
    eng.set_bound_pods(table)
    ora = Oracle(cluster.copy_state(), prof)
    se, so = Store(w), Store(w)
    nominated = 0
    for i in range(pods.n_pods):
        re = compat_cycle(eng, se, cluster, sp, pods, i, prio[i])
        ro = compat_cycle(ora, so, cluster, sp, pods, i, prio[i], table)
        assert re["chosen"] == ro["chosen"] and re["nominated"] == ro["nominated"], i
        assert annotations(se, pods, i) == annotations(so, pods, i), i
        nominated += re["nominated"] >= 0
    assert nominated > 0


def _nominated_run(fe, fo, pods, prio, table_for, steps, where):
    """One schedule_one per step on both mirrors; the outcomes, annotations and
    nominators must agree.  ``table_for(step)`` returns the bound-pod table."""
    stats = {"nominated": 0, "two_pass": 0, "nominated_eval": 0, "ineligible": 0}
    for step, i in enumerate(steps):
        table = table_for(step)
        re = fe.schedule_one(pods, i, prio[i], table)
        ro = fo.schedule_one(pods, i, prio[i], table)
        for k in ("chosen", "status", "nominated", "feasible", "failed", "evaluated", "next_start", "totals",
                  "victims", "eligible", "nominated_eval"):
            assert re.get(k) == ro.get(k), f"{where} step {step} pod {i} {k}: engine {re.get(k)} oracle {ro.get(k)}"
        assert annotations(fe.store, pods, i) == annotations(fo.store, pods, i), f"{where} pod {i} annotations"
        assert fe.nominator == fo.nominator and fe.terminating == fo.terminating, f"{where} step {step}"
        stats["nominated"] += re["nominated"] >= 0
        stats["ineligible"] += re.get("eligible") is False
        stats["nominated_eval"] += "nominated_eval" in re
        stats["two_pass"] += any(fe.pl.has_nominated(x) for x in re.get("evaluated", []))
    return stats


@pytest.mark.parametrize("seed", [1, 2])
def test_framework_nominated_preemption_chains(seed):
    """The racing mirror with the PodNominator over the engine and over the
    oracle: preemptors nominated (ksim_preempt_nominated keeps the nominated
    pods of priority >= the preemptor on each candidate), victims Terminating,
    the nominated pods re-queued (evaluateNominatedNode, then refused while
    their victims terminate), every other pod filtered with its two passes
    (ksim_fw_filter_nominated).  The bound-pod table grows with each bind."""
    import dataclasses
    from test_preemption import crowded
    nodes, bound, start, _ = crowded(n_nodes=400, seed=seed + 20)
    cluster, _ = encode_cluster(nodes, bound)
    rng = np.random.default_rng(seed)
    pods_o = [Pod(f"p{i}", priority=int(rng.choice([0, 5, 50, 500, 5000])),
                  containers=[Container({"cpu": f"{int(rng.integers(5, 300)) * 100}m",
                                         "memory": f"{int(rng.integers(2, 30))}Gi"})]) for i in range(160)]
    pods = encode_pods(cluster, pods_o)
    prio = [p.priority for p in pods_o]
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=0)
    prof = profile.compile_profile(sp)
    eng = Engine(0)
    eng.set_profile(prof)
    eng.set_cluster(cluster.copy_state())
    ora = Oracle(cluster.copy_state(), prof)
    w = profile.default_score_weights()
    fe = Framework(EnginePlugins(EngineBackend(eng), cluster, sp), sp, Store(w), seed=seed)
    fo = Framework(EnginePlugins(OracleBackend(ora), cluster, sp), sp, Store(w), seed=seed)
    placed = list(bound)
    tables = [bound_table(cluster, placed, start)]
    retries = []
    # the queue, step by step so the table grows with each bind; preemptors
    # come back three pods later
    stats = {"nominated": 0, "two_pass": 0, "nominated_eval": 0, "ineligible": 0}
    queue, step = list(range(len(pods_o))), 0
    while queue and step < 400:
        i = queue.pop(0)
        s = _nominated_run(fe, fo, pods, prio, lambda _: tables[-1], [i], f"seed {seed}")
        for k in stats:
            stats[k] += s[k]
        last = fe.log[-1]
        if last["status"] == abi.STATUS_SCHEDULED:
            placed.append(dataclasses.replace(pods_o[i], node_name=cluster.node_names[last["chosen"]]))
            start[pods_o[i].name] = 100 + step
            tables.append(bound_table(cluster, placed, start))
        elif last["nominated"] >= 0:
            retries.append(i)
        if len(retries) >= 3 or (not queue and retries):
            queue.extend(retries)
            retries = []
        step += 1
    es, os_ = eng.node_state(), ora.node_state()
    for k in es:
        np.testing.assert_array_equal(es[k], os_[k], err_msg=k)
    assert stats["nominated"] > 5 and stats["two_pass"] > 5 and stats["nominated_eval"] > 5, stats


def test_framework_seeded_nominations_topology():
    """Nominations seeded on spreading / anti-affine config-3 pods: the first
    pass's PodTopologySpread / InterPodAffinity state carries the nominated
    pods (assume, re-run, forget on the device), then the seeded pods try
    their nominated node first."""
    nodes, bound, incoming = gen.config3_objects(n_nodes=500, pods_per_node=4, n_incoming=400)
    cluster, _ = encode_cluster(nodes, bound)
    pods = encode_pods(cluster, incoming)
    prio = [p.priority for p in incoming]
    sp = profile.SchedulerProfile(percentage_of_nodes_to_score=0)
    prof = profile.compile_profile(sp)
    eng = Engine(0)
    eng.set_profile(prof)
    eng.set_cluster(cluster.copy_state())
    ora = Oracle(cluster.copy_state(), prof)
    w = profile.default_score_weights()
    fe = Framework(EnginePlugins(EngineBackend(eng), cluster, sp), sp, Store(w), seed=3)
    fo = Framework(EnginePlugins(OracleBackend(ora), cluster, sp), sp, Store(w), seed=3)
    rng = np.random.default_rng(9)
    seeded = list(range(60))
    for j in seeded:
        node = int(rng.integers(0, 40)) * 3
        fe.nominate(j, node, prio[j])
        fo.nominate(j, node, prio[j])
    stats = _nominated_run(fe, fo, pods, prio, lambda _: None, list(range(60, len(incoming))) + seeded, "config3")
    es, os_ = eng.node_state(), ora.node_state()
    for k in es:
        np.testing.assert_array_equal(es[k], os_[k], err_msg=k)
    np.testing.assert_array_equal(eng.class_count(), ora.class_count())
    assert stats["two_pass"] > 50 and stats["nominated_eval"] > 10, stats


def test_forget_during_framework_cycle():
    """Unreserve from the binding goroutine while the next cycle sits between
    PreFilter and Score: the engine queues the ksim_forget, the
    cycle's Score still sees the snapshot it started from, and the forget
    lands once the cycle has scored.  The oracle runs the same calls with the
    forget after the cycle's Reserve; every answer and the final node state,
    class counts included, must agree."""
    nodes, bound, incoming = gen.config3_objects(n_nodes=300, pods_per_node=3, n_incoming=120)
    cluster, _ = encode_cluster(nodes, bound)
    pods = encode_pods(cluster, incoming)
    prof = profile.compile_profile(profile.SchedulerProfile(percentage_of_nodes_to_score=0))
    eng = Engine(0)
    eng.set_profile(prof)
    eng.set_cluster(cluster.copy_state())
    ora = Oracle(cluster.copy_state(), prof)
    placed = []
    for i in range(pods.n_pods):
        e, o = eng.fw_prefilter(pods, i), ora.fw_prefilter(pods, i)
        np.testing.assert_array_equal(e["fail_plugin"], o["fail_plugin"], err_msg=f"prefilter {i}")
        forget = placed.pop(0) if (i % 3 == 2 and placed) else None
        if forget is not None:                 # engine: inside the cycle; oracle: after it
            eng.forget(pods, *forget)
        feas = np.flatnonzero(e["fail_plugin"] == abi.PASSED).astype(np.int32)
        if feas.size == 0:
            continue
        es, os_ = eng.fw_score(feas), ora.fw_score(feas)
        for k in ("raw", "norm", "total"):
            np.testing.assert_array_equal(es[k][..., feas], os_[k][..., feas], err_msg=f"score {k} {i}")
        node = int(feas[np.argmax(es["total"][feas])])
        eng.assume(pods, i, node)
        ora.assume(pods, i, node)
        if forget is not None:
            ora.forget(pods, *forget)
        placed.append((i, node))
    es, os_ = eng.node_state(), ora.node_state()
    for k in es:
        np.testing.assert_array_equal(es[k], os_[k], err_msg=k)
    np.testing.assert_array_equal(eng.class_count(), ora.class_count())
